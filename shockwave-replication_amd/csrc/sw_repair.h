/*
 * sw_repair.h — width-profile repair of a density-order placement that left
 * rounds unplaced.  Plain C99 + HIP qualifiers; shared by
 * the plan kernel (sw_kernels.hip, run by one thread), the sharded
 * controller (sw_shard_ctl.h, on the host) and the CPU twin.
 *
 * The reference's P2 (shockwave.py:281-328) is a MILP over the per-round
 * placement of fixed counts n_j with widths w_j.  The density order
 * p_j/(n_j·w_j) places rounds the way the MILP's LP relaxation would, but
 * with widths {1, 2, 4, 8} it can strand a wide job: the last rounds keep a
 * few free GPUs each, none with room for it.  The repair keeps the density
 * placement's per-width-class profile — how many jobs of each width run in
 * each round — and changes it only as much as the stranded rounds need:
 *
 *   for each class c, widest first, and each of its D_c unplaced rounds:
 *     ts = the round with the most free GPUs (ties: the latest) that still
 *          has a class-c job not running in it;
 *     while ts lacks w_c free GPUs: move one unit of a narrower class c2
 *          (narrowest first) from ts to the earliest other round with room
 *          for it and a class-c2 job not yet running there;
 *     give class c one more unit in ts.
 *
 * Each changed class is then repacked alone with unit widths inside its new
 * per-round capacities (the class-wise packer: exact for unit widths when
 * the profile admits the counts); unchanged classes keep their density rows.
 * On the simulator's P2 cases this lands within 1.04x of the P2 MILP where
 * the class-wise repack inside the P1 profile was up to 1.37x (tests/test_p2.py).
 */
#ifndef SW_REPAIR_H
#define SW_REPAIR_H

#include <stdint.h>

#include "sw_arith.h"

#define SW_RCLS_MAX 8 /* width classes the repair handles (traces: 4) */

typedef struct {
    int32_t ncls;                       /* classes present, ascending width     */
    int32_t wc[SW_RCLS_MAX];            /* class width                          */
    int32_t M[SW_RCLS_MAX];             /* jobs of the class with rounds        */
    int32_t D[SW_RCLS_MAX];             /* rounds of the class left unplaced    */
    int32_t changed[SW_RCLS_MAX];       /* profile changed: repack the class    */
    int32_t caps[SW_RCLS_MAX][SW_TMAX]; /* class jobs placed in round t         */
    int32_t L[SW_TMAX];                 /* free GPUs in round t                 */
} sw_repair_t;

/* Class index of width w (-1 if w is not a class). */
SW_HD int32_t sw_repair_class(const sw_repair_t* r, int32_t w) {
    for (int32_t c = 0; c < r->ncls; ++c)
        if (r->wc[c] == w) return c;
    return -1;
}

/* Inserts width w into the ascending class list; -1 when the list is full. */
SW_HD int32_t sw_repair_add_class(sw_repair_t* r, int32_t w) {
    int32_t c = sw_repair_class(r, w);
    if (c >= 0) return c;
    if (r->ncls >= SW_RCLS_MAX) return -1;
    int32_t i = r->ncls++;
    while (i > 0 && r->wc[i - 1] > w) {
        r->wc[i] = r->wc[i - 1];
        --i;
    }
    r->wc[i] = w;
    return i;
}

/* The repair itself on the filled-in profile; 0 on success, -1 when some
 * unplaced round finds no round to go to. */
SW_HD int32_t sw_profile_repair(sw_repair_t* r, int32_t T) {
    for (int32_t ci = r->ncls - 1; ci >= 0; --ci) {
        const int32_t c = r->wc[ci];
        for (int32_t d = 0; d < r->D[ci]; ++d) {
            int32_t ts = -1;
            for (int32_t t = 0; t < T; ++t)
                if (r->caps[ci][t] < r->M[ci] && (ts < 0 || r->L[t] >= r->L[ts])) ts = t;
            if (ts < 0) return -1;
            int32_t need = c - r->L[ts];
            for (int32_t c2 = 0; c2 < ci && need > 0; ++c2) {
                const int32_t w2 = r->wc[c2];
                while (need > 0 && r->caps[c2][ts] > 0) {
                    int32_t t2 = -1;
                    for (int32_t t = 0; t < T && t2 < 0; ++t)
                        if (t != ts && r->L[t] >= w2 && r->caps[c2][t] < r->M[c2]) t2 = t;
                    if (t2 < 0) break;
                    r->caps[c2][ts] -= 1;
                    r->L[ts] += w2;
                    r->caps[c2][t2] += 1;
                    r->L[t2] -= w2;
                    r->changed[c2] = 1;
                    need -= w2;
                }
            }
            if (r->L[ts] < c) return -1;
            r->caps[ci][ts] += 1;
            r->L[ts] -= c;
            r->changed[ci] = 1;
        }
    }
    return 0;
}

/*
 * Pattern search: an exact width-class profile for counts the orders and the
 * repair could not place.
 *
 * In P1 every round has capacity G and the objective sees only n_j, so rounds
 * are interchangeable: a P1 placement is a multiset of T round PATTERNS, a
 * pattern s giving the number of slots of each width class (Σ_c w_c·s_c ≤ G).
 * A class's counts fit its slots iff Gale–Ryser holds: with D_c(k) = the sum
 * of the class's k largest counts and S_c(k) = Σ_t min(s_ct, k),
 * S_c(k) ≥ D_c(k) for every k (each job at most once per round); the
 * class-wise packer (unit widths, the tier rule) then places them.  The
 * search is a depth-first walk over the rounds, each round's pattern no
 * larger (lexicographically, widest class first) than the previous one's —
 * every multiset once — over MAXIMAL patterns only (a pattern that could take
 * one more slot of a class with jobs left is dominated), pruned by
 *   S_c(k) + R·min(cap_c, k) ≥ D_c(k)  and  Σ_c w_c·max_k(D_c(k) − S_c(k)) ≤ R·G
 * with R rounds left and cap_c = min(M_c, ⌊G/w_c⌋).  It is exact up to a work
 * budget of SW_PAT_STEPS (each node costs 1 + Σ_c M_c steps, the size of its
 * Gale–Ryser check, and each pattern candidate ncls): found ⇒ a profile that
 * places every count.  The budget bounds the one-thread search on the GPU to
 * a few milliseconds in the worst case; it only runs for counts no order
 * placed.
 *
 * r: ncls, wc[], M[] filled by the caller; on success r->caps[c][t] holds the
 * profile and every class is marked changed.  hist: ncls × (T + 1) ints,
 * hist[c·(T+1) + v] = #{jobs of class c with n_j = v}.  scratch: SW_PAT_SCRATCH(A)
 * ints, A = the jobs with rounds (per-class caps and offsets, then the prefix
 * arrays Σ_c (M_c + 1) + Σ_c (cap_c + 1) ≤ 2·A + 2·SW_RCLS_MAX).
 * Returns 1 when found, 0 when not (infeasible, or the node cap).
 */
#define SW_PAT_STEPS (1 << 18)
#define SW_PAT_SCRATCH(A) (2 * (A) + 5 * SW_RCLS_MAX)

SW_HD void sw_pat_first(sw_repair_t* r, const int32_t* cap, int32_t G, int32_t t) {
    int64_t rem = G;
    for (int32_t c = r->ncls - 1; c >= 0; --c) {
        int64_t v = rem / r->wc[c];
        v = v < cap[c] ? v : cap[c];
        r->caps[c][t] = (int32_t)v;
        rem -= v * r->wc[c];
    }
}

/* the next maximal pattern below round t's in descending lexicographic order
 * (class ncls−1 most significant; class 0 always filled); 0 when none */
SW_HD int32_t sw_pat_next(sw_repair_t* r, const int32_t* cap, int32_t G, int32_t t,
                          int64_t* steps) {
    const int32_t K = r->ncls;
    while (1) {
        *steps += K; /* the budget counts every candidate, maximal or not */
        if (*steps > SW_PAT_STEPS) return 0;
        int32_t c = 1;
        while (c < K && r->caps[c][t] == 0) ++c;
        if (c >= K) return 0;
        r->caps[c][t] -= 1;
        int64_t rem = G;
        for (int32_t x = K - 1; x >= c; --x) rem -= (int64_t)r->wc[x] * r->caps[x][t];
        for (int32_t x = c - 1; x >= 0; --x) {
            int64_t v = rem / r->wc[x];
            v = v < cap[x] ? v : cap[x];
            r->caps[x][t] = (int32_t)v;
            rem -= v * r->wc[x];
        }
        int32_t maximal = 1;
        for (int32_t x = 0; x < K; ++x)
            if (r->caps[x][t] < cap[x] && (int64_t)r->wc[x] <= rem) maximal = 0;
        if (maximal) return 1;
    }
}

SW_HD int32_t sw_profile_search(sw_repair_t* r, int32_t T, int32_t G, const int32_t* hist,
                                int32_t* scratch, int64_t* nodes_out) {
    const int32_t K = r->ncls;
    /* per-class caps and offsets live in the scratch too (on the GPU one
     * thread runs this: no private arrays, so no scratch-memory frame) */
    int32_t* cap = scratch;
    int32_t* doff = scratch + SW_RCLS_MAX;
    int32_t* hoff = scratch + 2 * SW_RCLS_MAX;
    int64_t nodes = 0, steps = 0, per = 1;
    if (K <= 0 || K > SW_RCLS_MAX || T <= 0) return 0;
    int32_t o = 3 * SW_RCLS_MAX;
    for (int32_t c = 0; c < K; ++c) {
        const int32_t g = G / r->wc[c];
        cap[c] = r->M[c] < g ? r->M[c] : g;
        doff[c] = o;
        o += r->M[c] + 1;
        per += r->M[c];
    }
    for (int32_t c = 0; c < K; ++c) {
        hoff[c] = o;
        o += cap[c] + 1;
    }
    /* D_c(k): the class's demands in descending order, summed */
    for (int32_t c = 0; c < K; ++c) {
        int32_t* D = scratch + doff[c];
        int32_t k = 0;
        D[0] = 0;
        for (int32_t v = T; v >= 1; --v)
            for (int32_t i = 0; i < hist[c * (T + 1) + v] && k < r->M[c]; ++i, ++k) D[k + 1] = D[k] + v;
        for (; k < r->M[c]; ++k) D[k + 1] = D[k];
        int32_t* h = scratch + hoff[c];
        for (int32_t m = 0; m <= cap[c]; ++m) h[m] = 0;
    }
    int32_t t = 0, found = 0;
    sw_pat_first(r, cap, G, 0);
    while (1) {
        /* try round t's pattern */
        ++nodes;
        steps += per;
        if (steps > SW_PAT_STEPS) break;
        for (int32_t c = 0; c < K; ++c) {
            int32_t* h = scratch + hoff[c];
            for (int32_t m = 1; m <= r->caps[c][t]; ++m) h[m] += 1;
        }
        const int64_t R = T - 1 - t;
        int32_t ok = 1;
        int64_t needload = 0;
        for (int32_t c = 0; c < K && ok; ++c) {
            const int32_t* D = scratch + doff[c];
            const int32_t* h = scratch + hoff[c];
            int64_t Sk = 0, need = 0;
            for (int32_t k = 1; k <= r->M[c]; ++k) {
                if (k <= cap[c]) Sk += h[k];
                const int64_t fut = R * (int64_t)(k < cap[c] ? k : cap[c]);
                if (Sk + fut < D[k]) { ok = 0; break; }
                if (D[k] - Sk > need) need = D[k] - Sk;
            }
            needload += (int64_t)r->wc[c] * need;
        }
        if (ok && needload <= R * (int64_t)G) {
            if (t == T - 1) { found = 1; break; }
            for (int32_t c = 0; c < K; ++c) r->caps[c][t + 1] = r->caps[c][t];
            ++t;
            continue;
        }
        /* undo round t, advance it; exhausted rounds hand back to their parent */
        int32_t done = 0;
        while (1) {
            for (int32_t c = 0; c < K; ++c) {
                int32_t* h = scratch + hoff[c];
                for (int32_t m = 1; m <= r->caps[c][t]; ++m) h[m] -= 1;
            }
            if (sw_pat_next(r, cap, G, t, &steps)) break;
            if (t == 0 || steps > SW_PAT_STEPS) { done = 1; break; }
            --t;
        }
        if (done) break;
    }
    if (nodes_out) *nodes_out = nodes;
    if (!found) return 0;
    for (int32_t c = 0; c < K; ++c) r->changed[c] = 1;
    return 1;
}

#endif /* SW_REPAIR_H */
