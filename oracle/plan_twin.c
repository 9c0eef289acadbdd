/*
 * oracle/plan_twin.c — TEST INFRASTRUCTURE, NOT PRODUCT CODE.
 *
 * Sequential CPU restatement of the deterministic plan algorithm that the HIP
 * kernel in shockwave-replication_amd/csrc/sw_kernels.hip implements
 * (DESIGN.md §3).  Its job is to be the bit-exact checker the north star asks
 * for ("the rounding of the relaxed plan into a per-round job→worker
 * schedule, deterministic and bit-exact vs a CPU reimplementation").  It is
 * NOT the restatement of the reference solver — that is oracle/milp_ref.py
 * (HiGHS MILP of shockwave.py:330-388 / :281-328) — and it is never linked
 * into, loaded by, or used as a fallback for the product path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Reference semantics it follows (through the per-job reduction in
 * sw_arith.h): P1 = shockwave.py:330-388, P2 = shockwave.py:281-328,
 * schedule read-back = shockwave.py:390-398.
 *
 * Bit-exactness contract with the GPU:
 *   - per-job arithmetic is the shared sw_arith.h, -ffp-contract=off on both;
 *   - every float sum over jobs is sw_detsum (1024 contiguous chunks summed
 *     left to right, then a halving tree) — the GPU plan kernel runs exactly
 *     1024 threads per instance and reduces in the same order;
 *   - integer sums, maxima and lexicographic arg-max are order independent.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/shockwave_amd.h"
#include "../shockwave-replication_amd/csrc/sw_arith.h"
#include "../shockwave-replication_amd/csrc/sw_bnb.h"
#include "../shockwave-replication_amd/csrc/sw_repair.h"
#include "../shockwave-replication_amd/csrc/sw_reround.h"
#include "../shockwave-replication_amd/csrc/sw_validate.h"

typedef struct {
    int32_t N, T, G, nb;
    int64_t C;
    double k, A;
    const double* beta;
    const double* ell;
    double slope[SW_BMAX];
    sw_jobc* jc;
    int32_t* Tj; /* rounds job j may use: T, or 0 if w_j > G (shockwave.py:64-75) */
    float* key;  /* [N][T] */
    int64_t passes;
} twin_t;

#define K_(P, j, n) ((P)->key[(size_t)(j) * (P)->T + (n)])

/* Deterministic sum: SW_DET_LANES contiguous chunks summed
 * left to right; then, per wave of 64 lanes, a halving tree p[i] += p[i+h]
 * (h = 32 … 1); then the SW_DET_LANES/64 wave sums by the same halving tree.
 * The GPU does exactly this with wave shuffles and one LDS exchange. */
static double sw_detsum(const double* v, int32_t N) {
    double part[SW_DET_LANES];
    double wsum[SW_DET_LANES / 64];
    int32_t q = (N + SW_DET_LANES - 1) / SW_DET_LANES;
    for (int32_t lane = 0; lane < SW_DET_LANES; ++lane) {
        double s = 0.0;
        int32_t lo = lane * q, hi = lo + q < N ? lo + q : N;
        for (int32_t j = lo; j < hi; ++j) s = s + v[j];
        part[lane] = s;
    }
    for (int32_t w = 0; w < SW_DET_LANES / 64; ++w) {
        double* p = part + 64 * w;
        for (int32_t h = 32; h >= 1; h >>= 1)
            for (int32_t i = 0; i < h; ++i) p[i] = p[i] + p[i + h];
        wsum[w] = p[0];
    }
    for (int32_t h = SW_DET_LANES / 128; h >= 1; h >>= 1)
        for (int32_t i = 0; i < h; ++i) wsum[i] = wsum[i] + wsum[i + h];
    return wsum[0];
}

double twin_detsum(const double* v, int32_t N) { return sw_detsum(v, N); }

int32_t twin_p2x_plan(int32_t N, int32_t T, int32_t G, const int32_t* w, const double* prio,
                      const int32_t* n, uint8_t* y); /* p2x_twin.c */

static double fval(const twin_t* P, int32_t j, int32_t n) {
    return sw_f(&P->jc[j], n, P->nb, P->beta, P->ell, P->slope);
}

static int32_t lforce(const twin_t* P, int32_t j, double M) {
    int32_t c = 0;
    for (int32_t n = 0; n < P->Tj[j]; ++n) c += (sw_g(&P->jc[j], n) > M);
    return c;
}

static int32_t cnt_gt(const twin_t* P, int32_t j, uint32_t rho, int32_t l) {
    int32_t c = 0;
    for (int32_t n = l; n < P->Tj[j]; ++n) c += (sw_fbits_of(K_(P, j, n)) > rho);
    return c;
}

static int32_t cnt_ge(const twin_t* P, int32_t j, uint32_t rho, int32_t l) {
    int32_t c = 0;
    for (int32_t n = l; n < P->Tj[j]; ++n) c += (sw_fbits_of(K_(P, j, n)) >= rho);
    return c;
}

typedef struct {
    double U, Mact, J, ubound;
    uint32_t rho; /* price ρ* bits (0 when every item fits) */
} sel_eval_t;

/*
 * SELECT(M): forced prefix l_j = #{n<T : g_j(n) > M}, then the greedy over
 * the remaining increments in key order (key desc, j asc, n asc) with budget
 * C − Σ w l, computed as a price threshold ρ* (bisection over fp32 key bits),
 * the job-ordered tie group at ρ*, and a ≤7-unit width tail.  is_inf: M = +∞.
 */
/* [plo, phi]: a bracket of ρ*(M) from already evaluated levels — ρ* is
 * non-increasing in M (a larger level frees forced rounds, and the budget
 * grows by exactly their weight), so ρ*(M') ≤ ρ*(M) ≤ ρ*(M'') for
 * M'' < M < M'.  The bisection returns the same ρ* from any valid bracket. */
static int select_level(twin_t* P, double M, int is_inf, int32_t* n, int32_t* l,
                        int32_t* taken, double* tmp, sel_eval_t* ev, uint32_t plo,
                        uint32_t phi) {
    const int32_t N = P->N;
    int64_t Wf = 0, Wall = 0;
    for (int32_t j = 0; j < N; ++j) {
        l[j] = is_inf ? 0 : lforce(P, j, M);
        Wf += (int64_t)P->jc[j].w * l[j];
        Wall += (int64_t)P->jc[j].w * (P->Tj[j] - l[j]);
    }
    P->passes++;
    if (Wf > P->C) return -1;
    int64_t bud = P->C - Wf;
    double rho_d = 0.0;
    int64_t wgt_star = 0;
    ev->rho = 0;
    if (Wall <= bud) {
        for (int32_t j = 0; j < N; ++j) { n[j] = P->Tj[j]; taken[j] = P->Tj[j] - l[j]; }
        wgt_star = Wall;
    } else {
        /* Bisection snapped to key values.  A job's count is a function of
         * its raw count #{n < Tj : key > ρ}, which only changes at its key
         * values; so with mx = the largest key ≤ mid and mn = the smallest
         * key > mid over the jobs whose count still varies on [lo, hi]
         * ("open": cnt_ge(lo) ≠ cnt_gt(hi)), W is constant on [mx, mid] and
         * on [mid, mn).  A probe below budget moves hi to max(lo, mx), one
         * above it moves lo to min(hi, mn): same ρ* as the plain bisection,
         * fewer probes. */
        uint32_t lo = plo, hi = phi;
        /* Probes: the midpoint until both ends carry a measured W, then the
         * point where the line through (lo, W just below lo) and (hi, W(hi))
         * crosses the budget (interpolation over the key bits; integer
         * arithmetic).  Any probe inside the bracket keeps it valid, so ρ*
         * is the same; on C3 instances this takes a third fewer probes. */
        int64_t Wb = -1, Wh = -1;
        while (lo < hi) {
            uint32_t mid = lo + ((hi - lo) >> 1);
            if (Wb >= 0 && Wh >= 0) {
                mid = lo + (uint32_t)(((uint64_t)(hi - lo) * (uint64_t)(Wb - bud)) /
                                      (uint64_t)(Wb - Wh));
                if (mid >= hi) mid = hi - 1;
            }
            int64_t wg = 0;
            uint32_t mx = 0, mn = 0x7FFFFFFFu;
            for (int32_t j = 0; j < N; ++j) {
                wg += (int64_t)P->jc[j].w * cnt_gt(P, j, mid, l[j]);
                if (cnt_ge(P, j, lo, l[j]) == cnt_gt(P, j, hi, l[j])) continue;
                for (int32_t q = 0; q < P->Tj[j]; ++q) {
                    const uint32_t b = sw_fbits_of(K_(P, j, q));
                    if (b > mid) mn = b < mn ? b : mn;
                    else mx = b > mx ? b : mx;
                }
            }
            P->passes++;
            if (wg <= bud) { hi = mx > lo ? mx : lo; Wh = wg; }
            else { lo = mn < hi ? mn : hi; Wb = wg; }
        }
        uint32_t rho = lo;
        ev->rho = rho;
        rho_d = (double)sw_float_of(rho);
        int64_t wt = 0;
        for (int32_t j = 0; j < N; ++j) {
            taken[j] = cnt_gt(P, j, rho, l[j]);
            wt += (int64_t)P->jc[j].w * taken[j];
        }
        wgt_star = wt;
        int64_t rem = bud - wt;
        /* tie group (key == ρ*) taken in job order */
        int64_t excl = 0, used = 0;
        for (int32_t j = 0; j < N; ++j) {
            int32_t tie = cnt_ge(P, j, rho, l[j]) - taken[j];
            int64_t wj = P->jc[j].w;
            int32_t tt;
            if (excl + wj * tie <= rem) tt = tie;
            else if (excl <= rem) tt = (int32_t)((rem - excl) / wj);
            else tt = 0;
            n[j] = l[j] + taken[j] + tt;
            used += wj * tt;
            excl += wj * tie;
        }
        P->passes++;
        int64_t rem2 = rem - used;
        /* width tail: next item in key order among jobs that still fit */
        while (rem2 > 0) {
            int32_t best = -1;
            uint32_t bk = 0;
            for (int32_t j = 0; j < N; ++j) {
                if (n[j] < P->Tj[j] && (int64_t)P->jc[j].w <= rem2) {
                    uint32_t kb = sw_fbits_of(K_(P, j, n[j]));
                    if (best < 0 || kb > bk) { best = j; bk = kb; }
                }
            }
            P->passes++;
            if (best < 0) break;
            n[best] += 1;
            rem2 -= P->jc[best].w;
        }
    }
    double Mact = 0.0;
    for (int32_t j = 0; j < N; ++j) {
        tmp[j] = fval(P, j, n[j]);
        double gj = sw_g(&P->jc[j], n[j]);
        Mact = gj > Mact ? gj : Mact;
    }
    ev->U = sw_detsum(tmp, N);
    ev->Mact = Mact;
    ev->J = ev->U - P->k * Mact;
    /* Lagrangian bound of the concave relaxation at price ρ*·A */
    for (int32_t j = 0; j < N; ++j) tmp[j] = fval(P, j, l[j] + taken[j]);
    ev->ubound = sw_detsum(tmp, N) + (rho_d * P->A) * (double)(bud - wgt_star);
    P->passes++;
    return 0;
}

static int feasible_level(twin_t* P, double M) {
    int64_t Wf = 0;
    for (int32_t j = 0; j < P->N; ++j) Wf += (int64_t)P->jc[j].w * lforce(P, j, M);
    P->passes++;
    return Wf <= P->C;
}

static int64_t levels_between(twin_t* P, double a, double b) {
    int64_t c = 0;
    for (int32_t j = 0; j < P->N; ++j)
        for (int32_t n = 0; n <= P->Tj[j]; ++n) {
            double v = sw_g(&P->jc[j], n);
            c += (v > a && v < b);
        }
    P->passes++;
    return c;
}

/* ---- placement (P1 packing and P2): DESIGN.md §3.3 ----
 * Jobs are visited in a fixed order: (k1 desc, k2 desc, j asc). */
typedef struct {
    uint64_t k1;
    uint32_t k2;
    int32_t j;
} ord_t;

static int ord_cmp(const void* A, const void* B) {
    const ord_t* a = (const ord_t*)A;
    const ord_t* b = (const ord_t*)B;
    if (a->k1 != b->k1) return a->k1 > b->k1 ? -1 : 1;
    if (a->k2 != b->k2) return a->k2 > b->k2 ? -1 : 1;
    return (a->j < b->j) ? -1 : (a->j > b->j);
}

/* caps: per-round capacity (NULL = G in every round); unit: every width
 * counts 1 (the class-wise P2 repack, where a class's capacity is in jobs). */
static void pack(const twin_t* P, const int32_t* nin, const uint64_t* k1, const uint32_t* k2,
                 uint8_t* y, int32_t* placed, const int32_t* caps, int unit) {
    const int32_t N = P->N, T = P->T, G = P->G;
    size_t NN = N > 0 ? (size_t)N : 1;
    ord_t* ord = (ord_t*)malloc(sizeof(ord_t) * NN);
    int32_t* r = (int32_t*)malloc(sizeof(int32_t) * NN);
    int32_t* ww = (int32_t*)malloc(sizeof(int32_t) * NN);
    uint8_t* sel = (uint8_t*)malloc(NN);
    int32_t A = 0;
    for (int32_t j = 0; j < N; ++j)
        if (nin[j] > 0) { ord[A].k1 = k1[j]; ord[A].k2 = k2[j]; ord[A].j = j; ++A; }
    qsort(ord, (size_t)A, sizeof(ord_t), ord_cmp);
    for (int32_t i = 0; i < A; ++i) { r[i] = nin[ord[i].j]; ww[i] = unit ? 1 : P->jc[ord[i].j].w; }
    memset(y, 0, NN * (size_t)T);
    int64_t H[SW_TMAX + 1], SH[SW_TMAX + 1], need[SW_TMAX];
    int64_t Lsum[SW_TMAX + 1];
    int32_t fut[SW_TMAX];
    for (int32_t t = 0; t < T; ++t) {
        int32_t R = T - t;
        int64_t cap = caps ? caps[t] : G;
        for (int32_t v = 0; v <= R; ++v) { H[v] = 0; SH[v] = 0; }
        for (int32_t i = 0; i < A; ++i) H[r[i] < R ? r[i] : R] += ww[i];
        /* Lsum[x] = the x smallest capacities of the rounds after t: the room
         * jobs with more than m rounds left have after this round is
         * Lsum[R−1−m] (= G·(R−1−m) for uniform capacity) */
        Lsum[0] = 0;
        if (caps) {
            for (int32_t u = 0; u < R - 1; ++u) fut[u] = caps[t + 1 + u];
            for (int32_t u = 1; u < R - 1; ++u) { /* insertion sort, ascending */
                int32_t v = fut[u], x = u - 1;
                while (x >= 0 && fut[x] > v) { fut[x + 1] = fut[x]; --x; }
                fut[x + 1] = v;
            }
            for (int32_t u = 0; u < R - 1; ++u) Lsum[u + 1] = Lsum[u] + fut[u];
        } else {
            for (int32_t u = 0; u < R - 1; ++u) Lsum[u + 1] = Lsum[u] + G;
        }
        for (int32_t m = 0; m < R; ++m) {
            int64_t D = 0;
            for (int32_t v = m + 1; v <= R; ++v) D += H[v] * (int64_t)(v - m);
            need[m] = D - Lsum[R - 1 - m];
        }
        memset(sel, 0, (size_t)(A > 0 ? A : 1));
        /* tiers: jobs with more than m rounds left must shed enough now */
        for (int32_t m = R - 1; m >= 0; --m) {
            int64_t red = 0;
            for (int32_t v = m + 1; v <= R; ++v) red += SH[v];
            int64_t q = need[m] - red;
            if (q <= 0) continue;
            int64_t excl = 0, took = 0;
            for (int32_t i = 0; i < A; ++i) {
                int32_t rr = r[i] < R ? r[i] : R;
                if (sel[i] || rr <= m) continue;
                if (excl < q && excl + ww[i] <= cap) {
                    sel[i] = 1; SH[rr] += ww[i]; took += ww[i];
                }
                excl += ww[i];
            }
            cap -= took;
        }
        /* fill the rest of the round in order */
        {
            int64_t excl = 0, took = 0;
            for (int32_t i = 0; i < A; ++i) {
                if (sel[i] || r[i] <= 0) continue;
                if (excl + ww[i] <= cap) { sel[i] = 1; took += ww[i]; }
                excl += ww[i];
            }
            cap -= took;
        }
        /* width tail */
        while (cap > 0) {
            int32_t pick = -1;
            for (int32_t i = 0; i < A; ++i)
                if (!sel[i] && r[i] > 0 && ww[i] <= cap) { pick = i; break; }
            if (pick < 0) break;
            sel[pick] = 1; cap -= ww[pick];
        }
        for (int32_t i = 0; i < A; ++i)
            if (sel[i]) { y[(size_t)ord[i].j * T + t] = 1; r[i] -= 1; }
    }
    for (int32_t j = 0; j < N; ++j) placed[j] = 0;
    for (int32_t i = 0; i < A; ++i) placed[ord[i].j] = nin[ord[i].j] - r[i];
    free(ord); free(r); free(ww); free(sel);
}

/* Density placement with profile repair (sw_repair.h): yd / pd are the
 * density-order pack of nin that left rounds unplaced.  Builds the width
 * classes' profile and free GPUs per round from it, repairs the profile and
 * repacks every changed class alone (unit widths, order p_j/n_j) inside its
 * new capacities; unchanged classes keep their density rows.  Writes yout
 * and placed; returns 1 when every round of nin is placed. */
static int repack_classes(const twin_t* P, const sw_problem* pr, const int32_t* nin,
                          const sw_repair_t* Rp, uint8_t* yout, int32_t* placed);

static int repair_pack(const twin_t* P, const sw_problem* pr, const int32_t* nin, const uint8_t* yd,
                       const int32_t* pd, uint8_t* yout, int32_t* placed) {
    const int32_t N = P->N, T = P->T;
    sw_repair_t R;
    memset(&R, 0, sizeof(R));
    for (int32_t j = 0; j < N; ++j)
        if (nin[j] > 0 && sw_repair_add_class(&R, P->jc[j].w) < 0) return 0;
    for (int32_t t = 0; t < T; ++t) R.L[t] = P->G;
    for (int32_t j = 0; j < N; ++j) {
        for (int32_t t = 0; t < T; ++t) R.L[t] -= P->jc[j].w * yd[(size_t)j * T + t];
        if (nin[j] <= 0) continue;
        const int32_t c = sw_repair_class(&R, P->jc[j].w);
        R.M[c] += 1;
        R.D[c] += nin[j] - pd[j];
        for (int32_t t = 0; t < T; ++t) R.caps[c][t] += yd[(size_t)j * T + t];
    }
    if (sw_profile_repair(&R, T) != 0) return 0;
    size_t NN = N > 0 ? (size_t)N : 1;
    memcpy(yout, yd, NN * (size_t)T);
    memcpy(placed, pd, sizeof(int32_t) * NN);
    return repack_classes(P, pr, nin, &R, yout, placed);
}

/* Repack every changed class of the profile R alone with unit widths, order
 * p_j/n_j, inside its per-round capacities R->caps; the other rows of yout /
 * placed are kept.  Returns 1 when every round of nin is placed. */
static int repack_classes(const twin_t* P, const sw_problem* pr, const int32_t* nin,
                          const sw_repair_t* Rp, uint8_t* yout, int32_t* placed) {
    const int32_t N = P->N, T = P->T;
    const sw_repair_t R = *Rp;
    size_t NN = N > 0 ? (size_t)N : 1;
    int32_t* nc = (int32_t*)malloc(sizeof(int32_t) * NN);
    int32_t* pc = (int32_t*)malloc(sizeof(int32_t) * NN);
    uint64_t* k1 = (uint64_t*)malloc(sizeof(uint64_t) * NN);
    uint32_t* k2 = (uint32_t*)calloc(NN, sizeof(uint32_t));
    uint8_t* yc = (uint8_t*)malloc(NN * (size_t)(T > 0 ? T : 1));
    for (int32_t c = 0; c < R.ncls; ++c) {
        if (!R.changed[c]) continue;
        for (int32_t j = 0; j < N; ++j) {
            const int cls = nin[j] > 0 && P->jc[j].w == R.wc[c];
            nc[j] = cls ? nin[j] : 0;
            k1[j] = cls ? sw_ratio_key(pr->priority[j] / (double)nin[j]) : 0;
        }
        pack(P, nc, k1, k2, yc, pc, R.caps[c], 1);
        for (int32_t j = 0; j < N; ++j)
            if (nc[j] > 0) {
                memcpy(yout + (size_t)j * T, yc + (size_t)j * T, (size_t)T);
                placed[j] = pc[j];
            }
    }
    int ok = 1;
    for (int32_t j = 0; j < N; ++j) ok &= (placed[j] == nin[j]);
    free(nc); free(pc); free(k1); free(k2); free(yc);
    return ok;
}

/* Pattern placement (sw_profile_search): when neither the density order nor
 * its repair places nin, search an exact width-class profile over round
 * patterns and pack every class inside it (unit widths, order p_j/n_j).
 * Writes yout and placed; returns 1 when every round of nin is placed. */
static int pattern_pack(const twin_t* P, const sw_problem* pr, const int32_t* nin, uint8_t* yout,
                        int32_t* placed) {
    const int32_t N = P->N, T = P->T;
    sw_repair_t R;
    memset(&R, 0, sizeof(R));
    int32_t A = 0;
    for (int32_t j = 0; j < N; ++j)
        if (nin[j] > 0) {
            if (sw_repair_add_class(&R, P->jc[j].w) < 0) return 0;
            ++A;
        }
    if (A == 0) return 0;
    int32_t* hist = (int32_t*)calloc((size_t)R.ncls * (T + 1), sizeof(int32_t));
    int32_t* scratch = (int32_t*)malloc(sizeof(int32_t) * (size_t)SW_PAT_SCRATCH(A));
    for (int32_t j = 0; j < N; ++j)
        if (nin[j] > 0) {
            const int32_t c = sw_repair_class(&R, P->jc[j].w);
            R.M[c] += 1;
            hist[c * (T + 1) + nin[j]] += 1;
        }
    int64_t nodes = 0;
    const int32_t found = sw_profile_search(&R, T, P->G, hist, scratch, &nodes);
    free(hist);
    free(scratch);
    if (!found) return 0;
    size_t NN = N > 0 ? (size_t)N : 1;
    memset(yout, 0, NN * (size_t)T);
    for (int32_t j = 0; j < N; ++j) placed[j] = 0;
    return repack_classes(P, pr, nin, &R, yout, placed);
}

/* The packer over plain arrays, for the sharded CPU engine (oracle/shard_twin.c):
 * pack() reads only N, T, G and the widths. */
void twin_pack_arrays_caps(int32_t N, int32_t T, int32_t G, const int32_t* w, const int32_t* nin,
                           const uint64_t* k1, const uint32_t* k2, uint8_t* y, int32_t* placed,
                           const int32_t* caps, int unit) {
    twin_t P;
    memset(&P, 0, sizeof(P));
    P.N = N; P.T = T; P.G = G;
    P.jc = (sw_jobc*)calloc(N > 0 ? (size_t)N : 1, sizeof(sw_jobc));
    for (int32_t j = 0; j < N; ++j) P.jc[j].w = w[j];
    pack(&P, nin, k1, k2, y, placed, caps, unit);
    free(P.jc);
}

void twin_pack_arrays(int32_t N, int32_t T, int32_t G, const int32_t* w, const int32_t* nin,
                      const uint64_t* k1, const uint32_t* k2, uint8_t* y, int32_t* placed) {
    twin_pack_arrays_caps(N, T, G, w, nin, k1, k2, y, placed, NULL, 0);
}

static void build(twin_t* P, const sw_problem* pr) {
    const int32_t N = pr->num_jobs, T = pr->future_rounds;
    P->N = N; P->T = T; P->G = pr->num_gpus; P->nb = pr->num_bases;
    P->C = (int64_t)pr->num_gpus * T;
    P->k = pr->regularizer;
    P->beta = pr->bases; P->ell = pr->log_bases;
    sw_pwl_slopes(P->nb, P->beta, P->ell, P->slope);
    P->passes = 0;
    size_t NN = N > 0 ? (size_t)N : 1;
    P->jc = (sw_jobc*)malloc(sizeof(sw_jobc) * NN);
    P->key = (float*)malloc(sizeof(float) * NN * T);
    P->Tj = (int32_t*)malloc(sizeof(int32_t) * NN);
    double A = 0.0;
    for (int32_t j = 0; j < N; ++j) {
        P->jc[j] = sw_make_jobc(N, T, pr->round_duration, pr->nworkers[j], pr->epoch_duration[j],
                                pr->completed_epochs[j], pr->total_epochs[j],
                                pr->remaining_runtime[j], pr->priority[j]);
        A = P->jc[j].a > A ? P->jc[j].a : A;
        P->Tj[j] = pr->nworkers[j] <= pr->num_gpus ? T : 0;
    }
    P->A = A;
    for (int32_t j = 0; j < N; ++j) {
        const double ks = sw_key_scale(P->jc[j].w, A);
        double prev = fval(P, j, 0), vm = 0.0;
        for (int32_t n = 0; n < T; ++n) {
            double cur = fval(P, j, n + 1);
            double v = sw_pos(cur - prev);
            vm = (n == 0) ? v : sw_min(vm, v);
            K_(P, j, n) = sw_key(vm, ks);
            prev = cur;
        }
    }
}

/* Level search over the makespan M.  Writes the best
 * counts to nb, returns the upper bound U∞bound − k·M_lo. */
static double level_search(twin_t* P, int32_t* n, int32_t* nb, int32_t* l, int32_t* tk,
                           double* tmp) {
    const int32_t N = P->N;
    size_t NN = N > 0 ? (size_t)N : 1;
    sel_eval_t ev, best;
    if (!(N > 0 && P->k > 0.0)) { /* no makespan term: the utility optimum */
        select_level(P, 0.0, 1, n, l, tk, tmp, &ev, 0, SW_KEY_INF_BITS);
        memcpy(nb, n, sizeof(int32_t) * NN);
        return ev.ubound - P->k * ev.Mact;
    }
    /* M_lo = the smallest level whose forced rounds fit, min{M : F(M) ≤ C},
     * F(M) = Σ_j w_j·#{n < T_j : g_j(n) > M}, searched on [lb, top]:
     * lb = max_j g_j(T_j) (no plan does better), top = max_j g_j(0) (F = 0).
     * F only steps at the row values g_j(n), so the answer is one of them (or
     * lb): each probe also returns the largest row value ≤ it and the
     * smallest > it, and the bracket jumps to those.  Probes: the value
     * midpoint until both ends carry a measured F, then the level where the
     * line through (lo, F just below lo) and (hi, F(hi)) crosses C. */
    double lb = 0.0, top = 0.0;
    for (int32_t j = 0; j < N; ++j) {
        lb = sw_max(lb, sw_g(&P->jc[j], P->Tj[j]));
        top = sw_max(top, sw_g(&P->jc[j], 0));
    }
    uint64_t lo = sw_bits(lb), hi = sw_bits(top);
    int64_t Fb = -1, Fh = -1;
    while (lo < hi) {
        double x = (sw_from_bits(lo) + sw_from_bits(hi)) * 0.5;
        if (Fb >= 0 && Fh >= 0)
            x = sw_from_bits(lo) + (sw_from_bits(hi) - sw_from_bits(lo)) *
                                       ((double)(Fb - P->C) / (double)(Fb - Fh));
        if (sw_bits(x) >= hi) x = sw_from_bits(hi - 1);
        if (sw_bits(x) < lo) x = sw_from_bits(lo);
        int64_t F = 0;
        uint64_t bmax = 0, bmin = UINT64_MAX;
        for (int32_t j = 0; j < N; ++j) {
            const int32_t c = lforce(P, j, x);
            F += (int64_t)P->jc[j].w * c;
            if (c < P->Tj[j]) {
                const uint64_t b = sw_bits(sw_g(&P->jc[j], c));
                bmax = b > bmax ? b : bmax;
            }
            if (c > 0) {
                const uint64_t b = sw_bits(sw_g(&P->jc[j], c - 1));
                bmin = b < bmin ? b : bmin;
            }
        }
        P->passes++;
        if (F <= P->C) { hi = bmax >= lo ? bmax : lo; Fh = F; }
        else { lo = bmin <= hi ? bmin : hi; Fb = F; }
    }
    const double M_lo = sw_from_bits(lo);
    sel_eval_t elo;
    select_level(P, M_lo, 0, n, l, tk, tmp, &elo, 0, SW_KEY_INF_BITS);
    best = elo;
    memcpy(nb, n, sizeof(int32_t) * NN);
    /* Can any higher level win?  A level M > M_lo has J ≤ U_max − k·M with
     * U_max = Σ_j f_j(T_j), so only levels below M_lo + (U_max − U(M_lo))/k
     * can; F is constant between row values, so with no row value in that
     * window M_lo is optimal (ties go to the smaller makespan) and the
     * utility-only level +∞ is never evaluated — the common case when the
     * makespan term dominates (k·M ≫ U: the 256- and 64-GPU configurations). */
    for (int32_t j = 0; j < N; ++j) tmp[j] = fval(P, j, P->Tj[j]);
    const double U_max = sw_detsum(tmp, N);
    P->passes++;
    const double wmax = (U_max - elo.U) / P->k;
    if (!(wmax > 0.0) || levels_between(P, M_lo, M_lo + wmax) == 0) return elo.ubound - P->k * M_lo;
    /* the utility-only level +∞: its price is below ρ*(M_lo) */
    select_level(P, 0.0, 1, n, l, tk, tmp, &ev, 0, elo.rho);
    if (ev.J > best.J || (ev.J == best.J && ev.Mact < best.Mact)) {
        best = ev; memcpy(nb, n, sizeof(int32_t) * NN);
    }
    /* Branch and bound over the levels in (M_lo, M_free] (sw_bnb.h): plans
     * with makespan M_lo or ≥ M_free are bounded by the two evaluated
     * points; an open interval (a, b] by Vub(b) − k·a.  The interval of
     * largest bound is split at its midpoint; ρ*(b) ≤ ρ*(m) ≤ ρ*(a) brackets
     * the probe's price. */
    const double kk = P->k, M_free = ev.Mact;
    double cert = sw_max(elo.ubound - kk * M_lo, ev.ubound - kk * M_free);
    sw_bnb_ivl L[SW_BNB_CAP];
    int32_t nL = 0, probes = 0;
    if (M_lo < M_free) L[nL++] = sw_bnb_make(M_lo, M_free, ev.ubound, elo.rho, ev.rho);
    while (nL > 0) {
        double kb;
        const int32_t i = sw_bnb_pick(L, nL, kk, &kb);
        if (kb <= best.J) break; /* nothing left can beat the best plan */
        if (probes == SW_BNB_PROBES) { cert = sw_max(cert, kb); break; }
        const sw_bnb_ivl I = L[i];
        L[i] = L[--nL];
        if (levels_between(P, I.a, I.b) == 0) { /* only b itself, if b is a level */
            cert = sw_max(cert, I.vb - kk * I.b);
            continue;
        }
        const double m = sw_bnb_mid(I.a, I.b);
        sel_eval_t e;
        select_level(P, m, 0, n, l, tk, tmp, &e, I.rb, I.ra);
        ++probes;
        if (e.J > best.J || (e.J == best.J && e.Mact < best.Mact)) {
            best = e; memcpy(nb, n, sizeof(int32_t) * NN);
        }
        if (sw_bnb_key(e.ubound, kk, I.a) > best.J) L[nL++] = sw_bnb_make(I.a, m, e.ubound, I.ra, e.rho);
        if (sw_bnb_key(I.vb, kk, m) > best.J) L[nL++] = sw_bnb_make(m, I.b, I.vb, e.rho, I.rb);
    }
    return sw_max(cert, best.J);
}

/* Fill of stranded capacity (the reference MILP packs per
 * round, shockwave.py:64-75, so its optimum never leaves a round's room to a
 * job that gains from it).  After the reduced-budget re-solve the best P1 plan
 * y / n can leave GPUs idle in some rounds: add single rounds there, each time
 * the candidate (job j with n_j < T_j, first round t without j whose free
 * capacity fits w_j) of largest gain f(n_j + 1) − f(n_j) (sw_fill_key), until
 * none has a positive gain or SW_FILL_MAX rounds were added.  The makespan
 * term can only fall.  Returns the number of rounds added. */
static int fill_stranded(twin_t* P, int32_t* n, uint8_t* y) {
    const int32_t N = P->N, T = P->T, G = P->G;
    int64_t load[SW_TMAX];
    for (int32_t t = 0; t < T; ++t) load[t] = 0;
    for (int32_t j = 0; j < N; ++j)
        for (int32_t t = 0; t < T; ++t)
            if (y[(size_t)j * T + t]) load[t] += P->jc[j].w;
    int added = 0;
    for (int step = 0; step < SW_FILL_MAX; ++step) {
        uint64_t best = 0;
        for (int32_t j = 0; j < N; ++j) {
            if (n[j] >= P->Tj[j]) continue;
            const int64_t w = P->jc[j].w;
            int32_t tf = -1;
            for (int32_t t = 0; t < T; ++t)
                if (!y[(size_t)j * T + t] && w <= G - load[t]) { tf = t; break; }
            if (tf < 0) continue;
            const uint64_t key = sw_fill_key(fval(P, j, n[j] + 1) - fval(P, j, n[j]), j, tf);
            best = key > best ? key : best;
        }
        P->passes++;
        if (best == 0) break;
        const int64_t jb = sw_fill_job(best);
        const int32_t tb = sw_fill_round(best);
        y[(size_t)jb * T + tb] = 1;
        n[jb] += 1;
        load[tb] += P->jc[jb].w;
        ++added;
    }
    return added;
}

/* The plan's exact objective (the emit's deterministic sum) and makespan. */
static double plan_objective(const twin_t* P, const int32_t* n, double* tmp) {
    double M = 0.0;
    for (int32_t j = 0; j < P->N; ++j) {
        tmp[j] = fval(P, j, n[j]);
        M = sw_max(M, sw_g(&P->jc[j], n[j]));
    }
    return sw_detsum(tmp, P->N) - P->k * M;
}

/* Raises (sw_arith.h SW_RAISE_ITERS) on the plan n / y;
 * returns the number kept. */
static int raise_counts(twin_t* P, const sw_problem* pr, int32_t* n, uint8_t* y) {
    const int32_t N = P->N, T = P->T;
    const size_t NN = N > 0 ? (size_t)N : 1;
    int32_t* nt = (int32_t*)malloc(sizeof(int32_t) * NN);
    int32_t* pt = (int32_t*)malloc(sizeof(int32_t) * NN);
    uint8_t* yt = (uint8_t*)malloc(NN * (size_t)T);
    uint64_t* key = (uint64_t*)malloc(sizeof(uint64_t) * NN);
    double* tmp = (double*)malloc(sizeof(double) * NN);
    const int64_t C0 = (int64_t)P->G * T;
    int kept = 0;
    for (int it = 0; it < SW_RAISE_ITERS; ++it) {
        const double J = plan_objective(P, n, tmp);
        /* M, the first job attaining it, and the largest g of the others */
        double M = -1.0, M2 = 0.0;
        int32_t i1 = -1;
        for (int32_t j = 0; j < N; ++j) {
            const double g = sw_g(&P->jc[j], n[j]);
            if (g > M) { if (i1 >= 0) M2 = sw_max(M2, M); M = g; i1 = j; }
            else M2 = sw_max(M2, g);
        }
        if (M < 0.0) M = 0.0;
        int64_t load = 0;
        for (int32_t j = 0; j < N; ++j) {
            load += (int64_t)P->jc[j].w * n[j];
            key[j] = 0;
            if (n[j] >= P->Tj[j]) continue;
            const double Mo = j == i1 ? M2 : M;
            key[j] = sw_fill_key(sw_raise_gain(fval(P, j, n[j]), fval(P, j, n[j] + 1),
                                               sw_g(&P->jc[j], n[j] + 1), Mo, M, P->k), j, 0);
        }
        P->passes++;
        int took = 0;
        for (int tr = 0; tr < SW_RAISE_TRIES && !took; ++tr) {
            uint64_t best = 0;
            for (int32_t j = 0; j < N; ++j) best = key[j] > best ? key[j] : best;
            if (best == 0) break;
            const int32_t b = (int32_t)sw_fill_job(best);
            key[b] = 0;
            if (load + P->jc[b].w > C0) continue;
            memcpy(nt, n, sizeof(int32_t) * NN);
            nt[b] += 1;
            if (!pattern_pack(P, pr, nt, yt, pt)) continue;
            if (plan_objective(P, pt, tmp) > J) {
                memcpy(n, pt, sizeof(int32_t) * NN);
                memcpy(y, yt, NN * (size_t)T);
                took = 1;
            }
        }
        if (!took) break;
        ++kept;
    }
    free(nt); free(pt); free(yt); free(key); free(tmp);
    return kept;
}

/* ---- per-round exact re-optimisation (sw_reround.h: the specification the
 * GPU block function sw_reround_dev.h follows step for step) ---- */
typedef struct {
    int32_t N, T, G, nb;
    double k;
    const double *beta, *ell, *slope;
    const sw_jobc* jc;
    const int32_t* Tj;
    double *v, *h0, *h1, *tmp;
    uint8_t *S, *Sb, *cand;
    int32_t* items;
    uint64_t* bits;
    double* dp;
    int64_t budget, passes;
} rr_t;

static double rr_f(const rr_t* R, int32_t j, int32_t n) {
    return sw_f(&R->jc[j], n, R->nb, R->beta, R->ell, R->slope);
}

/* J(S) = detsum(S·v) − k·max(S ? h1 : h0) */
static double rr_value(rr_t* R, const uint8_t* S) {
    double m = 0.0;
    for (int32_t j = 0; j < R->N; ++j) {
        R->tmp[j] = S[j] ? R->v[j] : 0.0;
        const double h = S[j] ? R->h1[j] : R->h0[j];
        m = h > m ? h : m;
    }
    return sw_detsum(R->tmp, R->N) - R->k * m;
}

/* The knapsack of sw_reround.h over the jobs with cand[j], capacity cap;
 * sets S[j] = 1 for the jobs taken (S keeps its other entries).  Returns 0
 * when the knapsack is outside the limits (nothing set). */
static int rr_knap(rr_t* R, const uint8_t* cand, int64_t cap, uint8_t* S) {
    int32_t ni = 0;
    int64_t tot = 0;
    for (int32_t j = 0; j < R->N; ++j)
        if (cand[j]) { R->items[ni++] = j; tot += R->jc[j].w; }
    if (tot <= cap) {
        for (int32_t i = 0; i < ni; ++i) S[R->items[i]] = 1;
        return 1;
    }
    if (cap > SW_RR_CAPMAX) return 0;
    const int32_t nw = (int32_t)((cap + 64) / 64);
    if ((int64_t)ni * nw > SW_RR_WORDS || R->budget < ni) return 0;
    R->budget -= ni;
    for (int64_t c = 0; c <= cap; ++c) R->dp[c] = 0.0;
    for (int32_t i = 0; i < ni; ++i) {
        const int32_t j = R->items[i], w = R->jc[j].w;
        uint64_t* b = R->bits + (size_t)i * nw;
        for (int32_t x = 0; x < nw; ++x) b[x] = 0;
        for (int64_t c = cap; c >= w; --c) {
            const double x = R->dp[c - w] + R->v[j];
            if (x > R->dp[c]) { R->dp[c] = x; b[c >> 6] |= 1ull << (c & 63); }
        }
    }
    int64_t cs = 0;
    for (int64_t c = 1; c <= cap; ++c)
        if (R->dp[c] > R->dp[cs]) cs = c;
    for (int32_t i = ni - 1; i >= 0; --i)
        if ((R->bits[(size_t)i * nw + (cs >> 6)] >> (cs & 63)) & 1ull) {
            S[R->items[i]] = 1;
            cs -= R->jc[R->items[i]].w;
        }
    return 1;
}

/* One round t: returns 1 when its job set was replaced (y, n updated). */
static int rr_round(rr_t* R, int32_t t, int32_t* n, uint8_t* y) {
    const int32_t N = R->N, T = R->T;
    const double INF = 1.0 / 0.0;
    R->passes++;
    for (int32_t j = 0; j < N; ++j) {
        const int32_t in = y[(size_t)j * T + t] != 0, b = n[j] - in;
        const int el = R->Tj[j] > 0;
        R->v[j] = el ? rr_f(R, j, b + 1) - rr_f(R, j, b) : 0.0;
        R->h0[j] = sw_g(&R->jc[j], b);
        R->h1[j] = el ? sw_g(&R->jc[j], b + 1) : R->h0[j];
        R->Sb[j] = (uint8_t)in; /* the current set, for its value */
    }
    const double Jcur = rr_value(R, R->Sb);
    for (int32_t j = 0; j < N; ++j) {
        R->cand[j] = R->Tj[j] > 0 && R->v[j] > 0.0 && R->jc[j].w <= R->G;
        R->S[j] = 0;
    }
    if (!rr_knap(R, R->cand, R->G, R->S)) return 0;
    double D = 0.0;
    for (int32_t j = 0; j < N; ++j) R->tmp[j] = R->S[j] ? R->v[j] : 0.0;
    D = sw_detsum(R->tmp, N);
    double Jb = rr_value(R, R->S);
    memcpy(R->Sb, R->S, (size_t)N);
    /* the smallest feasible level θ0: every job above it must fit one more
     * round under it (θ ≥ h1_j, θ ≥ h0_j for a job wider than G) and the
     * forced widths Σ_{h0_j > θ} w_j must fit G — a bisection over the fp64
     * bits snapped to the h0 values (W only changes there) */
    double La = 0.0, hmax = 0.0;
    for (int32_t j = 0; j < N; ++j) {
        const double a = R->Tj[j] > 0 ? R->h1[j] : R->h0[j];
        La = a > La ? a : La;
        hmax = R->h0[j] > hmax ? R->h0[j] : hmax;
    }
    uint64_t lo = 0, hi = sw_bits(hmax);
    while (lo < hi) {
        const double x = sw_from_bits(lo + ((hi - lo) >> 1));
        int64_t W = 0;
        uint64_t mx = 0, mn = UINT64_MAX;
        for (int32_t j = 0; j < N; ++j) {
            const uint64_t b = sw_bits(R->h0[j]);
            if (R->h0[j] > x) { W += R->jc[j].w; mn = b < mn ? b : mn; }
            else mx = b > mx ? b : mx;
        }
        R->passes++;
        if (W <= R->G) hi = mx > lo ? mx : lo;
        else lo = mn < hi ? mn : hi;
    }
    const double th0 = sw_max(La, sw_from_bits(lo));
    double lvl = th0, prev = 0.0;
    int have_prev = 0;
    for (int32_t tried = 0; tried < SW_RR_LEVELS; ++tried) {
        double th = tried == 0 ? th0 : INF;
        if (tried > 0)
            for (int32_t j = 0; j < N; ++j) {
                if (R->h0[j] > lvl && R->h0[j] < th) th = R->h0[j];
                if (R->h1[j] > lvl && R->h1[j] < th) th = R->h1[j];
            }
        if (th == INF) break;
        if (have_prev && D - R->k * prev <= Jb) break;
        prev = th;
        have_prev = 1;
        lvl = th;
        R->passes++;
        int ok = 1;
        int64_t wf = 0;
        for (int32_t j = 0; j < N; ++j) {
            R->S[j] = R->h0[j] > th;
            if (R->S[j]) {
                if (R->Tj[j] == 0 || R->h1[j] > th) ok = 0;
                wf += R->jc[j].w;
            }
        }
        if (!ok || wf > R->G) continue;
        const int64_t cap = (int64_t)R->G - wf;
        for (int32_t j = 0; j < N; ++j)
            R->cand[j] = !R->S[j] && R->Tj[j] > 0 && R->v[j] > 0.0 && R->jc[j].w <= cap;
        if (!rr_knap(R, R->cand, cap, R->S)) continue;
        const double J = rr_value(R, R->S);
        if (J > Jb) {
            Jb = J;
            memcpy(R->Sb, R->S, (size_t)N);
        }
    }
    if (!(Jb - Jcur > SW_RR_TOL * (fabs(Jb) + fabs(Jcur)))) return 0;
    for (int32_t j = 0; j < N; ++j) {
        uint8_t* cell = &y[(size_t)j * T + t];
        if ((*cell != 0) != (R->Sb[j] != 0)) {
            n[j] += R->Sb[j] ? 1 : -1;
            *cell = R->Sb[j];
        }
    }
    return 1;
}

/* The step over the plan y ([N][T] bytes) with counts n (updated in place);
 * returns the number of rounds whose set changed; *passes grows by the
 * rounds visited and the levels tried.  Exported for the sharded CPU engine
 * (oracle/shard_twin.c), which runs it on the gathered placement. */
int32_t twin_reround_arrays(int32_t N, int32_t T, int32_t G, double k, int32_t nb,
                            const double* beta, const double* ell, const sw_jobc* jc,
                            int32_t* n, uint8_t* y, int64_t* passes) {
    rr_t R;
    double slope[SW_BMAX];
    sw_pwl_slopes(nb, beta, ell, slope);
    const size_t NN = N > 0 ? (size_t)N : 1;
    R.N = N; R.T = T; R.G = G; R.nb = nb; R.k = k;
    R.beta = beta; R.ell = ell; R.slope = slope; R.jc = jc;
    int32_t* Tj = (int32_t*)malloc(sizeof(int32_t) * NN);
    R.v = (double*)malloc(sizeof(double) * NN);
    R.h0 = (double*)malloc(sizeof(double) * NN);
    R.h1 = (double*)malloc(sizeof(double) * NN);
    R.tmp = (double*)malloc(sizeof(double) * NN);
    R.S = (uint8_t*)malloc(NN);
    R.Sb = (uint8_t*)malloc(NN);
    R.cand = (uint8_t*)malloc(NN);
    R.items = (int32_t*)malloc(sizeof(int32_t) * NN);
    R.bits = (uint64_t*)malloc(sizeof(uint64_t) * SW_RR_WORDS);
    R.dp = (double*)malloc(sizeof(double) * (SW_RR_CAPMAX + 1));
    R.budget = SW_RR_BUDGET;
    R.passes = 0;
    for (int32_t j = 0; j < N; ++j) Tj[j] = jc[j].w <= G ? T : 0;
    R.Tj = Tj;
    int32_t moves = 0;
    for (int32_t pass = 0; pass < SW_RR_PASSES; ++pass) {
        int changed = 0;
        for (int32_t t = 0; t < T; ++t) {
            const int c = rr_round(&R, t, n, y);
            changed |= c;
            moves += c;
        }
        if (!changed) break;
    }
    *passes += R.passes;
    free(Tj); free(R.v); free(R.h0); free(R.h1); free(R.tmp); free(R.S); free(R.Sb);
    free(R.cand); free(R.items); free(R.bits); free(R.dp);
    return moves;
}

/* Full plan solve; same contract as sw_plan_solve in include/shockwave_amd.h. */
int twin_plan_solve(const sw_problem* pr, sw_result* res) {
    if (sw_validate_problem(pr) != 0) return SW_ERR_INVALID;
    const int32_t N = pr->num_jobs, T = pr->future_rounds;
    twin_t P;
    build(&P, pr);
    size_t NN = N > 0 ? (size_t)N : 1;
    int32_t* n = (int32_t*)malloc(sizeof(int32_t) * NN);
    int32_t* nb = (int32_t*)malloc(sizeof(int32_t) * NN);
    int32_t* l = (int32_t*)malloc(sizeof(int32_t) * NN);
    int32_t* tk = (int32_t*)malloc(sizeof(int32_t) * NN);
    int32_t* placed = (int32_t*)malloc(sizeof(int32_t) * NN);
    double* tmp = (double*)malloc(sizeof(double) * NN);
    uint8_t* y1 = (uint8_t*)malloc(NN * T);
    uint8_t* y2 = (uint8_t*)malloc(NN * T);
    uint8_t* ybest = (uint8_t*)malloc(NN * T);
    int32_t* placed2 = (int32_t*)malloc(sizeof(int32_t) * NN);

    /* ---- P1: level search + packing, re-solved on a smaller budget when
     *      widths fragment the rounds ---- */
    int32_t status = 0;
    uint64_t* k1 = (uint64_t*)malloc(sizeof(uint64_t) * NN);
    uint32_t* k2 = (uint32_t*)malloc(sizeof(uint32_t) * NN);
    int32_t* nbest = (int32_t*)malloc(sizeof(int32_t) * NN);
    double bound = 0.0, Jbest = 0.0;
    int dens_best = 0; /* the best P1 plan is the density-order pack */
    int rep_best = 0;  /* ... with its width profile repaired (sw_repair.h) */
    int dskip_best = 0; /* density failed on exactly the final counts: P2 (a) would too */
    for (int it = 0; it < SW_REPACK_ITERS; ++it) {
        double b0 = level_search(&P, n, nb, l, tk, tmp);
        if (it == 0) bound = b0;
        double Mb = 0.0;
        for (int32_t j = 0; j < N; ++j) Mb = sw_max(Mb, sw_g(&P.jc[j], nb[j]));
        /* packing orders: first P2's density order p_j/(n_j·w_j) — when it
         * places every round it is also the P2 placement (same counts, same
         * order) and the solve needs no other pack; otherwise A = (critical
         * level, key) and B = (critical level, width, key), where critical =
         * losing the last round raises the makespan (only meaningful when
         * k > 0).  Keep the better packed plan of A and B. */
        int64_t deficit = 0;
        double Jp = 0.0;
        int dens = 0, rep = 0;
        for (int ord = -1; ord < 2; ++ord) {
            for (int32_t j = 0; j < N; ++j) {
                if (ord < 0) {
                    k1[j] = nb[j] > 0 ? sw_ratio_key(pr->priority[j] / (double)(nb[j] * P.jc[j].w)) : 0;
                    k2[j] = 0;
                } else if (nb[j] > 0) {
                    double lvl = sw_g(&P.jc[j], nb[j] - 1);
                    int crit = P.k > 0.0 && lvl > Mb;
                    k1[j] = crit ? (SW_CRIT_BIT | sw_bits(lvl)) : (ord ? (uint64_t)P.jc[j].w : 0);
                    k2[j] = sw_fbits_of(K_(&P, j, nb[j] - 1));
                } else {
                    k1[j] = 0; k2[j] = 0;
                }
            }
            pack(&P, nb, k1, k2, ord == 1 ? y2 : y1, ord == 1 ? placed2 : placed, NULL, 0);
            int64_t dfc = 0;
            double Mp = 0.0;
            const int32_t* pl = ord == 1 ? placed2 : placed;
            for (int32_t j = 0; j < N; ++j) {
                dfc += (int64_t)P.jc[j].w * (nb[j] - pl[j]);
                tmp[j] = fval(&P, j, pl[j]);
                Mp = sw_max(Mp, sw_g(&P.jc[j], pl[j]));
            }
            double Jo = sw_detsum(tmp, N) - P.k * Mp;
            P.passes++;
            if (ord < 0) {
                /* the density pack stranded rounds: repair its width profile
                 * (sw_repair.h); a repaired placement places every count and
                 * is also the P2 placement, like a density pack that fits */
                if (dfc != 0 && repair_pack(&P, pr, nb, y1, placed, y2, placed2)) {
                    memcpy(y1, y2, NN * (size_t)T);
                    memcpy(placed, placed2, sizeof(int32_t) * NN);
                    dfc = 0;
                    rep = 1;
                    Mp = 0.0;
                    for (int32_t j = 0; j < N; ++j) {
                        tmp[j] = fval(&P, j, placed[j]);
                        Mp = sw_max(Mp, sw_g(&P.jc[j], placed[j]));
                    }
                    Jo = sw_detsum(tmp, N) - P.k * Mp;
                    P.passes++;
                }
                if (dfc == 0) { Jp = Jo; dens = 1; break; }
                continue;
            }
            if (ord == 0 || Jo > Jp) {
                Jp = Jo;
                deficit = dfc;
                if (ord == 1) {
                    memcpy(placed, placed2, sizeof(int32_t) * NN);
                    memcpy(y1, y2, NN * (size_t)T);
                }
            }
            if (ord == 0 && dfc == 0) break; /* order A packed everything */
        }
        /* no order places nb: an exact width-class profile over round
         * patterns, when one exists (sw_profile_search) — the counts are
         * P1's as they are, no re-solve; P2 starts from its cascade */
        if (deficit != 0 && pattern_pack(&P, pr, nb, y1, placed)) {
            double Mp = 0.0;
            for (int32_t j = 0; j < N; ++j) {
                tmp[j] = fval(&P, j, placed[j]);
                Mp = sw_max(Mp, sw_g(&P.jc[j], placed[j]));
            }
            Jp = sw_detsum(tmp, N) - P.k * Mp;
            P.passes++;
            deficit = 0;
        }
        if (it == 0 || Jp > Jbest) {
            Jbest = Jp;
            dens_best = dens;
            rep_best = rep;
            dskip_best = !dens && deficit == 0;
            memcpy(nbest, placed, sizeof(int32_t) * NN);
            memcpy(ybest, y1, NN * (size_t)T);
        }
        if (deficit == 0) break;
        status |= SW_STATUS_P1_REPACKED;
        P.C -= deficit;
    }
    /* a re-solved P1 can strand capacity: fill it (the filled plan is no
     * longer a density pack, so P2 starts from (a) again) */
    if ((status & SW_STATUS_P1_REPACKED) && fill_stranded(&P, nbest, ybest) > 0) {
        dens_best = 0;
        rep_best = 0;
        dskip_best = 0;
    }
    /* ... and re-optimise it round by round (sw_reround.h) */
    if ((status & SW_STATUS_P1_REPACKED) &&
        twin_reround_arrays(N, T, P.G, P.k, P.nb, P.beta, P.ell, P.jc, nbest, ybest, &P.passes) > 0) {
        dens_best = 0;
        rep_best = 0;
        dskip_best = 0;
    }
    /* ... and try raises (sw_arith.h: SW_RAISE_ITERS) */
    if ((status & SW_STATUS_P1_REPACKED) && raise_counts(&P, pr, nbest, ybest) > 0) {
        dens_best = 0;
        rep_best = 0;
        dskip_best = 0;
    }
    memcpy(nb, nbest, sizeof(int32_t) * NN);
    memcpy(y1, ybest, NN * (size_t)T); /* y1 = best P1 plan */
    /* ---- P2: priority placement of the same counts (shockwave.py:281-328).
     * Σ_t t·y_jt is weighted by p_j/n_j per job while a job occupies w_j
     * GPUs, so the placements tried, first success kept, are
     *   (a) density order p_j/(n_j·w_j);
     *   (b) the weight order p_j/n_j;
     *   (c) class-wise: each width class, in ascending width, repacked with
     *       unit widths and order p_j/n_j inside the per-round capacity that
     *       class has in the P1 placement y1 (exact for unit widths, so it
     *       places every round);
     * and the P1 placement if none does (shockwave.py:325-326). ---- */
    int ok2 = 0;
    if (dens_best) { /* (a) is the P1 placement itself */
        memcpy(y2, y1, NN * (size_t)T);
        ok2 = 1;
        if (rep_best) status |= SW_STATUS_P2_REPAIRED;
    }
    for (int att = 0; att < 2 && !ok2; ++att) {
        if (att == 0 && dskip_best) continue;
        for (int32_t j = 0; j < N; ++j) {
            k1[j] = nb[j] > 0 ? sw_ratio_key(pr->priority[j] /
                                        (double)(att == 0 ? nb[j] * P.jc[j].w : nb[j]))
                              : 0;
            k2[j] = 0;
        }
        pack(&P, nb, k1, k2, y2, placed, NULL, 0);
        ok2 = 1;
        for (int32_t j = 0; j < N; ++j) ok2 &= (placed[j] == nb[j]);
        if (!ok2 && att == 0) { /* (a') density with its profile repaired */
            uint8_t* yr = (uint8_t*)malloc(NN * (size_t)T);
            ok2 = repair_pack(&P, pr, nb, y2, placed, yr, placed2);
            if (ok2) {
                memcpy(y2, yr, NN * (size_t)T);
                status |= SW_STATUS_P2_REPAIRED;
            }
            free(yr);
        }
        if (ok2 && att == 1) status |= SW_STATUS_P2_WEIGHT_ORDER;
    }
    if (!ok2) {
        int32_t caps[SW_TMAX];
        int32_t* nc = placed2; /* class counts: nb on the class, 0 elsewhere */
        uint8_t* yc = (uint8_t*)malloc(NN * T);
        memset(y2, 0, NN * (size_t)T);
        ok2 = 1;
        int32_t wprev = 0;
        while (1) {
            int32_t wc = 0x7FFFFFFF;
            for (int32_t j = 0; j < N; ++j)
                if (nb[j] > 0 && P.jc[j].w > wprev && P.jc[j].w < wc) wc = P.jc[j].w;
            if (wc == 0x7FFFFFFF) break;
            for (int32_t t = 0; t < T; ++t) caps[t] = 0;
            for (int32_t j = 0; j < N; ++j) {
                int cls = nb[j] > 0 && P.jc[j].w == wc;
                nc[j] = cls ? nb[j] : 0;
                k1[j] = cls ? sw_ratio_key(pr->priority[j] / (double)nb[j]) : 0;
                k2[j] = 0;
                if (cls)
                    for (int32_t t = 0; t < T; ++t) caps[t] += y1[(size_t)j * T + t];
            }
            pack(&P, nc, k1, k2, yc, placed, caps, 1);
            for (int32_t j = 0; j < N; ++j) {
                if (nc[j] > 0) {
                    ok2 &= (placed[j] == nc[j]);
                    memcpy(y2 + (size_t)j * T, yc + (size_t)j * T, (size_t)T);
                }
            }
            wprev = wc;
        }
        free(yc);
        if (ok2) status |= SW_STATUS_P2_CLASSWISE;
    }
    /* the exchange step (sw_p2x.h) on a P2 placement that
     * placed every round; a fallback keeps P1's x untouched (:325-326) */
    if (ok2 && twin_p2x_plan(N, T, P.G, pr->nworkers, pr->priority, nb, y2) > 0)
        status |= SW_STATUS_P2_EXCHANGED;
    uint8_t* yf = y2;
    if (!ok2) { yf = y1; status |= SW_STATUS_P2_FALLBACK; }
    free(k1); free(k2); free(nbest);
    int any = 0;
    for (int32_t j = 0; j < N; ++j) {
        int32_t c = 0;
        for (int32_t t = 0; t < T; ++t) c += yf[(size_t)j * T + t];
        nb[j] = c;
        any |= (c > 0);
    }
    if (!any) status |= SW_STATUS_NO_PLANNED;
    double Mact = 0.0;
    for (int32_t j = 0; j < N; ++j) {
        tmp[j] = fval(&P, j, nb[j]);
        Mact = sw_max(Mact, sw_g(&P.jc[j], nb[j]));
    }
    double U = sw_detsum(tmp, N);
    for (int32_t j = 0; j < N; ++j) {
        if (nb[j] > 0) {
            int64_t S = 0;
            for (int32_t t = 0; t < T; ++t) S += (int64_t)t * yf[(size_t)j * T + t];
            tmp[j] = ((double)S / (double)nb[j]) * pr->priority[j];
        } else {
            tmp[j] = 0.0;
        }
    }
    res->p2_objective = sw_detsum(tmp, N);
    res->utility = U;
    res->makespan = Mact;
    res->objective = U - P.k * Mact;
    res->bound = bound;
    if (sw_p1_uncertified(res->objective, bound)) status |= SW_STATUS_P1_UNCERTIFIED;
    res->iters = (int32_t)P.passes;
    res->status = status;
    if (res->plan && N > 0) memcpy(res->plan, yf, (size_t)N * T);
    if (res->planned_rounds && N > 0) memcpy(res->planned_rounds, nb, sizeof(int32_t) * (size_t)N);
    if (res->plan_masks)
        for (int32_t j = 0; j < N; ++j) {
            uint64_t m = 0;
            for (int32_t t = 0; t < T; ++t) m |= (uint64_t)(yf[(size_t)j * T + t] != 0) << t;
            res->plan_masks[j] = m;
        }
    free(P.jc); free(P.key); free(P.Tj); free(n); free(nb); free(l); free(tk);
    free(placed); free(placed2); free(tmp); free(y1); free(y2); free(ybest);
    return (status & SW_STATUS_P2_FALLBACK) ? SW_FALLBACK : SW_OK;
}

/* Exposed for tests: the per-job f, g rows (n = 0..T) and fp32 keys (n < T). */
int twin_job_rows(const sw_problem* pr, double* f, double* g, float* key) {
    if (sw_validate_problem(pr) != 0) return SW_ERR_INVALID;
    twin_t P;
    build(&P, pr);
    const int32_t N = pr->num_jobs, T = pr->future_rounds;
    for (int32_t j = 0; j < N; ++j) {
        for (int32_t n = 0; n <= T; ++n) {
            f[(size_t)j * (T + 1) + n] = fval(&P, j, n);
            g[(size_t)j * (T + 1) + n] = sw_g(&P.jc[j], n);
        }
        for (int32_t n = 0; n < T; ++n) key[(size_t)j * T + n] = K_(&P, j, n);
    }
    free(P.jc); free(P.key); free(P.Tj);
    return 0;
}

/* Exposed for tests: objective of given planned-round counts (no packing). */
double twin_eval_counts(const sw_problem* pr, const int32_t* ncount, double* makespan) {
    twin_t P;
    build(&P, pr);
    const int32_t N = pr->num_jobs;
    size_t NN = N > 0 ? (size_t)N : 1;
    double* tmp = (double*)malloc(sizeof(double) * NN);
    double M = 0.0;
    for (int32_t j = 0; j < N; ++j) {
        tmp[j] = fval(&P, j, ncount[j]);
        M = sw_max(M, sw_g(&P.jc[j], ncount[j]));
    }
    double U = sw_detsum(tmp, N);
    if (makespan) *makespan = M;
    free(P.jc); free(P.key); free(P.Tj); free(tmp);
    return U - pr->regularizer * M;
}
