/*
 * sw_p2x_dev.h — the P2 exchange step as a block function (sw_p2x.h;
 * DESIGN.md §3.6), bit-identical to the sequential specification
 * oracle/p2x_twin.c.  Used by the batch kernel (sw_p2x_kernel.hip) and by the
 * sharded engine on its gathered placement (sw_shard.hip).
 *
 * Mapping.  Active jobs are ranked inside their width class by (c desc, job
 * asc) with a bitonic sort (shuffles below stride 64, LDS above), and each
 * class's membership of each round becomes a rank bitset in LDS (one wave
 * ballot per 64-rank word), so the move an edge t → u makes is a few 64-bit
 * and-not / ctz / clz word operations.  Edge costs W[t][u] are built by all
 * threads, one (t, u) pair per thread, once per load size F and afterwards
 * only in the rows and columns of the rounds a cancelled cycle touched (the
 * other entries cannot change).  Bellman–Ford is block-wide: the eight waves
 * relax an eighth of the source rounds each (lane = target round), wave 0
 * combines them, handles the free-capacity node V as a wave-uniform scalar
 * and checks the predecessor graph by pointer doubling (⌈log2(T + 1)⌉
 * shuffles); each load size's runs start from its previous run's distances.  A
 * cycle's moves are applied with LDS atomics.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shockwave_amd.h"
#include "sw_arith.h"
#include "sw_block.h"
#include "sw_device.h"
#include "sw_p2x.h"

/* per-active-job arrays, index a = active jobs in job order (LDS on the
 * on-chip batch path, HBM workspace otherwise) */
struct sw_p2x_arrays {
    int32_t* cw;  /* width                       */
    int32_t* cj;  /* job id                      */
    double* cc;   /* c = p / n                   */
    uint64_t* cm; /* round mask (improved here)  */
};
static_assert(SW_P2X_ARR_BYTES == 2 * sizeof(int32_t) + sizeof(double) + sizeof(uint64_t),
              "SW_P2X_ARR_BYTES (sw_p2x.h) must cover the sw_p2x_arrays layout");

/* The step's set-up, prepared in HBM by several workgroups (the sharded
 * engine's k_p2x_pre*, sw_shard.hip) instead of by the step's one workgroup:
 * the classes (hdr: K, wc[8], M[8], off[9], nw[8], boff[8]), the positions'
 * active indices and c (ord, pc), the rank bitsets B (the layout of LDS
 * below) and, per load size index ki, the first edge-cost matrix (Wb: the
 * cheapest class's cost without δ, SW_P2X_NONE for none; Wk: its class) —
 * what sw_p2x_block would compute, the same values.  The matrices serve the
 * first build of each load size while nothing was cancelled. */
struct sw_p2x_pre {
    const int32_t* hdr;
    const int32_t* ord;
    const double* pc;
    const uint64_t* B;
    const double* Wb;
    const int8_t* Wk;
};
enum { SW_P2X_HDR_K = 0, SW_P2X_HDR_WC = 1, SW_P2X_HDR_M = 9, SW_P2X_HDR_OFF = 17,
       SW_P2X_HDR_NW = 26, SW_P2X_HDR_BOFF = 34, SW_P2X_HDR_A = 42, SW_P2X_HDR_INTS = 48 };

/* fixed LDS part */
struct sw_p2x_lds {
    sw_xchg X;
    int32_t wc[SW_P2X_KMAX], M[SW_P2X_KMAX], off[SW_P2X_KMAX + 1], nw[SW_P2X_KMAX],
        boff[SW_P2X_KMAX];
    int32_t K, len, nrec, pad;
    uint64_t touched; /* rounds the last cancelled cycle moved jobs in or out of */
    uint32_t wmap[8]; /* widths present (256 bits) */
    int32_t room[SW_TMAX];
    int32_t pr[SW_TMAX + 1];
    int32_t cyc[SW_TMAX + 2];
    double delta;
    /* block-wide Bellman–Ford: distances and predecessors (V at index T),
     * each wave's partial minima over its rows, the loop's exit flag */
    double bd[SW_TMAX + 1];
    int32_t bp[SW_TMAX + 1];
    double pv[SW_WAVES][64];
    int8_t pt[SW_WAVES][64];
    int32_t bfdone;
    int32_t fq[SW_P2X_KMAX]; /* F / w_k for the current load size (0: w_k ∤ F) */
    double dw[SW_P2X_KMAX][SW_TMAX + 1]; /* each load size's last Bellman–Ford distances */
};

/* LDS the variable part needs for up to maxA active jobs and T rounds:
 * position order and c by position, then the larger of (rank bitsets, W,
 * Wk, move records) and the rank sort's scratch (16 B per entry of the next
 * power of two) */
__host__ __device__ inline size_t sw_p2x_var_bytes(int maxA, int T) {
    const size_t a = (size_t)(maxA < SW_P2X_AMAX ? maxA : SW_P2X_AMAX);
    const size_t words = (size_t)T * ((a + 63) / 64 + SW_P2X_KMAX);
    size_t np = 1;
    while (np < a) np <<= 1;
    const size_t work = words * 8 + (size_t)T * T * 8 + (((size_t)T * T + 15) & ~(size_t)15) +
                        (size_t)SW_P2X_MAX_MOVES * 4;
    return a * 8 + ((a * 4 + 15) & ~(size_t)15) + (work > 16 * np ? work : 16 * np);
}

static __device__ __forceinline__ int p2x_class(const sw_p2x_lds* L, int32_t w) {
    int k = 0;
    while (k < L->K - 1 && L->wc[k] != w) ++k;
    return k;
}

/* Bellman–Ford of oracle/p2x_twin.c find_cycle, block-wide: each sweep,
 * every wave relaxes ⌈T / 8⌉ consecutive source rounds (lane u = target
 * round u: the smallest d[t] + W[t][u] of its rows and their first t, read
 * against the distances in LDS), then wave 0 combines the eight in round
 * order (strict <: the sequential scan's answer), adds V (a wave-uniform
 * scalar; its minimum by a DPP reduction), publishes the new distances and,
 * after the odd sweeps and the last, checks the predecessor graph for a
 * cycle by pointer doubling: 2^⌈log2(T + 1)⌉ ≥ T + 1 steps from a vertex are
 * still defined exactly when its walk enters a cycle, and the lowest such
 * vertex reaches the same cycle as the twin's walk from it.  Leaves the
 * cycle in L->cyc / L->len (0: none).  All threads call it. */
static __device__ __forceinline__ void p2x_find_cycle(sw_p2x_lds* L, const double* W, int T, int F,
                                                      double* dw, bool warm, uint64_t (&acc)[11]) {
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    (void)acc;
#ifdef SW_STAMPS
    /* stamps accumulate in the caller's registers (acc, sw_p2x_block's) */
    uint64_t bt_ = __builtin_amdgcn_s_memtime();
#define BF_STAMP(k)                                                   \
    do {                                                              \
        const uint64_t now_ = __builtin_amdgcn_s_memtime();           \
        acc[k] += now_ - bt_;                                         \
        bt_ = now_;                                                   \
    } while (0)
#else
#define BF_STAMP(k) \
    do {            \
    } while (0)
#endif
    const bool act = lane < T;
    if (tid <= T) { /* from this load size's last distances when warm (twin: find_cycle) */
        L->bd[tid] = warm ? dw[tid] : 0.0;
        L->bp[tid] = -1;
    }
    if (tid == 0) L->bfdone = 0;
    const bool roomok = wv == 0 && act && L->room[lane] >= F;
    const bool anyroom = __ballot(roomok) != 0; /* else V has no in-edge: it never changes */
    const int nq = (T + SW_WAVES - 1) / SW_WAVES; /* rows per relaxing wave */
    int ndbl = 0; /* pointer doublings: 2^ndbl ≥ T + 1 steps */
    while ((1 << ndbl) < T + 1) ++ndbl;
    __syncthreads();
    for (int it = 0; it <= T; ++it) {
#ifdef SW_STAMPS
        acc[7] += 1;
#endif
        BF_STAMP(10);
        {
            /* W[t][t] and missing edges are SW_P2X_NONE and every distance is
             * ≤ 0, so they never win: no per-edge tests */
            const int ul = act ? lane : 0;
            const int t0 = wv * nq, t1 = min(T, t0 + nq);
            double cb = SW_P2X_NONE;
            int ct = 0;
            for (int t = t0; t < t1; ++t) {
                const double v = L->bd[t] + W[t * T + ul];
                const bool take = v < cb;
                cb = take ? v : cb;
                ct = take ? t : ct;
            }
            L->pv[wv][lane] = cb;
            L->pt[wv][lane] = (int8_t)ct;
        }
        __syncthreads();
        BF_STAMP(9);
        if (wv == 0) {
            /* the sweep's serial part: the other waves wait at the barrier,
             * so issue it ahead of the CU's other workgroups */
            __builtin_amdgcn_s_setprio(3);
            double d = act ? L->bd[lane] : 0.0;
            int pr = act ? L->bp[lane] : -1;
            const double dV = L->bd[T];
            int prV = L->bp[T];
            double cb = L->pv[0][lane];
            int ct = L->pt[0][lane];
#pragma unroll
            for (int q = 1; q < SW_WAVES; ++q) {
                const double v = L->pv[q][lane];
                const bool take = q * nq < T && v < cb;
                cb = take ? v : cb;
                ct = take ? L->pt[q][lane] : ct;
            }
            double best = d;
            int bpr = pr;
            if (cb < best) {
                best = cb;
                bpr = ct;
            }
            if (act && dV < best) {
                best = dV;
                bpr = T;
            }
            /* V: the smallest d over rounds with F free GPUs, lowest round on ties */
            bool vbetter = false;
            double m = dV;
            uint64_t at = 0;
            if (anyroom) {
                m = wave_min_f64(roomok ? d : SW_P2X_NONE);
                at = __ballot(roomok && d == m);
                vbetter = m < dV;
            }
            const bool changed = __ballot(act && best < d) != 0 || vbetter;
            int done = 0;
            if (!changed) {
                done = 1;
                if (lane == 0) L->len = 0;
            } else {
                d = best;
                pr = bpr;
                if (vbetter) prV = (int)__builtin_ctzll(at);
                if (act) {
                    L->bd[lane] = d;
                    L->bp[lane] = pr;
                }
                if (lane == 0 && vbetter) {
                    L->bd[T] = m;
                    L->bp[T] = prV;
                }
                /* after the odd sweeps and the last (from d = 0, after the
                 * first every predecessor is a later round: no cycle can
                 * exist yet; from warm distances also after the first) */
                if ((it & 1) || it == T || (warm && it == 0)) {
                    int y = act ? pr : -1, yV = prV;
#pragma unroll
                    for (int s2 = 0; s2 < 7; ++s2) { /* 2^7 > SW_TMAX */
                        if (s2 >= ndbl) break;
                        const int g = __shfl(y, (y >= 0 && y < T) ? y : 0, 64);
                        /* yV (V's walk) is wave-uniform: a lane read, not a shuffle */
                        const int gV = (yV >= 0 && yV < T) ? __builtin_amdgcn_readlane(y, yV)
                                                           : (yV == T ? yV : -1);
                        y = y < 0 ? -1 : (y == T ? yV : g);
                        yV = gV;
                    }
                    const uint64_t cbits = __ballot(act && y >= 0);
                    if (cbits) {
                        done = 1;
                        const int y0 = __builtin_amdgcn_readlane(y, (int)__builtin_ctzll(cbits));
                        if (act) L->pr[lane] = pr;
                        if (lane == 0) L->pr[T] = prV;
                        wave_sync();
                        if (lane == 0) {
                            int lo = y0;
                            for (int v = L->pr[y0]; v != y0; v = L->pr[v]) lo = v < lo ? v : lo;
                            int len = 0, v = lo;
                            do {
                                L->cyc[len++] = v;
                                v = L->pr[v];
                            } while (v != lo && len <= T + 1);
                            double cost = 0.0;
                            for (int i = 0; i < len; ++i) {
                                const int u = L->cyc[i], t = L->pr[u];
                                if (u < T && t < T) cost = cost + W[t * T + u];
                            }
                            L->len = cost < 0.0 ? len : 0;
                        }
                    }
                }
                if (!done && it == T && lane == 0) L->len = 0;
            }
            if (lane == 0) L->bfdone = done;
            __builtin_amdgcn_s_setprio(0);
        }
        __syncthreads();
        if (L->bfdone) break;
    }
    if (tid <= T) dw[tid] = L->bd[tid]; /* read by this thread's next init only */
#undef BF_STAMP
}

/* sw_p2x_cost (sw_p2x.h) for classes of at most 256 jobs (≤ 4 words) and
 * q ≤ 4, for one direction (LO: u < t, ascending ranks; else descending):
 * the and-not words are loaded in scan order (the word count nw and q are
 * uniform over the wave, so the loads and the pick loop have no per-lane
 * selects), and each pick takes the first set bit (lowest, or highest) of
 * the first non-empty word; c is summed in selection order from 0.0, as the
 * twin does.  Other cases: sw_p2x_cost. */
template <bool LO, int NW>
static __device__ __forceinline__ double p2x_cost_nw(const uint64_t* Bt, const uint64_t* Bu, int nw, int ws,
                                                     int q, int t, int u, const double* c) {
    /* NW words of code for nw ≤ NW actual words (NW = 4 serves nw = 3 with
     * a zero word): y[s] is the s-th word in scan order */
    uint64_t y[NW];
#pragma unroll
    for (int s = 0; s < NW; ++s) {
        const int i = LO ? s : nw - 1 - s;
        y[s] = s < nw ? (Bt[i * ws] & ~Bu[i * ws]) : 0ull;
    }
    int avail = 0;
#pragma unroll
    for (int s = 0; s < NW; ++s) avail += __popcll(y[s]);
    if (avail < q) return SW_P2X_NONE;
    double sum = 0.0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        if (g >= q) break;
        /* the first non-empty word in scan order */
        int sidx = NW - 1;
        uint64_t ys = y[NW - 1];
#pragma unroll
        for (int s2 = NW - 2; s2 >= 0; --s2) {
            sidx = y[s2] ? s2 : sidx;
            ys = y[s2] ? y[s2] : ys;
        }
        const int b = LO ? __builtin_ctzll(ys) : 63 - __builtin_clzll(ys);
        const uint64_t cl = LO ? (ys & (ys - 1)) : (ys & ~(1ull << (b & 63)));
#pragma unroll
        for (int s2 = 0; s2 < NW; ++s2) y[s2] = s2 == sidx ? cl : y[s2];
        sum = sum + c[64 * (LO ? sidx : nw - 1 - sidx) + (b & 63)];
    }
    return sum * (double)(u - t);
}

/* sw_p2x_cost (sw_p2x.h) for classes of at most 256 jobs (≤ 4 words) and
 * q ≤ 4, for one direction (LO: u < t, ascending ranks; else descending),
 * specialised on the word count nw (1, 2, or up to 4; uniform per class, like
 * q): the and-not
 * words are loaded in scan order, each pick takes the first set bit (lowest,
 * or highest) of the first non-empty word, and c is summed in selection order
 * from 0.0, as the twin does.  Other cases: sw_p2x_cost. */
template <bool LO>
static __device__ __forceinline__ double p2x_cost_dir(const uint64_t* Bt, const uint64_t* Bu, int nw, int ws,
                                                      int q, int t, int u, const double* c) {
    if (q > 4 || nw > 4) return sw_p2x_cost(Bt, Bu, nw, ws, q, t, u, c);
    if (nw == 1) return p2x_cost_nw<LO, 1>(Bt, Bu, nw, ws, q, t, u, c);
    if (nw == 2) return p2x_cost_nw<LO, 2>(Bt, Bu, nw, ws, q, t, u, c);
    return p2x_cost_nw<LO, 4>(Bt, Bu, nw, ws, q, t, u, c);
}

/* W entries for load size F: every entry (all = true) or those in a row or
 * column of L->touched.  L->fq[k] = F / w_k for the classes that can carry F
 * (w_k | F), 0 for the others: set once per load size, so the per-entry loop
 * has no integer divisions.  The T(T − 1) off-diagonal pairs are walked as
 * two triangles, all u < t first, so every wave but one has a single move
 * direction (one code path of p2x_cost_dir); pair i of a triangle is (a, b),
 * b < a, with a(a − 1)/2 ≤ i < a(a + 1)/2. */
/* pair e of the two triangles (u < t first) */
static __device__ __forceinline__ void p2x_pair(int e, int P, int& t, int& u) {
    const bool lo = e < P;
    const int i = lo ? e : e - P;
    int a = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)i)) * 0.5f);
    if (a * (a - 1) / 2 > i) --a;
    if ((a + 1) * a / 2 <= i) ++a;
    const int b = i - a * (a - 1) / 2;
    t = lo ? a : b;
    u = lo ? b : a;
}

/* The cheapest class's cost of the edge t → u (W, Wk entry). */
static __device__ __forceinline__ void p2x_edge(const sw_p2x_lds* L, const uint64_t* B, const double* pc,
                                                double* W, int8_t* Wk, int T, double delta, int K, int t,
                                                int u) {
    const bool lo = u < t;
    double best = SW_P2X_NONE;
    int bk = -1;
#pragma unroll 1
    for (int k = 0; k < K; ++k) {
        const int q = L->fq[k];
        if (q == 0) continue;
        const int nw = L->nw[k];
        const uint64_t* Bk = B + L->boff[k]; /* word-major: word w of round t at w·T + t */
        const double cost = lo ? p2x_cost_dir<true>(Bk + t, Bk + u, nw, T, q, t, u, pc + L->off[k])
                               : p2x_cost_dir<false>(Bk + t, Bk + u, nw, T, q, t, u, pc + L->off[k]);
        if (cost < best) {
            best = cost;
            bk = k;
        }
    }
    W[t * T + u] = bk >= 0 ? best + delta : SW_P2X_NONE;
    Wk[t * T + u] = (int8_t)bk;
}

/* Touched pairs (a, b), a > b, a or b in S, in rows < a: all pairs of the
 * first a rows less those with neither round in S (a ≤ 63). */
static __device__ __forceinline__ int p2x_rows_before(uint64_t S, int a) {
    const int m = a - __popcll(S & ((1ull << a) - 1ull));
    return a * (a - 1) / 2 - m * (m - 1) / 2;
}

/* After a cancel (all = false) only the pairs in a row or column of the
 * touched rounds S change — 2·n·(T − 1) − n·(n − 1) of the T(T − 1) for n
 * touched rounds, ≈ 170 of 870 at T = 30 after a 3-round cycle.  Walking
 * all pairs left most lanes idle and the busy ones with two pairs each; the
 * touched pairs are dealt one per thread instead, in pair order (the u < t
 * triangle first, so the waves keep one move direction).  Thread j finds
 * its pair without a list: the touched pairs of the lower triangle are
 * counted row by row in closed form (p2x_rows_before), so a binary search
 * over the rows gives the row a, and the column is the r-th round of the
 * row's touched columns (all of them when a is in S, else the rounds of S
 * below a); the upper triangle is the transpose, in the same order.  (A
 * block-scanned list in LDS measured the same, but its loop spilled 8 B per
 * lane more in the fused pack kernel, and one wave listing them by ballots
 * was slower on the C5 sweep.) */
template <int NT>
static __device__ __forceinline__ void p2x_build_w(const sw_p2x_lds* L, const uint64_t* B,
                                                   const double* pc, double* W, int8_t* Wk, int T, double delta,
                                                   bool all) {
    const uint64_t tm = L->touched;
    const int K = L->K;
    const int P = T * (T - 1) / 2;
    if (all)
        for (int t = threadIdx.x; t < T; t += NT) {
            W[t * T + t] = SW_P2X_NONE;
            Wk[t * T + t] = (int8_t)-1;
        }
    if (!all) {
        const uint64_t S = T < 64 ? tm & ((1ull << T) - 1ull) : tm;
        const int nt = __popcll(S);
        const int half = nt * (T - 1) - nt * (nt - 1) / 2;
        for (int j = threadIdx.x; j < 2 * half; j += NT) {
            const bool lo = j < half;
            const int i = lo ? j : j - half;
            int a0 = 1, a1 = T - 1;
            while (a0 < a1) {
                const int mid = (a0 + a1 + 1) >> 1;
                if (p2x_rows_before(S, mid) <= i) a0 = mid;
                else a1 = mid - 1;
            }
            const int r = i - p2x_rows_before(S, a0);
            int b = r;
            if (!((S >> a0) & 1ull)) {
                uint64_t m = S & ((1ull << a0) - 1ull);
                for (int k = 0; k < r; ++k) m &= m - 1ull;
                b = __ffsll((long long)m) - 1;
            }
            p2x_edge(L, B, pc, W, Wk, T, delta, K, lo ? a0 : b, lo ? b : a0);
        }
        return;
    }
    for (int e = threadIdx.x; e < 2 * P; e += NT) {
        int t, u;
        p2x_pair(e, P, t, u);
        p2x_edge(L, B, pc, W, Wk, T, delta, K, t, u);
    }
}

/* diagnostic builds (SW_STAMPS): thread 0's cycles, accumulated in registers
 * (sp_a_) and added to sp[k] on return — a global read-modify-write per stamp
 * would add a memory round trip to each phase it times: 0 classes, 1 ranks,
 * 2 bitsets and δ, 3 edge builds, 4 Bellman–Ford, 5 selecting a cycle's
 * moves, 6 applying them; counts: 7 Bellman–Ford sweeps, 8 edge builds;
 * inside Bellman–Ford: 9 relaxations, 10 predecessor walks */
#ifdef SW_STAMPS
#define P2X_STAMP(k)                                                 \
    do {                                                             \
        const uint64_t now_ = __builtin_amdgcn_s_memtime();          \
        sp_a_[k] += now_ - sp_t_;                                    \
        sp_t_ = now_;                                                \
    } while (0)
#else
#define P2X_STAMP(k) \
    do {             \
    } while (0)
#endif

/* Bitonic sort of np = E·NT (class/key, job << 32 | a) pairs, E per thread
 * in registers (thread tid holds entries tid·E … tid·E + E − 1): strides
 * below E inside the thread, below 64·E by shuffles, larger ones through
 * the LDS exchange xs (16·np bytes).  Entries past A are (~0, ~0). */
template <int NT, int EMAX>
static __device__ __forceinline__ void p2x_sort_regs(uint64_t (&hi)[EMAX], uint64_t (&lo)[EMAX], int E,
                                                     int np, uint64_t* xs) {
    const int tid = threadIdx.x;
    for (int kk = 2; kk <= np; kk <<= 1) {
        for (int jj = kk >> 1; jj > 0; jj >>= 1) {
            if (jj < E) { /* both entries in this thread */
#pragma unroll
                for (int e = 0; e < EMAX; ++e) {
                    const int f = e ^ jj;
                    if (e < E && f > e) {
                        const int i = tid * E + e;
                        const bool up = (i & kk) == 0;
                        uint64_t ah = hi[e], al = lo[e], bh = 0, bl = 0;
#pragma unroll
                        for (int g = 0; g < EMAX; ++g)
                            if (g == f) { bh = hi[g]; bl = lo[g]; }
                        const bool gt = ah > bh || (ah == bh && al > bl);
                        if (up == gt) { /* swap */
                            hi[e] = bh; lo[e] = bl;
#pragma unroll
                            for (int g = 0; g < EMAX; ++g)
                                if (g == f) { hi[g] = ah; lo[g] = al; }
                        }
                    }
                }
            } else {
                uint64_t ph[EMAX], pl[EMAX];
                const int dj = jj / E; /* partner thread tid ^ dj, same slot */
                if (dj < 64) {
#pragma unroll
                    for (int e = 0; e < EMAX; ++e) {
                        ph[e] = __shfl_xor(hi[e], dj, 64);
                        pl[e] = __shfl_xor(lo[e], dj, 64);
                    }
                } else {
                    if (tid * E < np)
                        for (int e = 0; e < E; ++e) {
                            xs[tid * E + e] = hi[e];
                            xs[np + tid * E + e] = lo[e];
                        }
                    __syncthreads();
                    const int pt = tid ^ dj;
                    if (tid * E < np)
                        for (int e = 0; e < E; ++e) {
                            ph[e] = xs[pt * E + e];
                            pl[e] = xs[np + pt * E + e];
                        }
                    __syncthreads();
                }
                const bool lower = (tid & dj) == 0;
#pragma unroll
                for (int e = 0; e < EMAX; ++e) {
                    if (e >= E) continue;
                    const int i = tid * E + e;
                    const bool up = (i & kk) == 0;
                    const bool gt = hi[e] > ph[e] || (hi[e] == ph[e] && lo[e] > pl[e]);
                    if ((lower == up) ? gt : !gt) {
                        hi[e] = ph[e];
                        lo[e] = pl[e];
                    }
                }
            }
        }
    }
}

/* EMAX: entries per thread the rank sort may hold in registers (the sharded
 * engine's single-workgroup step, up to SW_P2X_AMAX positions, uses 8; the
 * batch kernel, capped at 64 VGPRs, 1 and an LDS network above 512) */
template <int NW, int EMAX = 1>
__device__ __forceinline__ int sw_p2x_block(sw_blk_t<NW>& blk, sw_p2x_lds* L, unsigned char* var,
                                            const sw_p2x_arrays& X, int A, int T, int G,
                                            uint64_t* sp = nullptr, const sw_p2x_pre* pre = nullptr) {
    constexpr int NT = NW * 64;
    const int tid = threadIdx.x;
    (void)sp;
    uint64_t sp_a_[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#ifdef SW_STAMPS
    uint64_t sp_t_ = __builtin_amdgcn_s_memtime();
#endif
    if (A <= 0 || T < 2 || A > SW_P2X_AMAX) return 0;
    if (pre && pre->hdr[SW_P2X_HDR_K] < 0) return 0; /* more than SW_P2X_KMAX classes */
    if (pre) { /* the prepared set-up: classes, positions, bitsets from HBM */
        if (tid < SW_P2X_KMAX) {
            L->wc[tid] = pre->hdr[SW_P2X_HDR_WC + tid];
            L->M[tid] = pre->hdr[SW_P2X_HDR_M + tid];
            L->nw[tid] = pre->hdr[SW_P2X_HDR_NW + tid];
            L->boff[tid] = pre->hdr[SW_P2X_HDR_BOFF + tid];
        }
        if (tid <= SW_P2X_KMAX) L->off[tid] = pre->hdr[SW_P2X_HDR_OFF + tid];
        if (tid == 0) L->K = pre->hdr[SW_P2X_HDR_K];
        __syncthreads();
    }
    if (!pre) {
    /* ---- width classes (ascending) ---- */
    if (tid < 8) L->wmap[tid] = 0u;
    __syncthreads();
    for (int a = tid; a < A; a += NT) atomicOr(&L->wmap[X.cw[a] >> 5], 1u << (X.cw[a] & 31));
    __syncthreads();
    if (tid == 0) {
        int K = 0;
        for (int i = 0; i < 8; ++i) K += __builtin_popcount(L->wmap[i]);
        if (K > SW_P2X_KMAX) {
            L->K = -1;
        } else {
            K = 0;
            for (int i = 0; i < 8; ++i)
                for (uint32_t b = L->wmap[i]; b; b &= b - 1) L->wc[K++] = 32 * i + __builtin_ctz(b);
            L->K = K;
            for (int k = 0; k < K; ++k) L->M[k] = 0;
        }
    }
    __syncthreads();
    if (L->K < 0) return 0;
    for (int a = tid; a < A; a += NT) atomicAdd(&L->M[p2x_class(L, X.cw[a])], 1);
    __syncthreads();
    if (tid == 0) {
        const int K = L->K;
        int o = 0, b = 0;
        for (int k = 0; k < K; ++k) {
            L->off[k] = o;
            L->nw[k] = (L->M[k] + 63) / 64;
            L->boff[k] = b;
            o += L->M[k];
            b += L->nw[k] * T;
        }
        L->off[K] = o;
    }
    } /* !pre */
    const int K = L->K;
    P2X_STAMP(0);
    /* LDS carve-up of var */
    double* pc = reinterpret_cast<double*>(var);                      /* c by position        */
    int32_t* ord = reinterpret_cast<int32_t*>(var + (size_t)A * 8);  /* position → a         */
    unsigned char* vb = var + (size_t)A * 8 + (((size_t)A * 4 + 15) & ~(size_t)15);
    __syncthreads();
    const int nwords = L->boff[K - 1] + L->nw[K - 1] * T;
    uint64_t* B = reinterpret_cast<uint64_t*>(vb);
    double* W = reinterpret_cast<double*>(vb + (size_t)nwords * 8);
    int8_t* Wk = reinterpret_cast<int8_t*>(W + T * T);
    int32_t* rec = reinterpret_cast<int32_t*>(reinterpret_cast<unsigned char*>(Wk) + ((T * T + 15) & ~15));
    /* ---- positions: (class asc, sw_p2x_ckey(c) desc, job asc) by a bitonic
     *      sort in LDS over the next power of two (the bitset / W area is
     *      free until the first build) ---- */
    if (pre) {
        for (int p = tid; p < A; p += NT) {
            ord[p] = pre->ord[p];
            pc[p] = pre->pc[p];
        }
        for (int i = tid; i < nwords; i += NT) B[i] = pre->B[i];
        __syncthreads();
    } else if (A <= NT) {
        /* one position per thread: (class, key) and (job << 32 | a), a
         * bitonic network over the next power of two np with shuffles for
         * strides < 64 and an LDS exchange above (16·np bytes, what the
         * LDS sort below uses; jobs are distinct, so the order is the same) */
        int np = 1;
        while (np < A) np <<= 1;
        uint64_t hi = ~0ull, lo = ~0ull;
        if (tid < A) {
            const uint64_t ck = sw_p2x_ckey(X.cc[tid]);
            hi = ((uint64_t)p2x_class(L, X.cw[tid]) << 61) | (~ck & ((1ull << 61) - 1));
            lo = ((uint64_t)(uint32_t)X.cj[tid] << 32) | (uint32_t)tid;
        }
        uint64_t* xs = reinterpret_cast<uint64_t*>(vb); /* [hi, lo][np] */
        for (int kk = 2; kk <= np; kk <<= 1) {
            for (int jj = kk >> 1; jj > 0; jj >>= 1) {
                uint64_t ph = ~0ull, pl = ~0ull;
                if (jj >= 64) {
                    if (tid < np) {
                        xs[tid] = hi;
                        xs[np + tid] = lo;
                    }
                    __syncthreads();
                    if (tid < np) {
                        ph = xs[tid ^ jj];
                        pl = xs[np + (tid ^ jj)];
                    }
                    __syncthreads();
                } else {
                    ph = __shfl_xor(hi, jj, 64);
                    pl = __shfl_xor(lo, jj, 64);
                }
                const bool up = (tid & kk) == 0, lower = (tid & jj) == 0;
                const bool gt = hi > ph || (hi == ph && lo > pl);
                if ((lower == up) ? gt : !gt) {
                    hi = ph;
                    lo = pl;
                }
            }
        }
        if (tid < A) {
            const int a = (int)(uint32_t)lo;
            ord[tid] = a;
            pc[tid] = X.cc[a];
        }
        __syncthreads(); /* the sort scratch is read before the bitsets overwrite it */
    } else if (EMAX > 1 && A <= EMAX * NT) {
        int np = 1;
        while (np < A) np <<= 1;
        const int E = np / NT; /* A > NT: np ≥ 2·NT */
        uint64_t hi[EMAX], lo[EMAX];
#pragma unroll
        for (int e = 0; e < EMAX; ++e) {
            const int i = tid * E + e;
            hi[e] = ~0ull;
            lo[e] = ~0ull;
            if (e < E && i < A) {
                const uint64_t ck = sw_p2x_ckey(X.cc[i]);
                hi[e] = ((uint64_t)p2x_class(L, X.cw[i]) << 61) | (~ck & ((1ull << 61) - 1));
                lo[e] = ((uint64_t)(uint32_t)X.cj[i] << 32) | (uint32_t)i;
            }
        }
        p2x_sort_regs<NT, EMAX>(hi, lo, E, np, reinterpret_cast<uint64_t*>(vb));
#pragma unroll
        for (int e = 0; e < EMAX; ++e) {
            const int p = tid * E + e;
            if (e < E && p < A) {
                const int a = (int)(uint32_t)lo[e];
                ord[p] = a;
                pc[p] = X.cc[a];
            }
        }
        __syncthreads(); /* the sort scratch is read before the bitsets overwrite it */
    } else {
        int np = 1;
        while (np < A) np <<= 1;
        uint64_t* k1 = reinterpret_cast<uint64_t*>(vb);
        uint32_t* k2 = reinterpret_cast<uint32_t*>(k1 + np); /* job */
        uint32_t* ka = k2 + np;                              /* a   */
        for (int i = tid; i < np; i += NT) {
            if (i < A) {
                const uint64_t ck = sw_p2x_ckey(X.cc[i]);
                k1[i] = ((uint64_t)p2x_class(L, X.cw[i]) << 61) | (~ck & ((1ull << 61) - 1));
                k2[i] = (uint32_t)X.cj[i];
                ka[i] = (uint32_t)i;
            } else {
                k1[i] = ~0ull;
                k2[i] = 0xFFFFFFFFu;
                ka[i] = 0u;
            }
        }
        __syncthreads();
        /* strides below a wave's chunk (np / NW entries, aligned) pair entries
         * of the same chunk: that wave runs those stages alone, with wave-level
         * ordering instead of block barriers */
        const int chunk = np / NW;
        const int lane = lane_id(), wv = wave_id();
        for (int k = 2; k <= np; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                const bool local = j < chunk;
                const int x0 = local ? lane : tid, xs = local ? 64 : NT;
                const int nx = local ? (chunk >> 1) : (np >> 1), base = local ? wv * chunk : 0;
                for (int x = x0; x < nx; x += xs) {
                    const int i = base + 2 * x - (x & (j - 1)), l = i + j;
                    const uint64_t a1 = k1[i], b1 = k1[l];
                    const uint32_t a2 = k2[i], b2 = k2[l];
                    const bool gt = a1 > b1 || (a1 == b1 && a2 > b2);
                    if (((i & k) == 0) == gt) { /* ascending blocks where bit k of i is clear */
                        k1[i] = b1; k1[l] = a1;
                        k2[i] = b2; k2[l] = a2;
                        const uint32_t t = ka[i]; ka[i] = ka[l]; ka[l] = t;
                    }
                }
                /* the next stage may pair across chunks: a block barrier
                 * unless it stays inside this wave's chunk */
                const int nj = j > 1 ? (j >> 1) : k; /* the next stage's stride (k doubles) */
                const bool next_local = (j > 1 || (k << 1) <= np) && nj < chunk;
                if (local && next_local) wave_sync();
                else __syncthreads();
            }
        }
        for (int p = tid; p < A; p += NT) {
            const int a = (int)ka[p];
            ord[p] = a;
            pc[p] = X.cc[a];
        }
        __syncthreads(); /* the sort scratch is read before the bitsets clear it */
    }
    P2X_STAMP(1);
    /* ---- rank bitsets, free capacity, δ ----
     * One wave per 64-rank word slot (class k, word w): lane r loads the
     * mask of rank 64·w + r and each round's word is a ballot, written once
     * (no clearing, no atomics: the per-position LDS atomics of 64 ranks into
     * one word, and of every position into T room counters, serialised). */
    {
        const int lane = lane_id(), wv = wave_id();
        int nslot = 0;
        for (int k = 0; k < K; ++k) nslot += L->nw[k];
        if (pre) nslot = 0; /* the bitsets came prepared */
        for (int sl = wv; sl < nslot; sl += NW) {
            int k = 0, w = sl;
            while (w >= L->nw[k]) w -= L->nw[k++];
            const int r = 64 * w + lane;
            const uint64_t m = r < L->M[k] ? X.cm[ord[L->off[k] + r]] : 0ull;
            uint64_t* Bk = B + L->boff[k] + (size_t)w * T;
            for (int t = 0; t < T; ++t) {
                const uint64_t word = __ballot((m >> t) & 1ull);
                if (lane == 0) Bk[t] = word;
            }
        }
        __syncthreads();
        if (tid < T) { /* G minus the round's width: Σ_k w_k · members of class k in t */
            int32_t used = 0;
            for (int k = 0; k < K; ++k) {
                const uint64_t* Bk = B + L->boff[k] + tid;
                int32_t c = 0;
                for (int w = 0; w < L->nw[k]; ++w) c += __popcll(Bk[w * T]);
                used += c * L->wc[k];
            }
            L->room[tid] = G - used;
        }
    }
    {
        /* sw_detsum over positions: lane l sums [l·q, (l+1)·q) left to right */
        const int q = (A + SW_DET_LANES - 1) / SW_DET_LANES;
        static_assert(NT == SW_DET_LANES, "one thread per deterministic-sum lane");
        double acc = 0.0;
        for (int p = tid * q; p < A && p < (tid + 1) * q; ++p) {
            int64_t S = 0;
            for (uint64_t x = X.cm[ord[p]]; x; x &= x - 1) S += __builtin_ctzll(x);
            acc = acc + pc[p] * (double)S;
        }
        const double P0 = blk.detsum(acc); /* its barrier publishes B, room */
        if (tid == 0) L->delta = sw_p2x_delta(P0, T, A);
    }
    __syncthreads();
    const double delta = L->delta;
    P2X_STAMP(2);
    /* ---- cancelling ---- */
    int ncancel = 0;
    /* cert[k]: the cancel count when load size k last had no cycle — while
     * nothing was cancelled since, its graph is unchanged and a repeat
     * Bellman–Ford would find none again, so the repeat pass skips it (the
     * specification's result, without the work) */
    int cert[SW_P2X_KMAX];
#pragma unroll
    for (int k = 0; k < SW_P2X_KMAX; ++k) cert[k] = -1;
    uint32_t havem = 0; /* load sizes with distances in L->dw (warm starts) */
    for (bool changed = true; changed && ncancel < SW_P2X_MAX_CANCEL;) {
        changed = false;
        for (int ki = 0; ki < K && ncancel < SW_P2X_MAX_CANCEL; ++ki) {
            const int F = L->wc[ki];
            int certk = -1;
#pragma unroll
            for (int k = 0; k < SW_P2X_KMAX; ++k) certk = k == ki ? cert[k] : certk;
            if (certk == ncancel) continue; /* uniform */
            if (tid < SW_P2X_KMAX) {
                const int wk = tid < K ? L->wc[tid] : 0;
                L->fq[tid] = (wk > 0 && wk <= F && F % wk == 0 && F / wk <= SW_P2X_QMAX) ? F / wk : 0;
            }
            __syncthreads();
            bool all = true;
            while (ncancel < SW_P2X_MAX_CANCEL) {
                if (pre && all && ncancel == 0) { /* the prepared first build of this load size */
                    const double* Wb = pre->Wb + (size_t)ki * T * T;
                    const int8_t* Wkb = pre->Wk + (size_t)ki * T * T;
                    for (int e = tid; e < T * T; e += NT) {
                        const double b = Wb[e];
                        W[e] = b < SW_P2X_NONE ? b + delta : SW_P2X_NONE;
                        Wk[e] = Wkb[e];
                    }
                } else {
                    p2x_build_w<NT>(L, B, pc, W, Wk, T, delta, all);
                }
                __syncthreads();
                P2X_STAMP(3);
                sp_a_[8] += 1;
                p2x_find_cycle(L, W, T, F, L->dw[ki], ((havem >> ki) & 1u) != 0, sp_a_);
                havem |= 1u << ki;
                P2X_STAMP(4);
                const int len = L->len;
                if (len == 0) {
#pragma unroll
                    for (int k = 0; k < SW_P2X_KMAX; ++k) cert[k] = k == ki ? ncancel : cert[k];
                    break;
                }
                /* the cycle's moves, all selected before any is applied: wave 0,
                 * one lane per edge (edge i: pred(cyc[i]) → cyc[i]) */
                if (wave_id() == 0) {
                    const int lane = lane_id();
                    int moves = 0;
                    uint64_t tm = 0;
                    for (int b0 = 0; b0 < len; b0 += 64) {
                        const int i = b0 + lane;
                        const int u = i < len ? L->cyc[i] : T, t = i < len ? L->cyc[(i + 1) % len] : T;
                        const bool real = u < T && t < T;
                        const int q = real ? F / L->wc[Wk[t * T + u]] : 0;
                        moves += wave_sum_i32(q);
                    }
                    int n0 = 0;
                    for (int b0 = 0; b0 < len; b0 += 64) {
                        const int i = b0 + lane;
                        const int u = i < len ? L->cyc[i] : T, t = i < len ? L->cyc[(i + 1) % len] : T;
                        const bool real = u < T && t < T;
                        const int k = real ? Wk[t * T + u] : 0;
                        const int q = real ? F / L->wc[k] : 0;
                        const int incl = wave_incscan_i32(q);
                        if (real) tm |= (1ull << t) | (1ull << u);
                        if (real && moves <= SW_P2X_MAX_MOVES) {
                            const uint64_t* Bt = B + L->boff[k] + t;
                            const uint64_t* Bu = B + L->boff[k] + u;
                            int r = sw_p2x_start(Bt, Bu, L->nw[k], T, q, u < t);
                            int n = n0 + incl - q;
                            for (int g = 0; g < q; ++g) {
                                rec[n++] = (k << 29) | (t << 23) | (u << 17) | r;
                                if (g + 1 < q) r = sw_p2x_next(Bt, Bu, L->nw[k], T, r + 1);
                            }
                        }
                        n0 += __shfl(incl, 63, 64);
                    }
                    /* every lane's touched rounds */
                    for (int o = 32; o >= 1; o >>= 1) {
                        const uint64_t v = (uint64_t)__shfl_xor((long long)tm, o, 64);
                        tm |= v;
                    }
                    if (lane == 0) {
                        L->nrec = moves <= SW_P2X_MAX_MOVES ? n0 : -1;
                        L->touched = tm;
                    }
                }
                __syncthreads();
                P2X_STAMP(5);
                const int nrec = L->nrec;
                if (nrec < 0) break;
                for (int i = tid; i < nrec; i += NT) {
                    const int32_t v = rec[i];
                    const int k = (v >> 29) & 7, t = (v >> 23) & 63, u = (v >> 17) & 63, r = v & 0x1FFFF;
                    uint64_t* Bk = B + L->boff[k];
                    const uint64_t bit = 1ull << (r & 63);
                    atomicAnd((unsigned long long*)&Bk[(r >> 6) * T + t], ~bit);
                    atomicOr((unsigned long long*)&Bk[(r >> 6) * T + u], bit);
                    atomicXor((unsigned long long*)&X.cm[ord[L->off[k] + r]], (1ull << t) | (1ull << u));
                    atomicAdd(&L->room[t], L->wc[k]);
                    atomicAdd(&L->room[u], -L->wc[k]);
                }
                __syncthreads();
                P2X_STAMP(6);
                ++ncancel;
                changed = true;
                all = false;
            }
        }
    }
#ifdef SW_STAMPS
    if (threadIdx.x == 0 && sp)
        for (int k = 0; k < 11; ++k) sp[k] += sp_a_[k];
#endif
    return ncancel;
}
