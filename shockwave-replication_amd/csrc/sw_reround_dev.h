/*
 * sw_reround_dev.h — the per-round exact re-optimisation of sw_reround.h as a
 * block function (one workgroup of SW_BLOCK threads), bit-identical to the
 * sequential specification oracle/plan_twin.c twin_reround_arrays.  Used by
 * the plan kernel (sw_kernels.hip, on-chip and workspace instances) and by
 * the sharded engine on its gathered plan (sw_shard.hip).
 *
 * Mapping.  Thread t owns jobs [t·q, (t+1)·q), q = ⌈N/SW_BLOCK⌉ — the lanes
 * of sw_detsum — so every set value J(S) is one detsum_max reduction.  The
 * per-job values v, h0, h1 of a round live with the owning thread (registers
 * on chip, a workspace otherwise).  The knapsack runs item by item in job
 * order with the capacities spread over the threads: each step reads row
 * dp[·] and writes dp'[·] (two rows, swapped), and the take bits of one step
 * are wave ballots — a wave's 64 lanes hold 64 consecutive capacities, i.e.
 * exactly one 64-bit word — stored by lane 0.  Items are compacted in job
 * order by a block scan, each with its width and value, so a step reads one
 * LDS word pair; thread 0 walks the take bits back.  Every decision (the
 * next level, the accept test) is a block reduction, so control flow is
 * uniform.
 *
 * Env (the caller's view of one instance) provides
 *   N, T, G, k, blk                         sizes, regularizer, block reductions
 *   for_jobs(f(j, s))                       this thread's jobs (s: slot)
 *   jc(j) → sw_jobc, f(c, n), tj(j)         constants of any job, f, schedulable
 *   y(j) (u64&), cnt(j), add_cnt(j, d)      the plan's masks and counts
 *   V/H0/H1(j, s) (double&)                 per-job values of the round
 *   S, Sb (uint8_t*, per job), items (u32: the job index), iv (double),
 *   dpA, dpB (SW_RR_CAPMAX + 1 doubles), bits (SW_RR_WORDS words).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sw_arith.h"
#include "sw_block.h"
#include "sw_reround.h"

/* J(S) = detsum(S·v) − k·max(S ? h1 : h0); U = the detsum part */
template <class Env>
__device__ __forceinline__ double sw_rr_value(Env& e, double& U) {
    double u = 0.0, m = 0.0;
    e.for_jobs([&](int j, int s) {
        const bool in = e.S[j] != 0;
        u = u + (in ? e.V(j, s) : 0.0);
        const double h = in ? e.H1(j, s) : e.H0(j, s);
        m = h > m ? h : m;
    });
    double M;
    e.blk.detsum_max(u, m, U, M);
    return U - e.k * M;
}

/* twin: rr_knap — adds the jobs taken to S; false when outside the limits */
template <class Env, class Cand>
__device__ __forceinline__ bool sw_rr_knap(Env& e, Cand&& cand, int64_t cap, int64_t& budget) {
    constexpr int NT = SW_BLOCK;
    const int tid = (int)threadIdx.x;
    int cnt = 0;
    int64_t tw = 0;
    e.for_jobs([&](int j, int s) {
        if (cand(j, s)) {
            ++cnt;
            tw += e.jc(j).w;
        }
    });
    int NI = 0;
    const int base = e.blk.exscan(cnt, NI);
    const int64_t TW = e.blk.sum(tw);
    if (TW <= cap) {
        e.for_jobs([&](int j, int s) {
            if (cand(j, s)) e.S[j] = 1;
        });
        return true;
    }
    if (cap > SW_RR_CAPMAX) return false;
    const int nw = (int)((cap + 64) / 64);
    if ((int64_t)NI * nw > SW_RR_WORDS || budget < NI) return false;
    budget -= NI;
    int p = base;
    e.for_jobs([&](int j, int s) {
        if (cand(j, s)) {
            e.items[p] = (uint32_t)j; /* the full job index; its width is read back from jc */
            e.iv[p] = e.V(j, s);
            ++p;
        }
    });
    for (int c = tid; c <= cap; c += NT) e.dpA[c] = 0.0;
    __syncthreads();
    double* cur = e.dpA;
    double* nxt = e.dpB;
    const int span = nw * 64; /* whole words: a wave's lanes share one */
    for (int i = 0; i < NI; ++i) {
        const int w = e.jc((int)e.items[i]).w;
        const double v = e.iv[i];
        for (int c = tid; c < span; c += NT) {
            bool tk = false;
            if (c <= cap) {
                double x = cur[c];
                if (c >= w) {
                    const double y = cur[c - w] + v;
                    if (y > x) {
                        x = y;
                        tk = true;
                    }
                }
                nxt[c] = x;
            }
            const uint64_t word = __ballot(tk);
            if (lane_id() == 0) e.bits[(size_t)i * nw + (c >> 6)] = word;
        }
        __syncthreads();
        double* sw = cur;
        cur = nxt;
        nxt = sw;
    }
    /* the smallest capacity with the largest value */
    double bv = -1.0;
    int bc = 0x7FFFFFFF;
    for (int c = tid; c <= cap; c += NT)
        if (cur[c] > bv) {
            bv = cur[c];
            bc = c;
        }
    const double mv = e.blk.dmax(bv);
    const int cs = e.blk.min32(bv == mv ? bc : 0x7FFFFFFF);
    if (tid == 0) {
        int c = cs;
        for (int i = NI - 1; i >= 0; --i)
            if ((e.bits[(size_t)i * nw + (c >> 6)] >> (c & 63)) & 1ull) {
                const int j = (int)e.items[i];
                e.S[j] = 1;
                c -= e.jc(j).w;
            }
    }
    __syncthreads();
    return true;
}

/* twin: rr_round — true when round t's job set was replaced */
template <class Env>
__device__ __forceinline__ bool sw_rr_round(Env& e, int t, int64_t& budget, int64_t& passes) {
    const int G = e.G;
    passes++;
    double ucur = 0.0, mcur = 0.0, La = 0.0, hmax = 0.0;
    e.for_jobs([&](int j, int s) {
        const sw_jobc c = e.jc(j);
        const int in = (int)((e.y(j) >> t) & 1ull);
        const int b = e.cnt(j) - in;
        const bool el = e.tj(j);
        const double v = el ? e.f(c, b + 1) - e.f(c, b) : 0.0;
        const double h0 = sw_g(&c, b);
        const double h1 = el ? sw_g(&c, b + 1) : h0;
        e.V(j, s) = v;
        e.H0(j, s) = h0;
        e.H1(j, s) = h1;
        ucur = ucur + (in ? v : 0.0);
        const double hc = in ? h1 : h0;
        mcur = hc > mcur ? hc : mcur;
        const double a = el ? h1 : h0;
        La = a > La ? a : La;
        hmax = h0 > hmax ? h0 : hmax;
        e.S[j] = 0;
    });
    double Ucur, Mcur;
    e.blk.detsum_max(ucur, mcur, Ucur, Mcur);
    const double Jcur = Ucur - e.k * Mcur;
    La = e.blk.dmax(La);
    hmax = e.blk.dmax(hmax);
    /* the unconstrained knapsack: its value D bounds every level */
    if (!sw_rr_knap(
            e, [&](int j, int s) { return e.tj(j) && e.V(j, s) > 0.0 && e.jc(j).w <= G; },
            (int64_t)G, budget))
        return false;
    double D;
    double Jb = sw_rr_value(e, D);
    e.for_jobs([&](int j, int s) {
        (void)s;
        e.Sb[j] = e.S[j];
    });
    /* the smallest feasible level θ0 (twin: the snapped bisection) */
    uint64_t lo = 0, hi = sw_bits(hmax);
    while (lo < hi) {
        const double x = sw_from_bits(lo + ((hi - lo) >> 1));
        int64_t W = 0;
        uint64_t mx = 0, mn = ~0ull;
        e.for_jobs([&](int j, int s) {
            const double h0 = e.H0(j, s);
            const uint64_t b = sw_bits(h0);
            if (h0 > x) {
                W += e.jc(j).w;
                mn = b < mn ? b : mn;
            } else {
                mx = b > mx ? b : mx;
            }
        });
        int64_t Ws;
        uint64_t MX, MN;
        e.blk.sum_max_min(W, mx, mn, Ws, MX, MN);
        passes++;
        if (Ws <= G) hi = MX > lo ? MX : lo;
        else lo = MN < hi ? MN : hi;
    }
    const double th0 = sw_max(La, sw_from_bits(lo));
    double lvl = th0, prev = 0.0;
    bool have_prev = false;
    for (int tried = 0; tried < SW_RR_LEVELS; ++tried) {
        double th = th0;
        if (tried > 0) {
            uint64_t nb = ~0ull; /* the smallest value above lvl (bits of values ≥ 0) */
            e.for_jobs([&](int j, int s) {
                const double a = e.H0(j, s), b = e.H1(j, s);
                if (a > lvl) nb = sw_bits(a) < nb ? sw_bits(a) : nb;
                if (b > lvl) nb = sw_bits(b) < nb ? sw_bits(b) : nb;
            });
            nb = ~e.blk.umax(~nb);
            if (nb == ~0ull) break;
            th = sw_from_bits(nb);
        }
        if (have_prev && D - e.k * prev <= Jb) break;
        prev = th;
        have_prev = true;
        lvl = th;
        passes++;
        int64_t wf = 0, bad = 0;
        e.for_jobs([&](int j, int s) {
            const bool f = e.H0(j, s) > th;
            e.S[j] = f ? 1 : 0;
            if (f) {
                const int32_t w = e.jc(j).w;
                bad += (!e.tj(j) || e.H1(j, s) > th) ? 1 : 0;
                wf += w;
            }
        });
        int64_t WF, BAD;
        e.blk.sum2(wf, bad, WF, BAD);
        if (BAD != 0 || WF > G) continue;
        const int64_t cap = (int64_t)G - WF;
        if (!sw_rr_knap(
                e,
                [&](int j, int s) {
                    return e.S[j] == 0 && e.tj(j) && e.V(j, s) > 0.0 && (int64_t)e.jc(j).w <= cap;
                },
                cap, budget))
            continue;
        double Ux;
        const double J = sw_rr_value(e, Ux);
        if (J > Jb) {
            Jb = J;
            e.for_jobs([&](int j, int s) {
                (void)s;
                e.Sb[j] = e.S[j];
            });
        }
    }
    if (!(Jb - Jcur > SW_RR_TOL * (fabs(Jb) + fabs(Jcur)))) return false;
    e.for_jobs([&](int j, int s) {
        (void)s;
        const uint64_t bit = 1ull << t;
        const bool in = (e.y(j) & bit) != 0;
        const bool want = e.Sb[j] != 0;
        if (in != want) {
            e.y(j) ^= bit;
            e.add_cnt(j, want ? 1 : -1);
        }
    });
    return true;
}

/* twin: twin_reround_arrays — the rounds swept until a pass changes nothing
 * (at most SW_RR_PASSES); returns the rounds whose set changed.  Ends with a
 * barrier: every thread sees the final plan and counts. */
template <class Env>
__device__ __forceinline__ int sw_rr_run(Env& e, int64_t& passes) {
    int64_t budget = SW_RR_BUDGET;
    int moves = 0;
    for (int pass = 0; pass < SW_RR_PASSES; ++pass) {
        bool changed = false;
        for (int t = 0; t < e.T; ++t) {
            const bool c = sw_rr_round(e, t, budget, passes);
            changed |= c;
            moves += c ? 1 : 0;
        }
        if (!changed) break;
    }
    __syncthreads();
    return moves;
}
