/*
 * sw_pack.h — the block-wide round loop of the placement (twin: the t loop of
 * pack() in oracle/plan_twin.c; reference: the per-round schedule the P1/P2
 * MILPs return, shockwave.py:281-328, :390-398).
 *
 * 512 threads (sw_block.h) own E consecutive positions each of the job order
 * (position p = E·tid + i), so a block exclusive scan is the twin's running
 * "excl" over positions.  Per-position state is packed in a VGPR:
 * r (rounds still to place, 8 bits) | w << 8 (width, 8 bits) | sel << 16.
 *
 * The width histogram over remaining rounds, Hu[v] = Σ w over positions with
 * r = v, is built once and then kept up to date: a position placed in round t
 * moves w from Hu[r] to Hu[r − 1] (2 LDS atomics per placed position instead
 * of one per position per round — the per-round rebuild was the kernel's LDS
 * bank-conflict hot spot at 10k jobs).  Hu is held in SW_HCOPIES copies by
 * lane (sw_pack_lds::Hc), summed at each round's start.  The round's clamped histogram
 * H[v] = Hu[v] (v < R), H[R] = Σ_{v ≥ R} Hu[v] is formed in registers.  The
 * tier histogram SH is per round and double-buffered by round parity, so
 * each round needs one barrier before its tiers.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sw_block.h"

#ifdef SW_STAMPS
/* diagnostic builds: cycles per round-loop phase, thread 0's view, kept in
 * registers and added to swp[k] on exit (0 setup, 1 histogram+need, 2 tiers,
 * 3 fill, 4 tail, 5 apply; swp[17..19] rounds, active tiers, width-tail
 * reductions; swp[20..22] the wave loop's tier parts: head, scan, take — its
 * "tiers" stamp then holds only the loop exits) — a global read-modify-write per stamp would add a memory
 * round trip to every phase it times */
#define SWP_DECL                                          \
    uint64_t swp_t_ = __builtin_amdgcn_s_memtime();       \
    uint64_t swp_a_[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; \
    uint32_t swp_c_[3] = {0, 0, 0}
#define SWP_STAMP(k)                                          \
    do {                                                      \
        const uint64_t now_ = __builtin_amdgcn_s_memtime();   \
        swp_a_[k] += now_ - swp_t_;                           \
        swp_t_ = now_;                                        \
    } while (0)
#define SWP_COUNT(k) (swp_c_[(k) - 17] += 1)
#define SWP_FLUSH                                                         \
    do {                                                                  \
        if (threadIdx.x == 0 && swp) {                                    \
            for (int k_ = 0; k_ < 6; ++k_) swp[k_] += swp_a_[k_];         \
            for (int k_ = 0; k_ < 3; ++k_) swp[17 + k_] += swp_c_[k_];    \
            for (int k_ = 6; k_ < 10; ++k_) swp[14 + k_] += swp_a_[k_];   \
        }                                                                 \
    } while (0)
#else
#define SWP_DECL \
    do {         \
    } while (0)
#define SWP_STAMP(k) \
    do {             \
    } while (0)
#define SWP_COUNT(k) \
    do {             \
    } while (0)
#define SWP_FLUSH \
    do {          \
    } while (0)
#endif

__device__ __forceinline__ uint32_t pk_r(uint32_t s) { return s & 0xFFu; }
__device__ __forceinline__ uint32_t pk_w(uint32_t s) { return (s >> 8) & 0xFFu; }

/* LDS the round loop needs: the running histogram's copies Hc; H and SH are
 * spare (kept for the carve-up of sw_kernels.hip). */
#ifndef SW_HCOPIES
#define SW_HCOPIES 4
#endif
struct sw_pack_lds {
    int32_t H[2][68];
    int32_t SH[2][68];
    /* the one-wave loop's histogram, in SW_HCOPIES copies by lane: the
     * positions a round places mostly share one or two remaining-round counts,
     * and their atomics on one bin serialise in the LDS (copy c's bin v sits
     * in bank 8c + v, so the copies of a bin never share a bank); four copies
     * measured best against one, two and eight (each round sums them) */
    int32_t Hc[SW_HCOPIES][72];
};

/*
 * Places the rounds of positions [0, A) into T rounds of capacity G.
 * st[i] holds position E·tid + i's packed state (0 past A); on return mk[i]
 * has bit t set when that position runs in round t and st[i]'s r field is
 * what could not be placed.
 *
 * Tiers (twin: the m loop of pack).  Tier m may take positions with rr > m
 * up to q = need[m] − red(m), red(m) = Σ_{v>m} SH[v] the width already taken
 * by this round's tiers with rr = v.  Tiers run from high m down and every
 * position a tier m' took has rr > m' > m, so red(m) is simply the running
 * total of tier takes: no per-round SH histogram is needed.
 *
 * The per-position loops are branch-free (predicated adds and selects): with
 * E up to 32 positions per thread, per-position branches each held a 64-bit
 * exec mask and spilled the SGPR file.
 */
/* Room after round t for jobs with more than m rounds left, lane m:
 * the R−1−m smallest capacities of rounds t+1 … T−1 (twin: Lsum[R−1−m]);
 * G·(R−1−m) when every round has capacity G (caps == nullptr).  cbase ≥ 0:
 * every capacity is cbase or cbase + 1 (the share placement's shares,
 * sw_share_caps): the x smallest of the later rounds then sum to
 * x·cbase + max(0, x − #{later rounds at cbase}), one ballot instead of a
 * wave sort — the same value. */
__device__ __forceinline__ int32_t sw_pack_caps_base(const int32_t* caps, int T) {
    if (!caps) return -1;
    const int lane = lane_id();
    const int32_t mn = wave_min_i32(lane < T ? caps[lane] : 0x7FFFFFFF);
    const int32_t mx = wave_max_i32(lane < T ? caps[lane] : (int32_t)0x80000000);
    return mx - mn <= 1 ? mn : -1;
}

__device__ __forceinline__ int32_t sw_pack_room(const int32_t* caps, int t, int R, int G,
                                                int32_t cbase = -1) {
    const int lane = lane_id();
    if (!caps) return G * (R - 1 - lane);
    if (cbase >= 0) {
        const int32_t nb = __popcll(__ballot(lane < R - 1 && caps[t + 1 + lane] == cbase));
        const int32_t x = R - 1 - lane;
        return x > 0 ? x * cbase + (x > nb ? x - nb : 0) : 0;
    }
    int32_t v = (lane < R - 1) ? caps[t + 1 + lane] : 0x7FFFFFFF;
    v = wave_sort_asc_i32(v);
    v = (lane < R - 1) ? v : 0;
    const int32_t ps = wave_incscan_i32(v);
    const int x = R - 1 - lane;
    const int32_t pv = __shfl(ps, x > 0 ? x - 1 : 0, 64);
    return x > 0 ? pv : 0;
}

/* The histogram copies → the cumulative form C[v] = Σ_{u ≥ v} Hu[u] in copy
 * 0 (the other copies zeroed), by one wave (its LDS reads issue before its
 * writes).  In that form a position placed in round t (r → r − 1) changes
 * C[r] alone — one atomic instead of two — and the round's need is one
 * suffix sum (sw_pack_need). */
__device__ __forceinline__ void sw_pack_cum(sw_pack_lds* L) {
    const int lane = lane_id();
    int32_t h = 0, h64 = 0;
#pragma unroll
    for (int c = 0; c < SW_HCOPIES; ++c) {
        h += L->Hc[c][lane];
        h64 += L->Hc[c][64];
    }
    const int32_t C = wave_sufscan_i32(h) + h64;
#pragma unroll
    for (int c = 0; c < SW_HCOPIES; ++c) {
        L->Hc[c][lane] = c == 0 ? C : 0;
        if (lane < 8) L->Hc[c][64 + lane] = (c == 0 && lane == 0) ? h64 : 0;
    }
}

/* need_m = Σ_{v>m} (v−m)·H[v] − room_m over the round's clamped histogram
 * (H[v] = Hu[v] for v < R, H[R] = Σ_{v ≥ R} Hu[v]), lane m < R (−1 above):
 * by parts, Σ_{v>m} (v−m)·H[v] = Σ_{v=m+1}^{R} C[v] — the same integer. */
__device__ __forceinline__ int32_t sw_pack_need(const sw_pack_lds* L, int R, int32_t room) {
    const int lane = lane_id();
    int32_t c1 = 0; /* C[lane + 1], the copies summed */
#pragma unroll
    for (int c = 0; c < SW_HCOPIES; ++c) c1 += L->Hc[c][lane + 1];
    const int32_t D = wave_sufscan_i32(lane + 1 <= R ? c1 : 0);
    return lane < R ? D - room : -1;
}

/* caps: per-round capacity in LDS (nullptr = G every round) — the class-wise
 * P2 repack, where positions carry unit widths */
template <int E, class BLK>
__device__ __forceinline__ void sw_pack_rounds(BLK& blk, sw_pack_lds* L, int A, int T, int G,
                                               uint32_t (&st)[E], uint64_t (&mk)[E],
                                               const int32_t* caps = nullptr,
                                               uint64_t* swp = nullptr) {
    (void)swp; /* phase stamps (SW_STAMPS builds) */
    const int tid = threadIdx.x;
    const int lane = lane_id();
    SWP_DECL;
    /* positions past A carry st = 0 (r = 0, w = 0): they fail every
     * eligibility test below, so no per-position bound check is needed */
    /* the running histogram in SW_HCOPIES copies by lane (L->Hc, as the
     * one-wave loop below): the positions a round places mostly share a few
     * remaining-round counts, and a wave's atomics on one LDS word serialise
     * over its lanes — with one copy the apply's atomics and the barrier
     * waiting on them were 48 % of the C4 placement's cycles */
    int32_t* Hm = L->Hc[lane & (SW_HCOPIES - 1)];
    for (int x = tid; x < SW_HCOPIES * 72; x += blockDim.x) (&L->Hc[0][0])[x] = 0;
#pragma unroll
    for (int i = 0; i < E; ++i) mk[i] = 0;
    const int32_t cbase = sw_pack_caps_base(caps, T);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < E; ++i)
        if (st[i] != 0u) atomicAdd(&Hm[pk_r(st[i])], (int32_t)pk_w(st[i]));
    __syncthreads();
    if (tid < 64) sw_pack_cum(L); /* the first round's barrier publishes it */
    /* here st[i] = r | w << 8 | ra << 16, ra = r while the position is open
     * this round and 0 once taken (as in the one-wave loop): with m < R,
     * min(r, R) > m is r > m, so every eligibility test is one compare of ra */
#define PK_RA(x) ((int32_t)(((x) >> 16) & 0xFFu))
#pragma unroll
    for (int i = 0; i < E; ++i) st[i] = (st[i] & 0xFFFFu) | ((st[i] & 0xFFu) << 16);
    SWP_STAMP(0);
    for (int t = 0; t < T; ++t) {
        const int R = T - t;
        int32_t cap = caps ? caps[t] : G;
        SWP_COUNT(17);
        __syncthreads(); /* the copies hold the placements of round t − 1 */
        /* need_m, lane m (every wave alike) */
        const int32_t need = sw_pack_need(L, R, sw_pack_room(caps, t, R, G, cbase));
        SWP_STAMP(1);
        /* tiers: jobs with more than m rounds left must shed enough now */
        int mstart = R - 1;
        int32_t red = 0;
        while (mstart >= 0) {
            const uint64_t mask = __ballot(lane <= mstart && need - red > 0);
            if (mask == 0) break;
            const int m = 63 - __builtin_clzll(mask);
            SWP_COUNT(18);
            const int32_t q = __builtin_amdgcn_readlane(need, m) - red;
            int32_t lt = 0;
#pragma unroll
            for (int i = 0; i < E; ++i) lt += PK_RA(st[i]) > m ? (int32_t)pk_w(st[i]) : 0;
            int32_t tot;
            int32_t ex = blk.exscan(lt, tot);
            int32_t took = 0;
#pragma unroll
            for (int i = 0; i < E; ++i) {
                const int32_t w = (int32_t)pk_w(st[i]);
                const bool elig = PK_RA(st[i]) > m;
                const bool take = elig && ex < q && ex + w <= cap;
                st[i] = take ? (st[i] & 0xFFFFu) : st[i];
                took += take ? w : 0;
                ex += elig ? w : 0;
            }
            took = blk.sum32(took);
            cap -= took;
            red += took;
            mstart = m - 1;
        }
        SWP_STAMP(2);
        /* fill the rest of the round in order */
        {
            int32_t lt = 0;
#pragma unroll
            for (int i = 0; i < E; ++i) lt += PK_RA(st[i]) > 0 ? (int32_t)pk_w(st[i]) : 0;
            int32_t tot;
            int32_t ex = blk.exscan(lt, tot);
            int32_t took = 0;
#pragma unroll
            for (int i = 0; i < E; ++i) {
                const int32_t w = (int32_t)pk_w(st[i]);
                const bool elig = PK_RA(st[i]) > 0;
                const bool take = elig && ex + w <= cap;
                st[i] = take ? (st[i] & 0xFFFFu) : st[i];
                took += take ? w : 0;
                ex += elig ? w : 0;
            }
            cap -= blk.sum32(took);
        }
        SWP_STAMP(3);
        /* width tail: first position in order that still fits; the key
         * carries (position << 8 | w) so the min also names the width */
        while (cap > 0) {
            int32_t best = 0x7FFFFFFF;
#pragma unroll
            for (int i = E - 1; i >= 0; --i) {
                const bool ok = PK_RA(st[i]) > 0 && (int32_t)pk_w(st[i]) <= cap;
                best = ok ? (((E * tid + i) << 8) | (int32_t)pk_w(st[i])) : best;
            }
            best = blk.min32(best);
            SWP_COUNT(19);
            if (best == 0x7FFFFFFF) break;
            const int pos = best >> 8;
#pragma unroll
            for (int i = 0; i < E; ++i) st[i] = (E * tid + i == pos) ? (st[i] & 0xFFFFu) : st[i];
            cap -= best & 0xFF;
        }
        SWP_STAMP(4);
        /* apply (all reads of the copies this round happened before the
         * fill's barrier): placed positions (r > 0, ra = 0) move their width
         * down one bin and open for the next round with ra = r − 1 */
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const uint32_t r = pk_r(st[i]);
            const bool sel = PK_RA(st[i]) == 0 && r > 0;
            mk[i] |= sel ? (1ull << t) : 0ull;
            if (sel) atomicAdd(&Hm[r], -(int32_t)pk_w(st[i])); /* C[r] alone */
            const uint32_t r2 = r - (sel ? 1u : 0u);
            st[i] = r2 | (st[i] & 0xFF00u) | (r2 << 16);
        }
        SWP_STAMP(5);
    }
#pragma unroll
    for (int i = 0; i < E; ++i) st[i] &= 0xFFFFu; /* r | w << 8, as the callers read it */
#undef PK_RA
    SWP_FLUSH;
    __syncthreads();
}

/* The width a tier (or the fill) took, without a reduction: a position is
 * taken when it is eligible, its eligible prefix ex is below the tier's quota
 * and ex + w fits the round, and both tests fail for every later eligible
 * position once they fail for one (ex grows by at least the failing width),
 * so the taken positions are a prefix of the eligible ones.  The wave's last
 * lane that took any then holds the end of that prefix: its eligible base
 * plus its own take (its eligible positions before its first untaken one). */
__device__ __forceinline__ int32_t sw_pack_took(int32_t base, int32_t took) {
    const uint64_t mk = __ballot(took > 0);
    if (mk == 0) return 0;
    return __builtin_amdgcn_readlane(base + took, 63 - __builtin_clzll(mk));
}

/*
 * The same round loop run by ONE wave over E1 positions per lane
 * (position p = E1·lane + i, so a wave exclusive scan of the lane totals is
 * again the twin's running "excl"), for instances with at most 64·E1
 * positions.  Tier m < R tests r > m directly (min(r, R) > m is the same
 * test when m < R).  The
 * block version issues every scan, reduction and partial combine in all
 * eight waves and waits at two barriers per tier; here one wave issues each
 * step once and never waits for the others (on a C3 instance the round loop
 * was two thirds of the pack kernel's VALU instructions).  The histogram
 * (L->Hc, four copies summed at each round's start) is updated by this wave
 * alone, so its LDS atomics and reads stay in program order.
 * Called by wave 0 only; st as in sw_pack_rounds, the round masks go to
 * xmk[position] (LDS or workspace) with an atomic OR per placement instead
 * of 2·E1 VGPRs held through the loop.
 */
template <int E1>
__device__ __forceinline__ void sw_pack_rounds_wave(sw_pack_lds* L, int T, int G, uint32_t (&st)[E1],
                                                    uint64_t* xmk, const int32_t* caps = nullptr,
                                                    uint64_t* swp = nullptr) {
    (void)swp;
    const int lane = lane_id();
    SWP_DECL;
    int32_t* Hm = L->Hc[lane & (SW_HCOPIES - 1)]; /* this lane's histogram copy */
    /* the state carries, besides the rounds still to place (rr) and the
     * width, the rounds still to place of a position not yet taken this
     * round (ra, 0 once taken): every eligibility test is one compare of ra */
    /* st[i] here: rr | w << 8 | ra << 16, one byte each (the compares read
     * the bytes in place) */
#define RR_(i) ((int32_t)(st[i] & 0xFFu))
#define WW_(i) ((int32_t)((st[i] >> 8) & 0xFFu))
#define RA_(i) ((int32_t)((st[i] >> 16) & 0xFFu))
#pragma unroll
    for (int i = 0; i < E1; ++i) st[i] = (st[i] & 0xFFFFu) | ((st[i] & 0xFFu) << 16);
#pragma unroll
    for (int c = 0; c < SW_HCOPIES; ++c) {
        L->Hc[c][lane] = 0;
        if (lane < 8) L->Hc[c][64 + lane] = 0;
    }
#pragma unroll
    for (int i = 0; i < E1; ++i) xmk[E1 * lane + i] = 0;
    wave_sync();
#pragma unroll
    for (int i = 0; i < E1; ++i)
        if (st[i] != 0u) atomicAdd(&Hm[RR_(i)], WW_(i));
    wave_sync();
    sw_pack_cum(L);
    const int32_t cbase = sw_pack_caps_base(caps, T);
    SWP_STAMP(0);
    for (int t = 0; t < T; ++t) {
        const int R = T - t;
        int32_t cap = caps ? caps[t] : G;
        SWP_COUNT(17);
        SWP_STAMP(9); /* diagnostic: the cost of one stamp */
        wave_sync(); /* the copies hold the placements of round t − 1 */
        const int32_t need = sw_pack_need(L, R, sw_pack_room(caps, t, R, G, cbase));
        SWP_STAMP(1);
        int mstart = R - 1;
        int32_t red = 0;
        while (mstart >= 0) {
            const uint64_t mask = __ballot(lane <= mstart && need - red > 0);
            if (mask == 0) break;
            const int m = 63 - __builtin_clzll(mask);
            SWP_COUNT(18);
            const int32_t q = __builtin_amdgcn_readlane(need, m) - red;
            SWP_STAMP(6);
            /* in-lane exclusive prefixes first, so the take tests of a
             * lane's positions are independent of each other */
            int32_t pre[E1];
            int32_t lt = 0;
#pragma unroll
            for (int i = 0; i < E1; ++i) {
                pre[i] = lt;
                lt += RA_(i) > m ? WW_(i) : 0;
            }
            const int32_t base = wave_incscan_i32(lt) - lt;
            SWP_STAMP(7);
            int32_t took = 0;
#pragma unroll
            for (int i = 0; i < E1; ++i) {
                const int32_t ex = base + pre[i];
                const bool take = RA_(i) > m && ex < q && ex + WW_(i) <= cap;
                took += take ? WW_(i) : 0;
                st[i] = take ? (st[i] & 0xFFFFu) : st[i];
            }
            took = sw_pack_took(base, took);
            cap -= took;
            red += took;
            mstart = m - 1;
            SWP_STAMP(8);
        }
        SWP_STAMP(2);
        {
            int32_t pre[E1];
            int32_t lt = 0;
#pragma unroll
            for (int i = 0; i < E1; ++i) {
                pre[i] = lt;
                lt += RA_(i) > 0 ? WW_(i) : 0;
            }
            const int32_t base = wave_incscan_i32(lt) - lt;
            int32_t took = 0;
#pragma unroll
            for (int i = 0; i < E1; ++i) {
                const bool take = RA_(i) > 0 && base + pre[i] + WW_(i) <= cap;
                took += take ? WW_(i) : 0;
                st[i] = take ? (st[i] & 0xFFFFu) : st[i];
            }
            cap -= sw_pack_took(base, took);
        }
        SWP_STAMP(3);
        while (cap > 0) {
            int32_t best = 0x7FFFFFFF;
#pragma unroll
            for (int i = E1 - 1; i >= 0; --i) {
                const bool ok = RA_(i) > 0 && WW_(i) <= cap;
                best = ok ? (((E1 * lane + i) << 8) | WW_(i)) : best;
            }
            best = wave_min_i32(best);
            SWP_COUNT(19);
            if (best == 0x7FFFFFFF) break;
            const int pos = best >> 8;
#pragma unroll
            for (int i = 0; i < E1; ++i) st[i] = (E1 * lane + i == pos) ? (st[i] & 0xFFFFu) : st[i];
            cap -= best & 0xFF;
        }
        SWP_STAMP(4);
#pragma unroll
        for (int i = 0; i < E1; ++i) {
            const int32_t r = RR_(i);
            const bool sel = RA_(i) == 0 && r > 0;
            if (sel) {
                atomicAdd(&Hm[r], -WW_(i)); /* C[r] alone */
                atomicOr((unsigned long long*)&xmk[E1 * lane + i], 1ull << t);
            }
            const uint32_t r2 = (uint32_t)(r - (sel ? 1 : 0));
            st[i] = r2 | (st[i] & 0xFF00u) | (r2 << 16);
        }
        SWP_STAMP(5);
    }
#pragma unroll
    for (int i = 0; i < E1; ++i) st[i] &= 0xFFFFu;
#undef RR_
#undef WW_
#undef RA_
    SWP_FLUSH;
    wave_sync();
}

/* sw_pack_rounds for at most 512 positions, one per thread (position tid):
 * the states are staged through LDS / workspace words xs (≥ 6 KB, free at the
 * call) into wave 0, which runs sw_pack_rounds_wave<E1> with E1 the even
 * number of positions per lane that covers A (2, 4, 6 or 8: a runtime bound
 * inside the unrolled loops costs the kernel's register budget) when MULTI,
 * else 6 or 8 (the plan kernel, whose register file four copies would
 * overflow); every thread of the block must call it. */
template <int E1>
__device__ __forceinline__ void sw_pack_rounds_wave_io(sw_pack_lds* L, int T, int G, uint32_t* xst,
                                                      uint64_t* xmk, const int32_t* caps,
                                                      uint64_t* swp) {
    const int lane = lane_id();
    uint32_t st[E1];
#pragma unroll
    for (int i = 0; i < E1; ++i) st[i] = xst[E1 * lane + i];
    /* the loop is the instance's critical path while the CU's other
     * workgroups run phases that only need throughput: issue it first */
    __builtin_amdgcn_s_setprio(3);
    sw_pack_rounds_wave<E1>(L, T, G, st, xmk, caps, swp);
    __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int i = 0; i < E1; ++i) xst[E1 * lane + i] = st[i];
}

template <bool MULTI>
__device__ __forceinline__ void sw_pack_rounds_one(sw_pack_lds* L, int A, int T, int G, uint32_t& st1,
                                                   uint64_t& mk1, uint64_t* xs,
                                                   const int32_t* caps = nullptr,
                                                   uint64_t* swp = nullptr) {
    uint32_t* xst = reinterpret_cast<uint32_t*>(xs);
    uint64_t* xmk = xs + SW_BLOCK / 2;
    xst[threadIdx.x] = st1; /* 0 past A */
    __syncthreads();
    if (wave_id() == 0) {
        if (!MULTI) {
            if (A <= 384) sw_pack_rounds_wave_io<6>(L, T, G, xst, xmk, caps, swp);
            else sw_pack_rounds_wave_io<8>(L, T, G, xst, xmk, caps, swp);
        } else if (A <= 128) sw_pack_rounds_wave_io<2>(L, T, G, xst, xmk, caps, swp);
        else if (A <= 256) sw_pack_rounds_wave_io<4>(L, T, G, xst, xmk, caps, swp);
        else if (A <= 384) sw_pack_rounds_wave_io<6>(L, T, G, xst, xmk, caps, swp);
        else sw_pack_rounds_wave_io<8>(L, T, G, xst, xmk, caps, swp);
    }
    __syncthreads();
    st1 = xst[threadIdx.x];
    mk1 = xmk[threadIdx.x];
}
