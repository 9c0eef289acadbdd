/*
 * sw_pack.h — the block-wide round loop of the placement (twin: the t loop of
 * pack() in oracle/plan_twin.c; reference: the per-round schedule the P1/P2
 * MILPs return, shockwave.py:281-328, :390-398).
 *
 * 512 threads (sw_block.h) own E consecutive positions each of the job order
 * (position p = E·tid + i), so a block exclusive scan is the twin's running
 * "excl" over positions.  Per-position state is packed in a VGPR:
 * r (rounds still to place, 8 bits) | w << 8 (width, 8 bits) | sel << 16.
 * Per-round histograms live in LDS and are double-buffered by round parity,
 * so each round needs one barrier before its tiers.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sw_block.h"

__device__ __forceinline__ uint32_t pk_r(uint32_t s) { return s & 0xFFu; }
__device__ __forceinline__ uint32_t pk_w(uint32_t s) { return (s >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t pk_sel(uint32_t s) { return (s >> 16) & 1u; }

/* LDS the round loop needs: two 68-entry buffers each for H and SH. */
struct sw_pack_lds {
    int32_t H[2][68];
    int32_t SH[2][68];
};

/*
 * Places the rounds of positions [0, A) into T rounds of capacity G.
 * st[i] holds position E·tid + i's packed state (0 past A); on return mk[i]
 * has bit t set when that position runs in round t and st[i]'s r field is
 * what could not be placed.
 */
template <int E>
__device__ __forceinline__ void sw_pack_rounds(sw_blk& blk, sw_pack_lds* L, int A, int T, int G,
                                               uint32_t (&st)[E], uint64_t (&mk)[E]) {
    const int tid = threadIdx.x;
    const int lane = lane_id();
    if (tid < 68) { L->H[0][tid] = 0; L->SH[0][tid] = 0; }
#pragma unroll
    for (int i = 0; i < E; ++i) mk[i] = 0;
    __syncthreads();
    for (int t = 0; t < T; ++t) {
        const int R = T - t;
        int32_t* Hc = L->H[t & 1];
        int32_t* SHc = L->SH[t & 1];
        int32_t cap = G;
#pragma unroll
        for (int i = 0; i < E; ++i) {
            if (E * tid + i < A) {
                const int rr = (int)pk_r(st[i]) < R ? (int)pk_r(st[i]) : R;
                atomicAdd(&Hc[rr], (int32_t)pk_w(st[i]));
            }
        }
        /* clear next round's buffers (read by nobody this round) */
        if (tid < 68) { L->H[(t + 1) & 1][tid] = 0; L->SH[(t + 1) & 1][tid] = 0; }
        __syncthreads();
        /* need_m = Σ_{v>m} (v−m)·H[v] − G·(R−1−m), lane m (every wave alike) */
        const int32_t hv = (lane + 1 <= R) ? Hc[lane + 1] : 0;
        const int32_t S0 = wave_sufscan_i32(hv);
        const int32_t S1 = wave_sufscan_i32(hv * (lane + 1));
        const int32_t need = (lane < R) ? (S1 - lane * S0) - G * (R - 1 - lane) : -1;
        /* tiers: jobs with more than m rounds left must shed enough now */
        int mstart = R - 1;
        while (mstart >= 0) {
            const int32_t shv = (lane + 1 <= R) ? SHc[lane + 1] : 0;
            const int32_t red = wave_sufscan_i32(shv);
            const uint64_t mask = __ballot(lane <= mstart && need - red > 0);
            if (mask == 0) break;
            const int m = 63 - __builtin_clzll(mask);
            const int32_t q = __shfl(need - red, m, 64);
            int32_t lt = 0;
#pragma unroll
            for (int i = 0; i < E; ++i) {
                const int rr = (int)pk_r(st[i]) < R ? (int)pk_r(st[i]) : R;
                if (E * tid + i < A && !pk_sel(st[i]) && rr > m) lt += (int32_t)pk_w(st[i]);
            }
            int32_t tot;
            int32_t ex = blk.exscan(lt, tot);
            int32_t took = 0;
#pragma unroll
            for (int i = 0; i < E; ++i) {
                const int rr = (int)pk_r(st[i]) < R ? (int)pk_r(st[i]) : R;
                if (E * tid + i < A && !pk_sel(st[i]) && rr > m) {
                    const int32_t w = (int32_t)pk_w(st[i]);
                    if (ex < q && ex + w <= cap) {
                        st[i] |= (1u << 16);
                        atomicAdd(&SHc[rr], w);
                        took += w;
                    }
                    ex += w;
                }
            }
            cap -= blk.sum32(took);
            mstart = m - 1;
        }
        /* fill the rest of the round in order */
        {
            int32_t lt = 0;
#pragma unroll
            for (int i = 0; i < E; ++i)
                if (E * tid + i < A && !pk_sel(st[i]) && pk_r(st[i]) > 0) lt += (int32_t)pk_w(st[i]);
            int32_t tot;
            int32_t ex = blk.exscan(lt, tot);
            int32_t took = 0;
#pragma unroll
            for (int i = 0; i < E; ++i) {
                if (E * tid + i < A && !pk_sel(st[i]) && pk_r(st[i]) > 0) {
                    const int32_t w = (int32_t)pk_w(st[i]);
                    if (ex + w <= cap) { st[i] |= (1u << 16); took += w; }
                    ex += w;
                }
            }
            cap -= blk.sum32(took);
        }
        /* width tail: first position in order that still fits; the key
         * carries (position << 8 | w) so the min also names the width */
        while (cap > 0) {
            int32_t best = 0x7FFFFFFF;
#pragma unroll
            for (int i = E - 1; i >= 0; --i) {
                if (E * tid + i < A && !pk_sel(st[i]) && pk_r(st[i]) > 0 && (int32_t)pk_w(st[i]) <= cap)
                    best = ((E * tid + i) << 8) | (int32_t)pk_w(st[i]);
            }
            best = blk.min32(best);
            if (best == 0x7FFFFFFF) break;
            const int pos = best >> 8;
            if (pos / E == tid) {
#pragma unroll
                for (int i = 0; i < E; ++i)
                    if (i == pos % E) st[i] |= (1u << 16);
            }
            cap -= best & 0xFF;
        }
#pragma unroll
        for (int i = 0; i < E; ++i) {
            if (E * tid + i < A && pk_sel(st[i])) {
                mk[i] |= (1ull << t);
                st[i] = (st[i] & 0xFF00u) | (pk_r(st[i]) - 1u);
            }
        }
    }
    __syncthreads();
}
