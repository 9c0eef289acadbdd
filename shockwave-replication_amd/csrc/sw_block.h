/*
 * sw_block.h — workgroup primitives for the plan kernel (1024 threads =
 * 16 wave64 wavefronts per instance).  Wave-level steps use cross-lane
 * shuffles (ds_swizzle / DPP under the hood), the cross-wave step goes through
 * LDS.  Every reduction whose result feeds a decision is exact (integers,
 * max, lexicographic max) or follows the fixed halving tree of sw_detsum, so
 * the result does not depend on wave scheduling.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SW_BLOCK 1024
#define SW_WAVES (SW_BLOCK / 64)

struct sw_scratch {
    double dtree[SW_BLOCK];       /* halving-tree scratch (8 KB)            */
    int64_t wsum[SW_WAVES][2];    /* per-wave partials                        */
    uint64_t wmax[SW_WAVES];
    double wdmax[SW_WAVES];
    int32_t wscan[SW_WAVES];
    int64_t bcast_i[4];
    double bcast_d[4];
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ int32_t wave_sum_i32(int32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        uint64_t x = __shfl_xor(v, o, 64);
        v = x > v ? x : v;
    }
    return v;
}

__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        double x = __shfl_xor(v, o, 64);
        v = x > v ? x : v;
    }
    return v;
}

/* Sum of two int64 values over the block (one pair of barriers). */
__device__ __forceinline__ void block_sum2(int64_t a, int64_t b, int64_t* ra, int64_t* rb,
                                           sw_scratch* s) {
    a = wave_sum_i64(a);
    b = wave_sum_i64(b);
    if (lane_id() == 0) { s->wsum[wave_id()][0] = a; s->wsum[wave_id()][1] = b; }
    __syncthreads();
    int64_t ta = 0, tb = 0;
#pragma unroll
    for (int i = 0; i < SW_WAVES; ++i) { ta += s->wsum[i][0]; tb += s->wsum[i][1]; }
    __syncthreads();
    *ra = ta;
    *rb = tb;
}

__device__ __forceinline__ int64_t block_sum(int64_t a, sw_scratch* s) {
    int64_t ra, rb;
    block_sum2(a, 0, &ra, &rb, s);
    return ra;
}

__device__ __forceinline__ uint64_t block_max_u64(uint64_t v, sw_scratch* s) {
    v = wave_max_u64(v);
    if (lane_id() == 0) s->wmax[wave_id()] = v;
    __syncthreads();
    uint64_t m = 0;
#pragma unroll
    for (int i = 0; i < SW_WAVES; ++i) m = s->wmax[i] > m ? s->wmax[i] : m;
    __syncthreads();
    return m;
}

__device__ __forceinline__ double block_max_d(double v, sw_scratch* s) {
    v = wave_max_d(v);
    if (lane_id() == 0) s->wdmax[wave_id()] = v;
    __syncthreads();
    double m = s->wdmax[0];
#pragma unroll
    for (int i = 1; i < SW_WAVES; ++i) m = s->wdmax[i] > m ? s->wdmax[i] : m;
    __syncthreads();
    return m;
}

/* Exclusive prefix sum over thread order (int32).  *total gets the sum. */
__device__ __forceinline__ int32_t block_exscan_i32(int32_t v, int32_t* total, sw_scratch* s) {
    int lane = lane_id();
    int32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s->wscan[wave_id()] = x;
    __syncthreads();
    int32_t base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < SW_WAVES; ++i) {
        int32_t t = s->wscan[i];
        base += (i < wave_id()) ? t : 0;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

/*
 * Deterministic sum (must equal sw_detsum in oracle/plan_twin.c): thread i
 * holds lane i's left-to-right partial; combine p[i] += p[i+h] for
 * h = 512 … 1.  h ≥ 64 through LDS, h ≤ 32 inside wave 0.
 */
__device__ __forceinline__ double block_detsum(double v, sw_scratch* s) {
    int tid = threadIdx.x;
    s->dtree[tid] = v;
    __syncthreads();
#pragma unroll
    for (int h = SW_BLOCK / 2; h >= 64; h >>= 1) {
        if (tid < h) s->dtree[tid] = s->dtree[tid] + s->dtree[tid + h];
        __syncthreads();
    }
    if (tid < 64) {
        double x = s->dtree[tid];
#pragma unroll
        for (int h = 32; h >= 1; h >>= 1) {
            double y = __shfl_down(x, h, 64);
            x = x + y;
        }
        if (tid == 0) s->bcast_d[0] = x;
    }
    __syncthreads();
    double r = s->bcast_d[0];
    __syncthreads();
    return r;
}
