/*
 * sw_block.h — workgroup and wavefront primitives for the plan kernel
 * (512 threads = 8 wave64 per instance).
 *
 * Block reductions take ONE barrier: each wave reduces with cross-lane
 * shuffles (DPP / ds_swizzle under the hood), lane 0 publishes its partial
 * to an LDS slot, one __syncthreads, every thread combines the 16 partials.
 * Successive reductions alternate between two slot sets, so no second
 * barrier is needed before a slot is rewritten.  Every reduction whose
 * result feeds a decision is exact (integers, max, lexicographic max) or
 * the fixed-order tree of sw_detsum (oracle/plan_twin.c), so results do not
 * depend on wave scheduling.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SW_BLOCK 512
#define SW_WAVES (SW_BLOCK / 64)

struct sw_xchg {
    int64_t i[2][SW_WAVES][2];
    double d[2][SW_WAVES][2];
    uint64_t u[2][SW_WAVES];
    int32_t s[2][SW_WAVES];
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

/* Order LDS accesses of one wave (the hardware keeps a wave's LDS ops in
 * order; this keeps the compiler from moving them). */
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        T x = __shfl_xor(v, o, 64);
        v = x > v ? x : v;
    }
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        T x = __shfl_xor(v, o, 64);
        v = x < v ? x : v;
    }
    return v;
}

/* Inclusive prefix sum over lanes. */
template <typename T>
__device__ __forceinline__ T wave_incscan(T v) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    return v;
}

/* Inclusive suffix sum over lanes (lane L gets Σ_{l ≥ L}). */
template <typename T>
__device__ __forceinline__ T wave_sufscan(T v) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T y = __shfl_down(v, o, 64);
        if (lane + o < 64) v += y;
    }
    return v;
}

/* Fixed halving tree over the wave (p[i] += p[i+h], h = 32 … 1); the result
 * is valid in lane 0. */
__device__ __forceinline__ double wave_dettree(double x) {
#pragma unroll
    for (int h = 32; h >= 1; h >>= 1) {
        double y = __shfl_down(x, h, 64);
        x = x + y;
    }
    return x;
}

struct sw_blk {
    sw_xchg* X;
    int par;

    __device__ __forceinline__ void flip() { par ^= 1; }

    __device__ __forceinline__ int32_t sum32(int32_t v) {
        v = wave_sum(v);
        if (lane_id() == 0) X->s[par][wave_id()] = v;
        __syncthreads();
        int32_t t = 0;
#pragma unroll
        for (int w = 0; w < SW_WAVES; ++w) t += X->s[par][w];
        flip();
        return t;
    }

    __device__ __forceinline__ int32_t min32(int32_t v) {
        v = wave_min(v);
        if (lane_id() == 0) X->s[par][wave_id()] = v;
        __syncthreads();
        int32_t t = X->s[par][0];
#pragma unroll
        for (int w = 1; w < SW_WAVES; ++w) t = X->s[par][w] < t ? X->s[par][w] : t;
        flip();
        return t;
    }

    __device__ __forceinline__ int64_t sum(int64_t v) {
        v = wave_sum(v);
        if (lane_id() == 0) X->i[par][wave_id()][0] = v;
        __syncthreads();
        int64_t t = 0;
#pragma unroll
        for (int w = 0; w < SW_WAVES; ++w) t += X->i[par][w][0];
        flip();
        return t;
    }

    __device__ __forceinline__ void sum2(int64_t a, int64_t b, int64_t& ra, int64_t& rb) {
        a = wave_sum(a);
        b = wave_sum(b);
        if (lane_id() == 0) { X->i[par][wave_id()][0] = a; X->i[par][wave_id()][1] = b; }
        __syncthreads();
        int64_t ta = 0, tb = 0;
#pragma unroll
        for (int w = 0; w < SW_WAVES; ++w) { ta += X->i[par][w][0]; tb += X->i[par][w][1]; }
        flip();
        ra = ta;
        rb = tb;
    }

    __device__ __forceinline__ uint64_t umax(uint64_t v) {
        v = wave_max(v);
        if (lane_id() == 0) X->u[par][wave_id()] = v;
        __syncthreads();
        uint64_t m = 0;
#pragma unroll
        for (int w = 0; w < SW_WAVES; ++w) m = X->u[par][w] > m ? X->u[par][w] : m;
        flip();
        return m;
    }

    __device__ __forceinline__ double dmax(double v) {
        v = wave_max(v);
        if (lane_id() == 0) X->d[par][wave_id()][0] = v;
        __syncthreads();
        double m = X->d[par][0][0];
#pragma unroll
        for (int w = 1; w < SW_WAVES; ++w) m = X->d[par][w][0] > m ? X->d[par][w][0] : m;
        flip();
        return m;
    }

    /* sw_detsum of the per-thread partials v, and the max of m, together. */
    __device__ __forceinline__ void detsum_max(double v, double m, double& S, double& M) {
        v = wave_dettree(v);
        m = wave_max(m);
        if (lane_id() == 0) { X->d[par][wave_id()][0] = v; X->d[par][wave_id()][1] = m; }
        __syncthreads();
        double s[SW_WAVES];
        double mm = X->d[par][0][1];
#pragma unroll
        for (int w = 0; w < SW_WAVES; ++w) {
            s[w] = X->d[par][w][0];
            mm = X->d[par][w][1] > mm ? X->d[par][w][1] : mm;
        }
#pragma unroll
        for (int h = SW_WAVES / 2; h >= 1; h >>= 1)
#pragma unroll
            for (int i = 0; i < h; ++i) s[i] = s[i] + s[i + h];
        flip();
        S = s[0];
        M = mm;
    }

    __device__ __forceinline__ double detsum(double v) {
        double S, M;
        detsum_max(v, 0.0, S, M);
        return S;
    }

    /* Exclusive prefix sum over thread order; also returns the total. */
    __device__ __forceinline__ int32_t exscan(int32_t v, int32_t& total) {
        int32_t x = wave_incscan(v);
        if (lane_id() == 63) X->s[par][wave_id()] = x;
        __syncthreads();
        int32_t base = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < SW_WAVES; ++w) {
            int32_t t = X->s[par][w];
            base += (w < wave_id()) ? t : 0;
            tot += t;
        }
        flip();
        total = tot;
        return base + x - v;
    }
};
