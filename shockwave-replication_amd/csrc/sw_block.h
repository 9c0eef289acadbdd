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

/* NW waves per workgroup: SW_WAVES for the plan kernel; the sharded
 * engine's placement also runs a 1024-thread (16-wave) round loop */
template <int NW>
struct sw_xchg_t {
    int64_t i[2][NW][2];
    double d[2][NW][2];
    uint64_t u[2][NW];
    uint64_t u2[2][NW][2];
    int32_t s[2][NW];
};
using sw_xchg = sw_xchg_t<SW_WAVES>;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

/* Block-reduction results are workgroup-uniform: they are returned through
 * v_readfirstlane so that the compiler keeps them (and what is derived from
 * them) in SGPRs instead of VGPRs — in the register-capped kernels uniform
 * state held per lane was spilled to scratch. */
__device__ __forceinline__ int32_t sw_u32(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t sw_u64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int64_t sw_i64(int64_t x) { return (int64_t)sw_u64((uint64_t)x); }
__device__ __forceinline__ double sw_f64u(double x) {
    return __builtin_bit_cast(double, sw_u64(__builtin_bit_cast(uint64_t, x)));
}

/* Order LDS accesses of one wave (the hardware keeps a wave's LDS ops in
 * order; this keeps the compiler from moving them). */
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

/* ---- DPP (data-parallel primitives) integer scans ----------------------
 * Hillis-Steele inside each 16-lane row with row_shr:1/2/4/8, then
 * row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) — the GFX9-family
 * cross-row steps that gfx950 keeps.  Each step is one v_add with a DPP
 * source operand (a few cycles), instead of a ds_bpermute round trip
 * through the LDS crossbar.  Integer ops only (associative, so the order
 * does not matter). */
__device__ __forceinline__ int32_t dpp_incscan_i32(int32_t x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false); /* row_shr:1 */
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false); /* row_shr:2 */
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false); /* row_shr:4 */
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false); /* row_shr:8 */
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false); /* row_bcast:15 */
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false); /* row_bcast:31 */
    return x;
}
__device__ __forceinline__ int32_t dpp_incmax_i32(int32_t x) {
    const int32_t lo = INT32_MIN;
    int32_t y;
    y = __builtin_amdgcn_update_dpp(lo, x, 0x111, 0xF, 0xF, false); x = y > x ? y : x;
    y = __builtin_amdgcn_update_dpp(lo, x, 0x112, 0xF, 0xF, false); x = y > x ? y : x;
    y = __builtin_amdgcn_update_dpp(lo, x, 0x114, 0xF, 0xF, false); x = y > x ? y : x;
    y = __builtin_amdgcn_update_dpp(lo, x, 0x118, 0xF, 0xF, false); x = y > x ? y : x;
    y = __builtin_amdgcn_update_dpp(lo, x, 0x142, 0xA, 0xF, false); x = y > x ? y : x;
    y = __builtin_amdgcn_update_dpp(lo, x, 0x143, 0xC, 0xF, false); x = y > x ? y : x;
    return x;
}
/* wave-wide results (uniform, via v_readlane of lane 63) */
__device__ __forceinline__ int32_t wave_sum_i32(int32_t v) {
    return __builtin_amdgcn_readlane(dpp_incscan_i32(v), 63);
}
__device__ __forceinline__ int32_t wave_max_i32(int32_t v) {
    return __builtin_amdgcn_readlane(dpp_incmax_i32(v), 63);
}
__device__ __forceinline__ int32_t wave_min_i32(int32_t v) {
    return -wave_max_i32(-v);
}
/* inclusive prefix / suffix over lanes */
__device__ __forceinline__ int32_t wave_incscan_i32(int32_t v) { return dpp_incscan_i32(v); }
__device__ __forceinline__ int32_t wave_sufscan_i32(int32_t v) {
    const int32_t inc = dpp_incscan_i32(v);
    return __builtin_amdgcn_readlane(inc, 63) - inc + v;
}

/* 64-bit wave reductions on DPP: each step moves both halves with the same
 * row_shr / row_bcast pattern as the integer scans (two DPP movs) and keeps
 * the larger / smaller; lanes without a source read the identity.  Used for
 * every max / min the block reductions take (the shuffle versions below cost
 * two ds_bpermute round trips per step). */
#define SW_DPP64(x, idv, ctrl, rm)                                                              \
    ((((uint64_t)(uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)((idv) >> 32),            \
                                                       (int)(uint32_t)((x) >> 32), ctrl, rm,    \
                                                       0xF, false)) << 32) |                    \
     (uint64_t)(uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(idv), (int)(uint32_t)(x),  \
                                                     ctrl, rm, 0xF, false))
#define SW_DPP64_STEPS(STEP) STEP(0x111, 0xF) STEP(0x112, 0xF) STEP(0x114, 0xF) STEP(0x118, 0xF) \
    STEP(0x142, 0xA) STEP(0x143, 0xC)

__device__ __forceinline__ uint64_t sw_readlane63_u64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
#define SW_MAXU_(c, rm)                               \
    {                                                 \
        const uint64_t y_ = SW_DPP64(x, 0ull, c, rm); \
        x = y_ > x ? y_ : x;                          \
    }
    SW_DPP64_STEPS(SW_MAXU_)
#undef SW_MAXU_
    return sw_readlane63_u64(x);
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#define SW_MINU_(c, rm)                                \
    {                                                  \
        const uint64_t y_ = SW_DPP64(x, ~0ull, c, rm); \
        x = y_ < x ? y_ : x;                           \
    }
    SW_DPP64_STEPS(SW_MINU_)
#undef SW_MINU_
    return sw_readlane63_u64(x);
}
/* max of doubles (identity −inf) */
__device__ __forceinline__ double wave_max_f64(double v) {
    uint64_t x = __builtin_bit_cast(uint64_t, v);
#define SW_MAXD_(c, rm)                                                       \
    {                                                                         \
        const uint64_t y_ = SW_DPP64(x, 0xFFF0000000000000ull, c, rm);        \
        x = __builtin_bit_cast(double, y_) > __builtin_bit_cast(double, x) ? y_ : x; \
    }
    SW_DPP64_STEPS(SW_MAXD_)
#undef SW_MAXD_
    return __builtin_bit_cast(double, sw_readlane63_u64(x));
}

/* min of doubles (identity +inf) */
__device__ __forceinline__ double wave_min_f64(double v) {
    uint64_t x = __builtin_bit_cast(uint64_t, v);
#define SW_MIND_(c, rm)                                                       \
    {                                                                         \
        const uint64_t y_ = SW_DPP64(x, 0x7FF0000000000000ull, c, rm);        \
        x = __builtin_bit_cast(double, y_) < __builtin_bit_cast(double, x) ? y_ : x; \
    }
    SW_DPP64_STEPS(SW_MIND_)
#undef SW_MIND_
    return __builtin_bit_cast(double, sw_readlane63_u64(x));
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

/* Ascending bitonic sort of one int32 per lane across the wave. */
__device__ __forceinline__ int32_t wave_sort_asc_i32(int32_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const int32_t o = __shfl_xor(v, j, 64);
            const bool up = (lane & k) == 0;
            const bool lower = (lane & j) == 0;
            v = (lower == up) ? min(v, o) : max(v, o);
        }
    }
    return v;
}

/* Fixed halving tree over the wave (p[i] += p[i+h], h = 32 … 1); the result
 * is valid in lane 0. */
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
    const int lo = __double2loint(x), hi = __double2hiint(x);
    return __hiloint2double(__builtin_amdgcn_update_dpp(0, hi, CTRL, 0xF, 0xF, false),
                            __builtin_amdgcn_update_dpp(0, lo, CTRL, 0xF, 0xF, false));
}

/* The tree's first two levels exchange wave halves (permlane32_swap) and row
 * pairs (permlane16_swap): in the lanes that carry on, the two results are
 * p[i] and p[i+h] in some order, and their sum is p[i] + p[i+h] bit for bit
 * (IEEE addition commutes).  The last four levels are DPP row_shl.  No lane
 * address register, unlike a __shfl_down (ds_bpermute) tree, whose hoisted
 * addresses the compiler keeps live or spills across a whole kernel. */
__device__ __forceinline__ double wave_dettree(double x) {
    {
        const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
        const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        x = __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
    }
    {
        const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
        const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        x = __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
    }
    x = x + dpp_f64<0x108>(x); /* row_shl:8 */
    x = x + dpp_f64<0x104>(x); /* row_shl:4 */
    x = x + dpp_f64<0x102>(x); /* row_shl:2 */
    x = x + dpp_f64<0x101>(x); /* row_shl:1 */
    return x;
}

template <int NW>
struct sw_blk_t {
    sw_xchg_t<NW>* X;
    int par;

    __device__ __forceinline__ void flip() { par ^= 1; }

    __device__ __forceinline__ int32_t sum32(int32_t v) {
        v = wave_sum_i32(v);
        if (lane_id() == 0) X->s[par][wave_id()] = v;
        __syncthreads();
        int32_t t = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += X->s[par][w];
        flip();
        return sw_u32(t);
    }

    __device__ __forceinline__ int32_t min32(int32_t v) {
        v = wave_min_i32(v);
        if (lane_id() == 0) X->s[par][wave_id()] = v;
        __syncthreads();
        int32_t t = X->s[par][0];
#pragma unroll
        for (int w = 1; w < NW; ++w) t = X->s[par][w] < t ? X->s[par][w] : t;
        flip();
        return sw_u32(t);
    }

    /* 64-bit sums of values that fit in 32 bits per wave (all callers sum
     * weighted counts ≤ 2^31 per wave) */
    __device__ __forceinline__ int64_t sum(int64_t v) {
        const int64_t w = wave_sum_i32((int32_t)v);
        if (lane_id() == 0) X->i[par][wave_id()][0] = w;
        __syncthreads();
        int64_t t = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) t += X->i[par][k][0];
        flip();
        return sw_i64(t);
    }

    __device__ __forceinline__ void sum2(int64_t a, int64_t b, int64_t& ra, int64_t& rb) {
        a = wave_sum_i32((int32_t)a);
        b = wave_sum_i32((int32_t)b);
        if (lane_id() == 0) { X->i[par][wave_id()][0] = a; X->i[par][wave_id()][1] = b; }
        __syncthreads();
        int64_t ta = 0, tb = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) { ta += X->i[par][w][0]; tb += X->i[par][w][1]; }
        flip();
        ra = sw_i64(ta);
        rb = sw_i64(tb);
    }

    __device__ __forceinline__ uint64_t umax(uint64_t v) {
        v = wave_max_u64(v);
        if (lane_id() == 0) X->u[par][wave_id()] = v;
        __syncthreads();
        uint64_t m = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) m = X->u[par][w] > m ? X->u[par][w] : m;
        flip();
        return sw_u64(m);
    }

    __device__ __forceinline__ double dmax(double v) {
        v = wave_max_f64(v);
        if (lane_id() == 0) X->d[par][wave_id()][0] = v;
        __syncthreads();
        double m = X->d[par][0][0];
#pragma unroll
        for (int w = 1; w < NW; ++w) m = X->d[par][w][0] > m ? X->d[par][w][0] : m;
        flip();
        return sw_f64u(m);
    }

    /* Σ v (fits 32 bits per wave), max mx and min mn, one barrier. */
    __device__ __forceinline__ void sum_max_min(int64_t v, uint64_t mx, uint64_t mn, int64_t& S,
                                                uint64_t& MX, uint64_t& MN) {
        const int64_t w = wave_sum_i32((int32_t)v);
        mx = wave_max_u64(mx);
        mn = wave_min_u64(mn);
        if (lane_id() == 0) {
            X->i[par][wave_id()][0] = w;
            X->u2[par][wave_id()][0] = mx;
            X->u2[par][wave_id()][1] = mn;
        }
        __syncthreads();
        int64_t t = 0;
        uint64_t a = 0, b = ~0ull;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            t += X->i[par][k][0];
            a = X->u2[par][k][0] > a ? X->u2[par][k][0] : a;
            b = X->u2[par][k][1] < b ? X->u2[par][k][1] : b;
        }
        flip();
        S = t;
        MX = a;
        MN = b;
    }

    /* Σ v, max mx and min mn of non-negative 32-bit values, one barrier
     * (the snapped price bisection: weighted count and the two key bits
     * that bound the step of W around the probe). */
    __device__ __forceinline__ int32_t sum32_max_min(int32_t v, int32_t mx, int32_t mn, int32_t& MX,
                                                     int32_t& MN) {
        v = wave_sum_i32(v);
        mx = wave_max_i32(mx);
        mn = wave_min_i32(mn);
        if (lane_id() == 0) {
            X->i[par][wave_id()][0] = v;
            X->i[par][wave_id()][1] = (int64_t)(((uint64_t)(uint32_t)mx << 32) | (uint32_t)mn);
        }
        __syncthreads();
        int32_t t = 0, a = 0, b = 0x7FFFFFFF;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            t += (int32_t)X->i[par][w][0];
            const uint64_t p = (uint64_t)X->i[par][w][1];
            const int32_t pm = (int32_t)(p >> 32), pn = (int32_t)(uint32_t)p;
            a = pm > a ? pm : a;
            b = pn < b ? pn : b;
        }
        flip();
        MX = sw_u32(a);
        MN = sw_u32(b);
        return sw_u32(t);
    }

    /* sw_detsum of the per-thread partials v, and the max of m, together. */
    __device__ __forceinline__ void detsum_max(double v, double m, double& S, double& M) {
        v = wave_dettree(v);
        m = wave_max_f64(m);
        if (lane_id() == 0) { X->d[par][wave_id()][0] = v; X->d[par][wave_id()][1] = m; }
        __syncthreads();
        double s[NW];
        double mm = X->d[par][0][1];
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            s[w] = X->d[par][w][0];
            mm = X->d[par][w][1] > mm ? X->d[par][w][1] : mm;
        }
#pragma unroll
        for (int h = NW / 2; h >= 1; h >>= 1)
#pragma unroll
            for (int i = 0; i < h; ++i) s[i] = s[i] + s[i + h];
        flip();
        S = sw_f64u(s[0]);
        M = sw_f64u(mm);
    }

    /* sw_detsum of a and of b, the max of m ≥ 0 and the sum of the small
     * counts c, one barrier (the emit's four results) */
    __device__ __forceinline__ void detsum2_max_cnt(double a, double b, double m, int32_t c,
                                                    double& SA, double& SB, double& M, int64_t& C) {
        a = wave_dettree(a);
        b = wave_dettree(b);
        m = wave_max_f64(m);
        c = wave_sum_i32(c);
        if (lane_id() == 0) {
            X->d[par][wave_id()][0] = a;
            X->d[par][wave_id()][1] = b;
            X->i[par][wave_id()][0] = c;
            X->u[par][wave_id()] = (uint64_t)__double_as_longlong(m);
        }
        __syncthreads();
        double sa[NW], sb[NW];
        double mm = __longlong_as_double((long long)X->u[par][0]);
        int64_t t = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            sa[w] = X->d[par][w][0];
            sb[w] = X->d[par][w][1];
            const double mw = __longlong_as_double((long long)X->u[par][w]);
            mm = mw > mm ? mw : mm;
            t += X->i[par][w][0];
        }
#pragma unroll
        for (int h = NW / 2; h >= 1; h >>= 1)
#pragma unroll
            for (int i = 0; i < h; ++i) {
                sa[i] = sa[i] + sa[i + h];
                sb[i] = sb[i] + sb[i + h];
            }
        flip();
        SA = sw_f64u(sa[0]);
        SB = sw_f64u(sb[0]);
        M = sw_f64u(mm);
        C = sw_i64(t);
    }

    __device__ __forceinline__ double detsum(double v) {
        double S, M;
        detsum_max(v, 0.0, S, M);
        return S;
    }

    /* Exclusive prefix sum over thread order; also returns the total. */
    __device__ __forceinline__ int32_t exscan(int32_t v, int32_t& total) {
        int32_t x = wave_incscan_i32(v);
        if (lane_id() == 63) X->s[par][wave_id()] = x;
        __syncthreads();
        int32_t base = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            int32_t t = X->s[par][w];
            base += (w < wave_id()) ? t : 0;
            tot += t;
        }
        flip();
        total = sw_u32(tot);
        return base + x - v;
    }
};
using sw_blk = sw_blk_t<SW_WAVES>;
