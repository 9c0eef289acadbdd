/*
 * sw_mmf.hip — the Gavel MaxMinFairness allocation (the Fig-9 baseline,
 * SURVEY.md §8(f) row 3) as one HIP workgroup, behind sw_mmf_allocate().
 *
 * Replaces the ECOS solve of policies/max_min_fairness.py:68-93 for one worker
 * type.  The mathematics is in sw_mmf.h.  The kernel is a 512-thread
 * workgroup; thread L owns the contiguous job chunk [L·q, (L+1)·q) of the
 * deterministic sum (q = ⌈N/512⌉), so every reduction is sw_detsum and the
 * CPU twin (oracle/mmf_twin.c) returns the same bits.
 *
 *   pass 1   min_j c_j and Σ_j sf_j/c_j (one block reduction)  → t*
 *   pass 2   Σ sf_j over the pinned jobs (c_j = t*)            → free capacity
 *   ≤ 64×    μ-probe: x_j(μ) per free job (bisection in registers) and
 *            the block's sw_detsum of sf_j·x_j                 → bisection on μ bits
 *   final    x_j(μ*) written to HBM
 * Inputs are read from HBM/L2 on each probe (12 B per job); the working set
 * is a few KB, the kernel is latency-bound.
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>

#include "../../include/shockwave_amd.h"
#include "sw_block.h"
#include "sw_handle.h"
#include "sw_mmf.h"
#include "sw_mmf_lp.h"

namespace {

__global__ __launch_bounds__(SW_BLOCK) void sw_mmf_kernel(int32_t N, int32_t G,
                                                          const int32_t* __restrict__ sf,
                                                          const double* __restrict__ coef,
                                                          double* __restrict__ x,
                                                          double* __restrict__ out) {
    __shared__ sw_xchg X;
    sw_blk blk{&X, 0};
    const int32_t q = (N + SW_BLOCK - 1) / SW_BLOCK;
    const int32_t lo = (int32_t)threadIdx.x * q;
    const int32_t hi = lo + q < N ? lo + q : N;

    double part = 0.0, negmin = -INFINITY;
    for (int32_t j = lo; j < hi; ++j) {
        const double c = coef[j];
        part = part + (double)sf[j] / c;
        negmin = -c > negmin ? -c : negmin;
    }
    double S, M;
    blk.detsum_max(part, negmin, S, M);
    const double minc = -M;
    const double capb = (double)G / S;

    if (capb <= minc) { /* capacity binds: the unique optimum x_j = t* / c_j */
        for (int32_t j = lo; j < hi; ++j) x[j] = capb / coef[j];
        if (threadIdx.x == 0) { out[0] = capb; out[1] = 0.0; }
        return;
    }
    const double t = minc;
    int64_t pinned = 0;
    for (int32_t j = lo; j < hi; ++j) pinned += coef[j] <= t ? sf[j] : 0;
    const double gfree = (double)((int64_t)G - blk.sum(pinned));

    uint64_t blo = SW_MMF_MU_LO, bhi = SW_MMF_MU_HI;
    for (int it = 0; it < SW_MMF_ITERS && bhi - blo > 1; ++it) {
        const uint64_t bmid = blo + (bhi - blo) / 2;
        const double mu = sw_from_bits(bmid);
        double s = 0.0;
        for (int32_t j = lo; j < hi; ++j) {
            const double c = coef[j];
            if (c <= t) continue;
            s = s + (double)sf[j] * sw_mmf_x(c, (double)sf[j], t, mu);
        }
        const double slack = gfree - blk.detsum(s);
        if (slack > 0.0 && mu * slack >= 1.0) bhi = bmid; else blo = bmid;
    }
    const double mu = sw_from_bits(bhi);
    for (int32_t j = lo; j < hi; ++j) {
        const double c = coef[j];
        x[j] = c <= t ? 1.0 : sw_mmf_x(c, (double)sf[j], t, mu);
    }
    if (threadIdx.x == 0) { out[0] = t; out[1] = mu; }
}

/*
 * The heterogeneity-aware LP over worker types (sw_mmf_lp.h): the primal
 * simplex on a dense tableau in HBM (L2-resident at Gavel sizes: 200 jobs ×
 * 3 types is 3.2 MB).  A pivot is a rank-one update of the whole tableau, so
 * it runs on the whole GPU as two kernels chained on the stream, with the
 * simplex state in device memory and no host round trip per pivot:
 *   k_lp_select  (one workgroup) the entering column (first negative
 *                objective entry: a block min over column stripes), the
 *                leaving row (least ratio, then least basic index: a wave
 *                butterfly and an eight-way combine), the entering column's
 *                entries f_i and the divided pivot row p_j into buffers, the
 *                basis update; sets the done flag at the optimum;
 *   k_lp_update  (a workgroup per row) a_ij − f_i·p_j, the pivot row := p
 *                (rows with f_i = 0 are skipped).
 * The host enqueues pivots in chunks and reads the flag between chunks.  The
 * pivots and every element's arithmetic are oracle/mmf_twin.c's, so the
 * tableau's bits are the twin's.  (A first single-workgroup form, rows
 * updated by its eight waves, took 45 ms at 200 jobs × 3 types — 124 µs per
 * pivot of L2 latency — profiles/r7f_mmf_types_timing.json.)
 */
struct LpKey {
    double r;
    int32_t b, i;
};

__device__ __forceinline__ void lp_take(LpKey& k, const LpKey& o) {
    if (o.i >= 0 && (k.i < 0 || sw_lp_before(o.r, o.b, k.r, k.b))) k = o;
}

/* simplex state in device memory: [0] done (0 running, 1 optimal, -2 no
 * leaving row, -3 pivot cap), [1] pivots, [2] pivot row r, [3] entering e */
struct LpState {
    int64_t done, piv, r, e;
};

constexpr int kLpTB = 256;

__global__ __launch_bounds__(kLpTB) void k_lp_init(int32_t m, int32_t n, const int32_t* workers, const int32_t* sf,
                                                   const double* coef, double* a, int32_t* basis, LpState* st) {
    const sw_lp_dims d = sw_lp_dims_of(m, n);
    const int64_t W = d.W, cells = ((int64_t)d.R + 1) * W;
    const int64_t g = (int64_t)blockIdx.x * kLpTB + threadIdx.x, stride = (int64_t)gridDim.x * kLpTB;
    for (int64_t e = g; e < cells; e += stride) a[e] = sw_lp_init(&d, workers, sf, coef, (int32_t)(e / W), (int32_t)(e % W));
    for (int64_t i = g; i < d.R; i += stride) basis[i] = m * n + 1 + (int32_t)i;
    if (g == 0) { st->done = 0; st->piv = 0; st->r = -1; st->e = -1; }
}

__global__ __launch_bounds__(SW_BLOCK) void k_lp_select(int32_t m, int32_t n, const double* a, int32_t* basis,
                                                        double* f, double* p, LpState* st) {
    __shared__ sw_xchg X;
    __shared__ LpKey wk[SW_WAVES];
    __shared__ int32_t sr;
    if (st->done != 0) return; /* uniform: the optimum (or a stop) was reached */
    const int64_t piv0 = st->piv; /* read once: thread 0 advances it below */
    sw_blk blk{&X, 0};
    const sw_lp_dims d = sw_lp_dims_of(m, n);
    const int64_t W = d.W, R1 = (int64_t)d.R + 1;
    const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
    const double* obj = a + (int64_t)d.R * W;
    int32_t el = 0x7FFFFFFF;
    for (int32_t c = tid; c < d.C; c += SW_BLOCK)
        if (obj[c] < -SW_LP_EPS) { el = c; break; }
    const int32_t e = blk.min32(el);
    if (e == 0x7FFFFFFF) {
        if (tid == 0) st->done = 1;
        return;
    }
    LpKey k;
    k.r = 0.0; k.b = 0; k.i = -1;
    for (int32_t i = tid; i < d.R; i += SW_BLOCK) {
        const double v = a[(int64_t)i * W + e];
        if (v > SW_LP_EPS) {
            LpKey o;
            o.r = a[(int64_t)i * W + d.C] / v;
            o.b = basis[i];
            o.i = i;
            lp_take(k, o);
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        LpKey o;
        o.r = __shfl_xor(k.r, off, 64);
        o.b = __shfl_xor(k.b, off, 64);
        o.i = __shfl_xor(k.i, off, 64);
        lp_take(k, o);
    }
    if (lane == 0) wk[wv] = k;
    __syncthreads();
    if (tid == 0) {
        LpKey kk = wk[0];
        for (int w = 1; w < SW_WAVES; ++w) lp_take(kk, wk[w]);
        sr = kk.i;
    }
    __syncthreads();
    const int32_t r = sr;
    if (r < 0 || piv0 + 1 > sw_lp_max_pivots(&d)) {
        if (tid == 0) st->done = r < 0 ? -2 : -3;
        return;
    }
    for (int64_t i = tid; i < R1; i += SW_BLOCK) f[i] = a[i * W + e];
    const double pe = a[(int64_t)r * W + e];
    for (int64_t c = tid; c < W; c += SW_BLOCK) p[c] = a[(int64_t)r * W + c] / pe;
    if (tid == 0) {
        basis[r] = e;
        st->piv = piv0 + 1;
        st->r = r;
        st->e = e;
    }
}

__global__ __launch_bounds__(kLpTB) void k_lp_update(int32_t m, int32_t n, double* a, const double* f, const double* p,
                                                     const LpState* st) {
    if (st->done != 0) return;
    const sw_lp_dims d = sw_lp_dims_of(m, n);
    const int64_t W = d.W, i = blockIdx.x;
    const int64_t r = st->r;
    double* ai = a + i * W;
    if (i == r) {
        for (int64_t c = threadIdx.x; c < W; c += kLpTB) ai[c] = p[c];
        return;
    }
    const double fi = f[i];
    if (fi == 0.0) return;
    for (int64_t c = threadIdx.x; c < W; c += kLpTB) ai[c] = ai[c] - fi * p[c];
}

__global__ __launch_bounds__(SW_BLOCK) void k_lp_result(int32_t m, int32_t n, const double* a, const int32_t* basis,
                                                        const LpState* st, double* x, double* out) {
    const sw_lp_dims d = sw_lp_dims_of(m, n);
    const int64_t W = d.W;
    const int tid = threadIdx.x;
    for (int32_t j = tid; j < m * n; j += SW_BLOCK) x[j] = 0.0;
    if (tid == 0) out[0] = 0.0;
    __syncthreads();
    for (int32_t i = tid; i < d.R; i += SW_BLOCK) {
        const int32_t b = basis[i];
        const double v = a[(int64_t)i * W + d.C];
        if (b < m * n) x[b] = v;
        else if (b == m * n) out[0] = v;
    }
    if (tid == 0) {
        out[1] = (double)st->piv;
        out[2] = (double)(st->done == 1 ? 0 : st->done);
    }
}

struct MmfBufs {
    DevBuf<int32_t> sf;
    DevBuf<double> c, x, out;
    HostBuf<int32_t> hsf;
    HostBuf<double> hc, hx, hout;
    /* the LP over worker types */
    DevBuf<int32_t> lw, lsf, lbasis;
    DevBuf<double> lc, lx, lout, tab, lf, lp;
    DevBuf<LpState> lst;
    HostBuf<LpState> hlst;
    HostBuf<int32_t> hlw, hlsf;
    HostBuf<double> hlc, hlx, hlout;
};

int mmf_fail(sw_handle* h, int code, const std::string& msg) {
    h->err = msg;
    return code;
}

#define MMF_HIP(h, call)                                                                     \
    do {                                                                                     \
        hipError_t _e = (call);                                                              \
        if (_e != hipSuccess)                                                                \
            return mmf_fail((h), SW_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(_e)); \
    } while (0)

}  // namespace

void sw_mmf_release(sw_handle* h) {
    if (!h || !h->mmf) return;
    MmfBufs* b = (MmfBufs*)h->mmf;
    b->sf.release(); b->c.release(); b->x.release(); b->out.release();
    b->hsf.release(); b->hc.release(); b->hx.release(); b->hout.release();
    b->lw.release(); b->lsf.release(); b->lc.release(); b->lx.release(); b->lout.release(); b->tab.release();
    b->lbasis.release(); b->lf.release(); b->lp.release(); b->lst.release(); b->hlst.release();
    b->hlw.release(); b->hlsf.release(); b->hlc.release(); b->hlx.release(); b->hlout.release();
    delete b;
    h->mmf = nullptr;
}

extern "C" int sw_mmf_allocate(sw_handle* h, int32_t num_jobs, int32_t num_workers,
                               const int32_t* scale_factors, const double* coefficients,
                               double* allocation, double* level) {
    if (!h) return SW_ERR_INVALID;
    if (num_jobs < 0 || num_workers <= 0 || (num_jobs > 0 && (!scale_factors || !coefficients ||
                                                              !allocation)))
        return mmf_fail(h, SW_ERR_INVALID, "sw_mmf_allocate: bad sizes or null pointers");
    for (int32_t j = 0; j < num_jobs; ++j) {
        const double c = coefficients[j];
        if (scale_factors[j] < 1 || scale_factors[j] > SW_MAX_WIDTH || !(c > 0.0) || !isfinite(c))
            return mmf_fail(h, SW_ERR_INVALID,
                            "sw_mmf_allocate: scale factors must be in [1,255] and "
                            "coefficients finite and > 0");
    }
    if (level) { level[0] = 0.0; level[1] = 0.0; }
    if (num_jobs == 0) return SW_OK; /* policy.flatten returns None (policy.py:20-22) */
    MMF_HIP(h, hipSetDevice(h->device));
    if (!h->mmf) h->mmf = new MmfBufs();
    MmfBufs* b = (MmfBufs*)h->mmf;
    const size_t n = (size_t)num_jobs;
    MMF_HIP(h, b->sf.reserve(n));
    MMF_HIP(h, b->c.reserve(n));
    MMF_HIP(h, b->x.reserve(n));
    MMF_HIP(h, b->out.reserve(2));
    MMF_HIP(h, b->hsf.reserve(n));
    MMF_HIP(h, b->hc.reserve(n));
    MMF_HIP(h, b->hx.reserve(n));
    MMF_HIP(h, b->hout.reserve(2));
    memcpy(b->hsf.p, scale_factors, n * sizeof(int32_t));
    memcpy(b->hc.p, coefficients, n * sizeof(double));
    MMF_HIP(h, hipMemcpyAsync(b->sf.p, b->hsf.p, n * sizeof(int32_t), hipMemcpyHostToDevice,
                              h->stream));
    MMF_HIP(h, hipMemcpyAsync(b->c.p, b->hc.p, n * sizeof(double), hipMemcpyHostToDevice,
                              h->stream));
    hipLaunchKernelGGL(sw_mmf_kernel, dim3(1), dim3(SW_BLOCK), 0, h->stream, num_jobs,
                       num_workers, b->sf.p, b->c.p, b->x.p, b->out.p);
    MMF_HIP(h, hipGetLastError());
    MMF_HIP(h, hipMemcpyAsync(b->hx.p, b->x.p, n * sizeof(double), hipMemcpyDeviceToHost,
                              h->stream));
    MMF_HIP(h, hipMemcpyAsync(b->hout.p, b->out.p, 2 * sizeof(double), hipMemcpyDeviceToHost,
                              h->stream));
    MMF_HIP(h, hipStreamSynchronize(h->stream));
    memcpy(allocation, b->hx.p, n * sizeof(double));
    if (level) { level[0] = b->hout.p[0]; level[1] = b->hout.p[1]; }
    return SW_OK;
}

extern "C" int sw_mmf_allocate_types(sw_handle* h, int32_t num_jobs, int32_t num_types,
                                     const int32_t* workers, const int32_t* scale_factors,
                                     const double* coefficients, double* allocation, double* level) {
    if (!h) return SW_ERR_INVALID;
    if (num_jobs < 0 || num_jobs > SW_LP_MAX_JOBS || num_types < 1 || num_types > SW_LP_MAX_TYPES ||
        !workers || (num_jobs > 0 && (!scale_factors || !coefficients || !allocation)))
        return mmf_fail(h, SW_ERR_INVALID, "sw_mmf_allocate_types: bad sizes or null pointers");
    for (int32_t k = 0; k < num_types; ++k)
        if (workers[k] < 0)
            return mmf_fail(h, SW_ERR_INVALID, "sw_mmf_allocate_types: worker counts must be >= 0");
    for (int32_t j = 0; j < num_jobs; ++j) {
        if (scale_factors[j] < 1 || scale_factors[j] > SW_MAX_WIDTH)
            return mmf_fail(h, SW_ERR_INVALID, "sw_mmf_allocate_types: scale factors must be in [1,255]");
        for (int32_t k = 0; k < num_types; ++k) {
            const double c = coefficients[(size_t)j * num_types + k];
            if (!(c >= 0.0) || !isfinite(c))
                return mmf_fail(h, SW_ERR_INVALID,
                                "sw_mmf_allocate_types: coefficients must be finite and >= 0");
        }
    }
    if (level) { level[0] = 0.0; level[1] = 0.0; }
    if (num_jobs == 0) return SW_OK; /* policy.flatten returns None (policy.py:28-33) */
    const sw_lp_dims d = sw_lp_dims_of(num_jobs, num_types);
    const size_t cells = (size_t)(d.R + 1) * (size_t)d.W;
    if (cells * sizeof(double) > ((size_t)1 << 28))
        return mmf_fail(h, SW_ERR_CAPACITY, "sw_mmf_allocate_types: tableau above 256 MB");
    MMF_HIP(h, hipSetDevice(h->device));
    if (!h->mmf) h->mmf = new MmfBufs();
    MmfBufs* b = (MmfBufs*)h->mmf;
    const size_t m = (size_t)num_jobs, mn = m * (size_t)num_types;
    MMF_HIP(h, b->lw.reserve((size_t)num_types));
    MMF_HIP(h, b->lsf.reserve(m));
    MMF_HIP(h, b->lc.reserve(mn));
    MMF_HIP(h, b->lx.reserve(mn));
    MMF_HIP(h, b->lout.reserve(4));
    MMF_HIP(h, b->tab.reserve(cells));
    MMF_HIP(h, b->lbasis.reserve((size_t)d.R));
    MMF_HIP(h, b->lf.reserve((size_t)d.R + 1));
    MMF_HIP(h, b->lp.reserve((size_t)d.W));
    MMF_HIP(h, b->lst.reserve(1));
    MMF_HIP(h, b->hlst.reserve(1));
    MMF_HIP(h, b->hlw.reserve((size_t)num_types));
    MMF_HIP(h, b->hlsf.reserve(m));
    MMF_HIP(h, b->hlc.reserve(mn));
    MMF_HIP(h, b->hlx.reserve(mn));
    MMF_HIP(h, b->hlout.reserve(4));
    memcpy(b->hlw.p, workers, (size_t)num_types * sizeof(int32_t));
    memcpy(b->hlsf.p, scale_factors, m * sizeof(int32_t));
    memcpy(b->hlc.p, coefficients, mn * sizeof(double));
    hipStream_t st = h->stream;
    MMF_HIP(h, hipMemcpyAsync(b->lw.p, b->hlw.p, (size_t)num_types * 4, hipMemcpyHostToDevice, st));
    MMF_HIP(h, hipMemcpyAsync(b->lsf.p, b->hlsf.p, m * 4, hipMemcpyHostToDevice, st));
    MMF_HIP(h, hipMemcpyAsync(b->lc.p, b->hlc.p, mn * 8, hipMemcpyHostToDevice, st));
    const unsigned gi = (unsigned)std::min<size_t>((cells + kLpTB - 1) / kLpTB, 4096);
    hipLaunchKernelGGL(k_lp_init, dim3(gi), dim3(kLpTB), 0, st, num_jobs, num_types, b->lw.p, b->lsf.p, b->lc.p,
                       b->tab.p, b->lbasis.p, b->lst.p);
    MMF_HIP(h, hipGetLastError());
    /* pivots in chunks, the done flag read between them */
    constexpr int kChunk = 32;
    const int64_t maxp = sw_lp_max_pivots(&d);
    for (int64_t done_piv = 0;; done_piv += kChunk) {
        for (int q = 0; q < kChunk; ++q) {
            hipLaunchKernelGGL(k_lp_select, dim3(1), dim3(SW_BLOCK), 0, st, num_jobs, num_types, b->tab.p,
                               b->lbasis.p, b->lf.p, b->lp.p, b->lst.p);
            hipLaunchKernelGGL(k_lp_update, dim3((unsigned)(d.R + 1)), dim3(kLpTB), 0, st, num_jobs, num_types,
                               b->tab.p, b->lf.p, b->lp.p, b->lst.p);
        }
        MMF_HIP(h, hipGetLastError());
        MMF_HIP(h, hipMemcpyAsync(b->hlst.p, b->lst.p, sizeof(LpState), hipMemcpyDeviceToHost, st));
        MMF_HIP(h, hipStreamSynchronize(st));
        if (b->hlst.p->done != 0 || done_piv > maxp) break;
    }
    hipLaunchKernelGGL(k_lp_result, dim3(1), dim3(SW_BLOCK), 0, st, num_jobs, num_types, b->tab.p, b->lbasis.p,
                       b->lst.p, b->lx.p, b->lout.p);
    MMF_HIP(h, hipGetLastError());
    MMF_HIP(h, hipMemcpyAsync(b->hlx.p, b->lx.p, mn * 8, hipMemcpyDeviceToHost, st));
    MMF_HIP(h, hipMemcpyAsync(b->hlout.p, b->lout.p, 3 * 8, hipMemcpyDeviceToHost, st));
    MMF_HIP(h, hipStreamSynchronize(st));
    const int status = (int)b->hlout.p[2];
    if (status != 0)
        return mmf_fail(h, SW_ERR_CAPACITY,
                        status == -3 ? "sw_mmf_allocate_types: pivot cap reached"
                                     : "sw_mmf_allocate_types: no leaving row (unbounded)");
    memcpy(allocation, b->hlx.p, mn * sizeof(double));
    if (level) { level[0] = b->hlout.p[0]; level[1] = b->hlout.p[1]; }
    return SW_OK;
}
