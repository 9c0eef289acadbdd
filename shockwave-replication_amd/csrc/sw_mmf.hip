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

#include <string>

#include "../../include/shockwave_amd.h"
#include "sw_block.h"
#include "sw_handle.h"
#include "sw_mmf.h"

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

struct MmfBufs {
    DevBuf<int32_t> sf;
    DevBuf<double> c, x, out;
    HostBuf<int32_t> hsf;
    HostBuf<double> hc, hx, hout;
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
