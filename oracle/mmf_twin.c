/*
 * oracle/mmf_twin.c — TEST INFRASTRUCTURE: CPU bit-exact twin of the
 * MaxMinFairness allocation kernel (shockwave-replication_amd/csrc/sw_mmf.hip).
 *
 * Same algorithm, same per-job arithmetic (sw_mmf.h, -ffp-contract=off) and
 * the same deterministic job sums (sw_detsum), so it returns the bits the GPU
 * returns.  It is pinned against the LP itself by tests/test_mmf.py: the
 * optimum level t* matches scipy's HiGHS solution of the reference's LP
 * (policies/max_min_fairness.py:68-93) and the allocation satisfies the
 * analytic-centre optimality conditions.  Never linked into the product.
 */
#include <math.h>
#include <stdint.h>

#include "../shockwave-replication_amd/csrc/sw_mmf.h"

static double detsum(const double* v, int32_t N) {
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

/* v is caller scratch of N doubles */
int mmf_twin_allocate(int32_t N, int32_t G, const int32_t* sf, const double* c, double* x,
                      double* level, double* v) {
    if (N <= 0) {
        if (level) { level[0] = 0.0; level[1] = 0.0; }
        return 0;
    }
    double minc = INFINITY;
    for (int32_t j = 0; j < N; ++j) {
        v[j] = (double)sf[j] / c[j];
        minc = c[j] < minc ? c[j] : minc;
    }
    const double capb = (double)G / detsum(v, N);
    if (capb <= minc) {
        for (int32_t j = 0; j < N; ++j) x[j] = capb / c[j];
        if (level) { level[0] = capb; level[1] = 0.0; }
        return 0;
    }
    const double t = minc;
    int64_t pinned = 0;
    for (int32_t j = 0; j < N; ++j) pinned += c[j] <= t ? sf[j] : 0;
    const double gfree = (double)((int64_t)G - pinned);
    uint64_t blo = SW_MMF_MU_LO, bhi = SW_MMF_MU_HI;
    for (int it = 0; it < SW_MMF_ITERS && bhi - blo > 1; ++it) {
        const uint64_t bmid = blo + (bhi - blo) / 2;
        const double mu = sw_from_bits(bmid);
        for (int32_t j = 0; j < N; ++j)
            v[j] = c[j] <= t ? 0.0 : (double)sf[j] * sw_mmf_x(c[j], (double)sf[j], t, mu);
        const double slack = gfree - detsum(v, N);
        if (slack > 0.0 && mu * slack >= 1.0) bhi = bmid; else blo = bmid;
    }
    const double mu = sw_from_bits(bhi);
    for (int32_t j = 0; j < N; ++j) x[j] = c[j] <= t ? 1.0 : sw_mmf_x(c[j], (double)sf[j], t, mu);
    if (level) { level[0] = t; level[1] = mu; }
    return 0;
}
