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

/* ---- the heterogeneity-aware LP over worker types (sw_mmf_lp.h) ---------- */
#include <stdlib.h>

#include "../shockwave-replication_amd/csrc/sw_mmf_lp.h"

/* The kernel's pivots, one after the other (sw_mmf.hip sw_mmf_lp_kernel).
 * x: m·n doubles (row-major), level[0] = t*; *pivots the pivots taken.
 * Returns 0, or -2 (no leaving row: cannot happen on this bounded LP) /
 * -3 (pivot cap) / -1 (allocation). */
int mmf_twin_allocate_types(int32_t m, int32_t n, const int32_t* workers, const int32_t* sf,
                            const double* coef, double* x, double* level, int64_t* pivots) {
    const sw_lp_dims d = sw_lp_dims_of(m, n);
    const size_t W = (size_t)d.W, R1 = (size_t)d.R + 1;
    double* a = (double*)malloc(R1 * W * sizeof(double));
    double* f = (double*)malloc(R1 * sizeof(double));
    int32_t* basis = (int32_t*)malloc((size_t)(d.R > 0 ? d.R : 1) * sizeof(int32_t));
    if (!a || !f || !basis) { free(a); free(f); free(basis); return -1; }
    for (size_t i = 0; i < R1; ++i)
        for (size_t c = 0; c < W; ++c) a[i * W + c] = sw_lp_init(&d, workers, sf, coef, (int32_t)i, (int32_t)c);
    for (int32_t i = 0; i < d.R; ++i) basis[i] = m * n + 1 + i;
    const int64_t maxp = sw_lp_max_pivots(&d);
    int64_t piv = 0;
    int rc = 0;
    const double* obj = a + (size_t)d.R * W;
    for (;;) {
        int32_t e = -1;
        for (int32_t c = 0; c < d.C; ++c)
            if (obj[c] < -SW_LP_EPS) { e = c; break; }
        if (e < 0) break; /* optimal */
        int32_t r = -1, bb = 0;
        double rb = 0.0;
        for (int32_t i = 0; i < d.R; ++i) {
            const double v = a[(size_t)i * W + e];
            if (v > SW_LP_EPS) {
                const double ratio = a[(size_t)i * W + d.C] / v;
                if (r < 0 || sw_lp_before(ratio, basis[i], rb, bb)) { r = i; rb = ratio; bb = basis[i]; }
            }
        }
        if (r < 0) { rc = -2; break; }
        if (++piv > maxp) { rc = -3; break; }
        for (size_t i = 0; i < R1; ++i) f[i] = a[i * W + (size_t)e];
        const double pe = f[r];
        double* pr = a + (size_t)r * W;
        for (size_t c = 0; c < W; ++c) pr[c] = pr[c] / pe;
        for (size_t i = 0; i < R1; ++i) {
            const double fi = f[i];
            if ((int32_t)i == r || fi == 0.0) continue;
            double* ai = a + i * W;
            for (size_t c = 0; c < W; ++c) ai[c] = ai[c] - fi * pr[c];
        }
        basis[r] = e;
    }
    double t = 0.0;
    for (int32_t j = 0; j < m * n; ++j) x[j] = 0.0;
    for (int32_t i = 0; i < d.R; ++i) {
        const double v = a[(size_t)i * W + d.C];
        if (basis[i] < m * n) x[basis[i]] = v;
        else if (basis[i] == m * n) t = v;
    }
    level[0] = t;
    *pivots = piv;
    free(a); free(f); free(basis);
    return rc;
}
