/*
 * sw_mmf_lp.h — the heterogeneity-aware MaxMinFairness LP over several worker
 * types (policies/max_min_fairness.py:44-100, MaxMinFairnessPolicyWithPerf;
 * base constraints policy.py:57-63), solved by the primal simplex method on a
 * dense tableau.  Shared by the HIP kernel (sw_mmf.hip, one workgroup, the
 * tableau in HBM/L2) and the CPU twin (oracle/mmf_twin.c), which run the same
 * pivots with the same per-element arithmetic (-ffp-contract=off), so they
 * return the same bits.
 *
 * The LP, m jobs × n worker types, x[j][k] = share of time job j runs on
 * type k (coef[j][k] = throughput · priority weight · scale factor, the
 * caller's normalisation, max_min_fairness.py:57-73):
 *     maximise t
 *     s.t.  t − Σ_k coef[j][k]·x[j][k] ≤ 0      (m value rows)
 *           Σ_j sf_j·x[j][k] ≤ workers[k]       (n capacity rows)
 *           Σ_k x[j][k] ≤ 1                     (m time rows)
 *           x ≥ 0, t ≥ 0
 * Tableau: rows 0 … R−1 the constraints (value rows, capacity rows, time rows;
 * R = 2m + n), row R the objective (z − c form: −1 under t); columns x[j][k]
 * at j·n + k, t at m·n, the slack of row i at m·n + 1 + i, the right-hand
 * side last (row stride SW_LP_W = m·n + 2 + R).  The slack basis is feasible
 * (right-hand sides 0, workers, 1).
 *
 * Pivot rule (Bland's, so no cycling on this degenerate LP — every value row
 * starts tight at t = 0): the entering column is the lowest index whose
 * objective entry is below −SW_LP_EPS; the leaving row is the one of least
 * ratio rhs_i / a_ie over a_ie > SW_LP_EPS, ties to the lowest basic
 * variable index.  A pivot divides the pivot row by the pivot element
 * (p_j = a_rj / a_re), then every other row i subtracts f_i·p_j with f_i its
 * entry in the entering column before the pivot.  The optimum found is a
 * vertex of the LP: its level t* is the LP's (unique) optimum; the allocation
 * is one optimal vertex (the reference's ECOS returns an interior point of
 * the same optimal face, so allocations agree only where the optimum is
 * unique — tests/test_mmf.py checks the level against HiGHS and the
 * allocation for feasibility and optimality).
 */
#ifndef SW_MMF_LP_H
#define SW_MMF_LP_H

#include "sw_arith.h"

#define SW_LP_EPS 1e-11
#define SW_LP_MAX_TYPES 16    /* worker types the call accepts */
#define SW_LP_MAX_JOBS 2048   /* jobs (the tableau: (2m + n + 1)·(m·n + 2m + n + 2) doubles) */

typedef struct {
    int32_t m, n, R, C, W; /* jobs, types, constraint rows, columns (no rhs), row stride */
} sw_lp_dims;

SW_HD sw_lp_dims sw_lp_dims_of(int32_t m, int32_t n) {
    sw_lp_dims d;
    d.m = m;
    d.n = n;
    d.R = 2 * m + n;
    d.C = m * n + 1 + d.R;
    d.W = d.C + 1;
    return d;
}

/* Entry (i, c) of the initial tableau. */
SW_HD double sw_lp_init(const sw_lp_dims* d, const int32_t* workers, const int32_t* sf,
                        const double* coef, int32_t i, int32_t c) {
    const int32_t m = d->m, n = d->n, tcol = m * n, rhs = d->C;
    if (i == d->R) return c == tcol ? -1.0 : 0.0; /* objective: maximise t */
    if (c == tcol + 1 + i) return 1.0;            /* the row's slack */
    if (i < m) {                                  /* value row of job i */
        if (c == tcol) return 1.0;
        if (c >= i * n && c < (i + 1) * n) return -coef[c];
        return 0.0;
    }
    if (i < m + n) { /* capacity row of type k */
        const int32_t k = i - m;
        if (c == rhs) return (double)workers[k];
        if (c < tcol && c % n == k) return (double)sf[c / n];
        return 0.0;
    }
    { /* time row of job j */
        const int32_t j = i - m - n;
        if (c == rhs) return 1.0;
        if (c >= j * n && c < (j + 1) * n) return 1.0;
        return 0.0;
    }
}

/* the leaving-row order: smaller ratio, then smaller basic variable */
SW_HD int sw_lp_before(double r, int32_t b, double rb, int32_t bb) {
    return r < rb || (r == rb && b < bb);
}

/* pivots the call may take before it gives up (SW_ERR_CAPACITY) */
SW_HD int64_t sw_lp_max_pivots(const sw_lp_dims* d) { return 50 * (int64_t)(d->R + d->C) + 1000; }

#endif /* SW_MMF_LP_H */
