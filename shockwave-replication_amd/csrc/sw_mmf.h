/*
 * sw_mmf.h — per-job arithmetic of the Gavel MaxMinFairness allocation,
 * shared by the HIP kernel (sw_mmf.hip) and its CPU twin (oracle/mmf_twin.c).
 *
 * The reference baseline (policies/max_min_fairness.py:14-95, policy.py:57-63,
 * proportional.py:27-44) solves, with ECOS, for one worker type:
 *
 *     maximise  min_j c_j·x_j
 *     s.t.      Σ_j sf_j·x_j ≤ G,   0 ≤ x_j ≤ 1,
 *
 * with c_j = sf_j / priority_weight_j (MaxMinFairnessPolicy sets every
 * throughput to 1.0, so every proportional throughput is 1.0).
 *
 * The optimum level is closed-form: t* = min(min_j c_j, G / Σ_j sf_j/c_j).
 *   - If G / Σ sf/c ≤ min c, capacity binds and x_j = t* / c_j is the unique optimum.
 *   - Otherwise t* = min c: jobs with c_j = t* are pinned at x_j = 1 and the
 *     optimal face leaves every other x_j free in [t* / c_j, 1] under
 *     Σ sf·x ≤ G.  An interior-point solver (ECOS) ends at the analytic
 *     centre of that face, the maximiser of
 *         Σ_free [log x_j + log(1 − x_j) + log(c_j x_j − t*)] + log(G − Σ sf x).
 *     Its stationarity condition per free job is h_j(x_j) = sf_j·μ with
 *         h_j(x) = 1/x − 1/(1−x) + c_j/(c_j x − t*),  μ = 1/(G − Σ sf x);
 *     h_j is strictly decreasing, so x_j(μ) is a bisection, and μ is the
 *     smallest value with μ·slack(μ) ≥ 1 — a bisection over the bits of μ.
 *
 * Only IEEE +, −, ×, ÷ and comparisons (no transcendental functions), with
 * -ffp-contract=off on both sides, and the slack sum is sw_detsum: the GPU
 * and the twin produce the same bits.
 */
#ifndef SW_MMF_H
#define SW_MMF_H

#include "sw_arith.h"

/* μ is searched over [2^-64, 2^64] (G ≤ 2^31, so 1/G > 2^-64) */
#define SW_MMF_MU_LO 0x3BF0000000000000ull /* 2^-64 */
#define SW_MMF_MU_HI 0x43F0000000000000ull /* 2^64  */
#define SW_MMF_ITERS 64

/* x_j(μ): the root of h_j(x) = sf·μ on (t/c, 1), by bisection to adjacent
 * doubles. */
SW_HD double sw_mmf_x(double c, double sf, double t, double mu) {
    double lo = t / c, hi = 1.0;
    const double target = sf * mu;
    for (int it = 0; it < SW_MMF_ITERS; ++it) {
        double mid = (lo + hi) * 0.5;
        if (!(mid > lo && mid < hi)) break;
        double den = c * mid - t;
        int up;
        if (den <= 0.0) {
            up = 1;
        } else {
            double h = 1.0 / mid - 1.0 / (1.0 - mid) + c / den;
            up = h > target;
        }
        if (up) lo = mid; else hi = mid;
    }
    return (lo + hi) * 0.5;
}

#endif /* SW_MMF_H */
