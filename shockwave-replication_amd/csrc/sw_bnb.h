/*
 * sw_bnb.h — the level search's branch and bound over makespan levels
 * (DESIGN.md §3.3), shared by the HIP kernels (sw_kernels.hip), the sharded
 * controller (sw_shard_ctl.h) and the CPU twin (oracle/plan_twin.c).  Plain
 * C99 + HIP qualifiers.
 *
 * P1 (shockwave.py:330-382) is max over plans of U − k·makespan.  With
 * V(θ) = the best utility of a plan whose makespan is at most θ, the optimum
 * is max_θ V(θ) − k·θ over the finitely many levels θ = g_j(n).  V is
 * nondecreasing, so every plan whose makespan lies in (a, b] has
 *     J ≤ V(b) − k·a ≤ Vub(b) − k·a,
 * Vub(b) being the Lagrangian bound SELECT(b) returns (its ubound: the
 * concave relaxation at the price ρ*(b)).  The search keeps a list of open
 * level intervals (a, b] with Vub(b) known, splits the one of largest bound at
 * its midpoint (one SELECT), and drops every interval whose bound does not
 * beat the best plan found.  When the list empties the level search is exact
 * relative to SELECT; the largest bound it leaves is a certified upper bound
 * on the aggregate P1 optimum (and so on the reference MILP's).
 *
 * This replaces a golden-section search that assumed J unimodal in the level:
 * on small or lumpy instances it is not (tests/golden/frag_fuzz.json seed
 * 50115: the best level lies below a local optimum the golden section stays
 * in), and on small-k configurations the golden section ran its 32 steps
 * where a handful of bounded probes prove the utility-only level optimal.
 */
#ifndef SW_BNB_H
#define SW_BNB_H

#include "sw_arith.h"

/* probes after M_lo and +∞ — the golden section's worst case (2 + 32) */
#define SW_BNB_PROBES 34
#define SW_BNB_CAP (SW_BNB_PROBES + 1)

typedef struct {
    double a, b; /* the open interval (a, b] of levels */
    double vb;   /* Vub(b): SELECT(b)'s ubound (a bound on V over the interval) */
    uint32_t ra, rb; /* ρ*(a) and a lower bound of ρ*(b): the price bracket of any probe inside */
    uint32_t pad_;
} sw_bnb_ivl;

/* the bound of every plan with makespan in (a, b] */
SW_HD double sw_bnb_key(double vb, double k, double a) { return vb - k * a; }

SW_HD double sw_bnb_mid(double a, double b) { return a + (b - a) * 0.5; }

/* index of the interval to split next: the first one of largest key */
SW_HD int32_t sw_bnb_pick(const sw_bnb_ivl* L, int32_t n, double k, double* key) {
    int32_t bi = 0;
    double bk = sw_bnb_key(L[0].vb, k, L[0].a);
    for (int32_t i = 1; i < n; ++i) {
        const double x = sw_bnb_key(L[i].vb, k, L[i].a);
        if (x > bk) { bk = x; bi = i; }
    }
    *key = bk;
    return bi;
}

SW_HD sw_bnb_ivl sw_bnb_make(double a, double b, double vb, uint32_t ra, uint32_t rb) {
    sw_bnb_ivl v;
    v.a = a;
    v.b = b;
    v.vb = vb;
    v.ra = ra;
    v.rb = rb;
    v.pad_ = 0u;
    return v;
}

/* Result status: the plan's objective is not certified within the north
 * star's 1e-3 of the returned bound (SW_STATUS_P1_UNCERTIFIED). */
SW_HD int sw_p1_uncertified(double J, double bound) {
    const double aj = J < 0.0 ? -J : J;
    return (bound - J) > 1e-3 * aj;
}

#endif /* SW_BNB_H */
