/*
 * sw_arith.h — per-job arithmetic shared by the HIP kernels and the CPU
 * bit-exact twin (oracle/plan_twin.c).  Plain C99 + HIP qualifiers.
 *
 * Everything here is elementwise and uses only IEEE-754 +, -, *, /,
 * comparisons and the fp64→fp32 conversion (no transcendental functions,
 * compiled with -ffp-contract=off on both sides), so the GPU and the CPU
 * produce the same bits.  The log table and the priorities are computed by
 * the host exactly as the reference does (shockwave.py:99-105, :368) and are
 * inputs here.
 *
 * The P1 model of the reference (shockwave.py:330-388) reduces per job to
 * functions of n = Σ_t x[j][t]:
 *   e(n)  = min((Δ/d)·n, E − F)      planned epochs: d·e ≤ Δ·Σx (:126-129), and
 *                                    Σω β = (F+e)/E ≤ 1 bounds e (:173-179)
 *   u(n)  = (F + e(n)) / E           :132-134
 *   φ(u)  = adjacent-pair interpolation of log over β  (SOS2, :162-181)
 *   f(n)  = p/(N·T) · φ(u(n))        :367-377
 *   g(n)  = max(0, R − d·e(n))       :260-263
 * Both objective terms are non-decreasing in e, so the optimal e for a given
 * n is the upper bound e(n).
 */
#ifndef SW_ARITH_H
#define SW_ARITH_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define SW_HD __host__ __device__ static inline
#else
#define SW_HD static inline
#endif

#define SW_TMAX 64
#define SW_BMAX 8
/* Deterministic-reduction width: jobs are split into SW_DET_LANES contiguous
 * chunks, each summed left to right, then combined by a halving tree.  The
 * plan kernel runs exactly this many threads per instance. */
#define SW_DET_LANES 512
/* fp32 +inf bits: upper end of the price (key) bisection. */
#define SW_KEY_INF_BITS 0x7F800000u
#define SW_FLT_MIN 1.1754943508222875e-38
#define SW_FLT_MAX 3.4028234663852886e+38

typedef union { double d; uint64_t u; } sw_dbits;
typedef union { float f; uint32_t u; } sw_fbits;

SW_HD uint64_t sw_bits(double x) { sw_dbits c; c.d = x; return c.u; }
SW_HD double sw_from_bits(uint64_t u) { sw_dbits c; c.u = u; return c.d; }
SW_HD uint32_t sw_fbits_of(float x) { sw_fbits c; c.f = x; return c.u; }
SW_HD float sw_float_of(uint32_t u) { sw_fbits c; c.u = u; return c.f; }

SW_HD double sw_min(double a, double b) { return a < b ? a : b; }
SW_HD double sw_max(double a, double b) { return a > b ? a : b; }

/* Per-job constants (one division each, done once). */
typedef struct {
    double rate; /* Δ / d                  */
    double cap;  /* E − F (max epochs)     */
    double d;    /* epoch duration         */
    double R;    /* remaining runtime      */
    double a;    /* p / (N·T)              */
    double Fd;   /* F as double            */
    double Ed;   /* E as double            */
    double invE; /* 1 / E                  */
    int32_t w;   /* nworkers               */
} sw_jobc;

SW_HD sw_jobc sw_make_jobc(int32_t N, int32_t T, double delta, int32_t w, double d, int32_t F,
                           int32_t E, double R, double p) {
    sw_jobc c;
    c.rate = delta / d;
    c.cap = (double)(E - F);
    c.d = d;
    c.R = R;
    c.a = p / ((double)N * (double)T);
    c.Fd = (double)F;
    c.Ed = (double)E;
    c.invE = 1.0 / (double)E;
    c.w = w;
    return c;
}

/* e(n) — planned epochs with n planned rounds. */
SW_HD double sw_e(const sw_jobc* c, int32_t n) {
    double e = c->rate * (double)n;
    return e < c->cap ? e : c->cap;
}

/* g(n) — the job's makespan term max(0, R − d·e). */
SW_HD double sw_g(const sw_jobc* c, int32_t n) {
    double v = c->R - c->d * sw_e(c, n);
    return v > 0.0 ? v : 0.0;
}

/* Segment slopes of the log interpolation, once per problem:
 * slope_b = (ℓ_{b+1} − ℓ_b) / (β_{b+1} − β_b), 0 past the last segment. */
SW_HD void sw_pwl_slopes(int32_t nb, const double* beta, const double* ell, double* slope) {
    for (int32_t b = 0; b < SW_BMAX; ++b)
        slope[b] = b < nb - 1 ? (ell[b + 1] - ell[b]) / (beta[b + 1] - beta[b]) : 0.0;
}

/* φ(u): interpolation of log over the bases on the segment holding u
 * (segment = largest b ≤ nb-2 with β_b ≤ u): ℓ_b + slope_b·(u − β_b), the
 * reference's ω-weighted sum of the two breakpoints (shockwave.py:162-181)
 * up to rounding, with no division per evaluation. */
SW_HD double sw_phi(double u, int32_t nb, const double* beta, const double* ell,
                    const double* slope) {
    int32_t b = 0;
    for (int32_t i = 1; i < nb - 1; ++i)
        if (beta[i] <= u) b = i;
    return ell[b] + slope[b] * (u - beta[b]);
}

/* f(n) — weighted log-utility with n planned rounds. */
SW_HD double sw_f(const sw_jobc* c, int32_t n, int32_t nb, const double* beta,
                  const double* ell, const double* slope) {
    double u = (c->Fd + sw_e(c, n)) * c->invE;
    return c->a * sw_phi(u, nb, beta, ell, slope);
}

/*
 * Ranking key of the job's (n+1)-th planned round: the monotonised marginal
 * utility per GPU-round, normalised by A = max_j a_j and rounded to fp32:
 *   vm(n) = min(vm(n−1), max(0, f(n+1) − f(n)))       (nonincreasing in n)
 *   key(n) = fp32(vm(n) · s), s = 1 / (w·A) once per job (sw_key_scale),
 *   flushed to 0 below FLT_MIN.
 * Keys are ≥ +0, so their bit patterns order like their values.
 */
SW_HD double sw_key_scale(int32_t w, double A) { return A > 0.0 ? 1.0 / ((double)w * A) : 0.0; }

SW_HD float sw_key(double vm, double scale) {
    double k = vm * scale;
    if (k < SW_FLT_MIN) return 0.0f;
    if (k > SW_FLT_MAX) k = SW_FLT_MAX;
    return (float)k;
}

SW_HD double sw_pos(double v) { return v > 0.0 ? v : 0.0; }

/* Placement-order key of a priority ratio (p_j/(n_j·w_j) or p_j/n_j, ≥ 0):
 * the fp64 bits without the 11 lowest mantissa bits (relative resolution
 * 2^-41), so that on the on-chip path the key and an 11-bit job index share
 * one 64-bit word and the placement sort moves 64 bits per element, not 128.
 * Ratios that agree to 2^-41 are ordered by job index, like exact ties. */
SW_HD uint64_t sw_ratio_key(double r) { return sw_bits(r) >> 11; }

/* Fill of stranded capacity: when P1 needed the reduced-
 * budget re-solve, single rounds are added into rounds with room, largest
 * utility gain f(n+1) − f(n) first.  Key of one candidate: the gain in fp32
 * (clamped to [FLT_MIN, FLT_MAX], so every positive gain keeps a nonzero
 * key), then the job index descending (26 bits), then the round (6 bits);
 * 0 when the gain is not positive.  At most SW_FILL_MAX rounds are added. */
#define SW_FILL_MAX 512
SW_HD uint64_t sw_fill_key(double gain, int64_t j, int32_t t) {
    if (!(gain > 0.0)) return 0;
    double k = gain;
    if (k < SW_FLT_MIN) k = SW_FLT_MIN;
    if (k > SW_FLT_MAX) k = SW_FLT_MAX;
    const uint32_t gb = sw_fbits_of((float)k);
    return ((uint64_t)gb << 32) | ((uint64_t)(0x3FFFFFFu - (uint32_t)j) << 6) | (uint64_t)t;
}
SW_HD int64_t sw_fill_job(uint64_t key) { return (int64_t)(0x3FFFFFFu - (uint32_t)((key >> 6) & 0x3FFFFFFu)); }
SW_HD int32_t sw_fill_round(uint64_t key) { return (int32_t)(key & 63u); }

/* Raises: after the fill and the per-round re-optimisation
 * of a re-solved plan, up to SW_RAISE_ITERS times one job gets one more
 * round and the whole plan is re-placed by the pattern search — a count
 * vector the fill cannot reach when no round has room for the job until
 * others move.  Candidates are the jobs with n_j < T_j, ranked by the gain of
 * one more round, f_j(n_j + 1) − f_j(n_j) − k·(max(M_j⁻, g_j(n_j + 1)) − M),
 * M the plan's makespan and M_j⁻ the largest g of the other jobs (sw_fill_key
 * of the gain, round 0); the first SW_RAISE_TRIES are tried in that order,
 * and a try is kept when the pattern search places it within G·T and its
 * objective beats the plan's. */
#define SW_RAISE_ITERS 4
#define SW_RAISE_TRIES 4
SW_HD double sw_raise_gain(double f0, double f1, double g1, double Mo, double M, double k) {
    const double Mn = Mo > g1 ? Mo : g1;
    return (f1 - f0) - k * (Mn - M);
}

/* Golden-section constants (fp64 literals, identical on both sides). */
#define SW_GS_A 0.3819660112501051
#define SW_GS_B 0.6180339887498949
#define SW_GS_ITERS 32
#define SW_REPACK_ITERS 3
/* marks makespan-critical jobs in the P1 packing order key */
#define SW_CRIT_BIT 0x8000000000000000ULL

#endif /* SW_ARITH_H */
