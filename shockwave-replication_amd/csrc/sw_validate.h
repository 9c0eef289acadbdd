/*
 * sw_validate.h — input validation of one sw_problem (host side, C99).
 *
 * The reference has no explicit checks; these reject inputs for which its
 * model is undefined or numerically meaningless:
 *   - T < 1 or > SW_MAX_ROUNDS, fewer than 2 bases, bases not increasing
 *     (the SOS2 interpolation of shockwave.py:162-179 needs an ordered grid),
 *     or a grid that does not span [0, 1]: the model's progress
 *     u = (F + e)/E starts at F/E ≥ 0 and Σ ω β = u with Σ ω = 1 caps it at
 *     the last base, so the per-job reduction (e ≤ E − F, sw_arith.h) holds
 *     exactly when bases[0] = 0 (log(0) is replaced by log(1e-6),
 *     shockwave.py:102-103; a negative base has no log) and the last is 1;
 *   - Δ ≤ 0, k < 0 (k < 0 makes the reference's max-makespan term unbounded);
 *   - w < 1, E < 1, F ∉ [0, E] (job_metadata.py:75-78 asserts F ≤ E),
 *     d ≤ 0, non-finite R or priority < 0 (FTF^λ ≥ 0, shockwave.py:368);
 *   - a schedulable job (w ≤ G) wider than SW_MAX_WIDTH GPUs: the placement
 *     packs w into 8 bits (reference traces use scale factors 1–8).  Jobs
 *     wider than the cluster are accepted at any width; they are never
 *     scheduled (shockwave.py:64-75).
 */
#ifndef SW_VALIDATE_H
#define SW_VALIDATE_H

#include "../../include/shockwave_amd.h"

static inline int sw_finite(double x) { return x == x && x < 1e308 && x > -1e308; }

static inline int sw_validate_problem(const sw_problem* pr) {
    if (!pr) return -1;
    if (pr->num_jobs < 0 || pr->future_rounds < 1 || pr->future_rounds > SW_MAX_ROUNDS) return -1;
    if (pr->num_bases < 2 || pr->num_bases > SW_MAX_BASES || pr->num_gpus < 0) return -1;
    if (!(pr->round_duration > 0.0) || !sw_finite(pr->round_duration)) return -1;
    if (!(pr->regularizer >= 0.0) || !sw_finite(pr->regularizer)) return -1;
    if (!pr->bases || !pr->log_bases) return -1;
    for (int32_t b = 0; b < pr->num_bases; ++b) {
        if (!sw_finite(pr->log_bases[b]) || !sw_finite(pr->bases[b])) return -1;
        if (b > 0 && !(pr->bases[b] > pr->bases[b - 1])) return -1;
    }
    if (pr->bases[0] != 0.0 || pr->bases[pr->num_bases - 1] != 1.0) return -1;
    if (pr->num_jobs > 0 && (!pr->nworkers || !pr->epoch_duration || !pr->completed_epochs ||
                             !pr->total_epochs || !pr->remaining_runtime || !pr->priority))
        return -1;
    for (int32_t j = 0; j < pr->num_jobs; ++j) {
        if (pr->nworkers[j] < 1 || pr->total_epochs[j] < 1) return -1;
        if (pr->nworkers[j] <= pr->num_gpus && pr->nworkers[j] > SW_MAX_WIDTH) return -1;
        if (pr->completed_epochs[j] < 0 || pr->completed_epochs[j] > pr->total_epochs[j]) return -1;
        if (!(pr->epoch_duration[j] > 0.0) || !sw_finite(pr->epoch_duration[j])) return -1;
        if (!sw_finite(pr->remaining_runtime[j])) return -1;
        if (!(pr->priority[j] >= 0.0) || !sw_finite(pr->priority[j])) return -1;
    }
    return 0;
}

#endif /* SW_VALIDATE_H */
