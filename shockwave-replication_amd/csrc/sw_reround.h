/*
 * sw_reround.h — per-round exact re-optimisation of a re-solved P1 plan
 * (DESIGN.md §3.3).  Plain C99; the constants and the specification are
 * shared by the GPU block function (sw_reround_dev.h: the batch kernel and
 * the sharded engine) and the CPU twins (oracle/plan_twin.c
 * twin_reround_arrays, called by oracle/shard_twin.c too).
 *
 * Why.  The reference's P1 (shockwave.py:330-382, capacity rows :64-75) is a
 * MILP over x_jt: it packs any widths exactly.  The count-then-pack reduction
 *  is exact while the level search's counts pack; when widths
 * fragment the rounds (clusters of a few times the widest job, jobs wider
 * than G/2) the re-solve on a reduced budget (SW_STATUS_P1_REPACKED) and the
 * fill leave plans up to a few percent below the MILP.  This step closes
 * most of that, on exactly those instances (the headline configurations
 * never re-solve, so their path is untouched).
 *
 * The step.  For each round t in turn, every other round fixed (b_j = n_j −
 * y_jt), the round's job set S is replaced by the one that maximises the
 * exact P1 objective
 *     Σ_j f_j(b_j + [j ∈ S]) − k·max_j g_j(b_j + [j ∈ S]),  Σ_{j∈S} w_j ≤ G,
 * when that beats the current set by more than SW_RR_TOL (relative).  With
 * v_j = f_j(b_j + 1) − f_j(b_j), h0_j = g_j(b_j), h1_j = g_j(b_j + 1) (h1 = h0
 * and v = 0 for a job wider than G) the value of a set is
 *     J(S) = detsum_j([j ∈ S]·v_j) − k·max_j([j ∈ S] ? h1_j : h0_j).
 * The utility part is a 0/1 knapsack over capacity G; the makespan part is
 * handled by its level θ: at level θ every job with h0_j > θ is forced into
 * S (it needs h1_j ≤ θ and a width that fits), the others are items.  The
 * unconstrained knapsack (no level) is solved first; its value D bounds
 * every level, so the levels — the distinct values of h0 ∪ h1 ∪ {0} — are
 * visited ascending and the scan stops at the first level θ whose
 * predecessor θ⁻ has D − k·θ⁻ ≤ the best J so far (a set whose makespan is
 * ≤ θ⁻ was already available at θ⁻).  Rounds are swept in order, passes
 * repeat until one changes nothing (at most SW_RR_PASSES).  Exact per round
 * while the knapsacks stay inside the limits below.
 *
 * The knapsack (items in job order, capacity cap): when the items' widths
 * fit cap all are taken; otherwise dp[c] over c = 0..cap, item by item,
 * dp'[c] = dp[c − w] + v if that is strictly larger than dp[c] (a take bit
 * per item and capacity), the smallest c with the largest dp[c], and the
 * take bits walked back from the last item.  It is solved only when cap ≤
 * SW_RR_CAPMAX, items × ⌈(cap + 1)/64⌉ ≤ SW_RR_WORDS (the take bits' 64-bit
 * words) and the solve's remaining item budget (SW_RR_BUDGET item steps)
 * covers it; otherwise that level (or, for the unconstrained knapsack, the
 * round) is skipped.  At most SW_RR_LEVELS levels are tried per round.
 */
#ifndef SW_REROUND_H
#define SW_REROUND_H

#define SW_RR_PASSES 4      /* sweeps over the rounds                          */
#define SW_RR_CAPMAX 1023   /* knapsack capacity handled                       */
#define SW_RR_WORDS 3072    /* take-bit words of one knapsack (24 KB)          */
#define SW_RR_LEVELS 64     /* makespan levels tried per round                 */
#ifndef SW_RR_BUDGET
#define SW_RR_BUDGET 65536  /* knapsack item steps per solve                   */
#endif
#define SW_RR_TOL 1e-12     /* a move must gain more than TOL·(|J_new| + |J_cur|) */

#endif /* SW_REROUND_H */
