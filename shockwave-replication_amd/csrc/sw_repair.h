/*
 * sw_repair.h — width-profile repair of a density-order placement that left
 * rounds unplaced.  Plain C99 + HIP qualifiers; shared by
 * the plan kernel (sw_kernels.hip, run by one thread), the sharded
 * controller (sw_shard_ctl.h, on the host) and the CPU twin.
 *
 * The reference's P2 (shockwave.py:281-328) is a MILP over the per-round
 * placement of fixed counts n_j with widths w_j.  The density order
 * p_j/(n_j·w_j) places rounds the way the MILP's LP relaxation would, but
 * with widths {1, 2, 4, 8} it can strand a wide job: the last rounds keep a
 * few free GPUs each, none with room for it.  The repair keeps the density
 * placement's per-width-class profile — how many jobs of each width run in
 * each round — and changes it only as much as the stranded rounds need:
 *
 *   for each class c, widest first, and each of its D_c unplaced rounds:
 *     ts = the round with the most free GPUs (ties: the latest) that still
 *          has a class-c job not running in it;
 *     while ts lacks w_c free GPUs: move one unit of a narrower class c2
 *          (narrowest first) from ts to the earliest other round with room
 *          for it and a class-c2 job not yet running there;
 *     give class c one more unit in ts.
 *
 * Each changed class is then repacked alone with unit widths inside its new
 * per-round capacities (the class-wise packer: exact for unit widths when
 * the profile admits the counts); unchanged classes keep their density rows.
 * On the simulator's P2 cases this lands within 1.04x of the P2 MILP where
 * the class-wise repack inside the P1 profile was up to 1.37x (tests/test_p2.py).
 */
#ifndef SW_REPAIR_H
#define SW_REPAIR_H

#include <stdint.h>

#include "sw_arith.h"

#define SW_RCLS_MAX 8 /* width classes the repair handles (traces: 4) */

typedef struct {
    int32_t ncls;                       /* classes present, ascending width     */
    int32_t wc[SW_RCLS_MAX];            /* class width                          */
    int32_t M[SW_RCLS_MAX];             /* jobs of the class with rounds        */
    int32_t D[SW_RCLS_MAX];             /* rounds of the class left unplaced    */
    int32_t changed[SW_RCLS_MAX];       /* profile changed: repack the class    */
    int32_t caps[SW_RCLS_MAX][SW_TMAX]; /* class jobs placed in round t         */
    int32_t L[SW_TMAX];                 /* free GPUs in round t                 */
} sw_repair_t;

/* Class index of width w (-1 if w is not a class). */
SW_HD int32_t sw_repair_class(const sw_repair_t* r, int32_t w) {
    for (int32_t c = 0; c < r->ncls; ++c)
        if (r->wc[c] == w) return c;
    return -1;
}

/* Inserts width w into the ascending class list; -1 when the list is full. */
SW_HD int32_t sw_repair_add_class(sw_repair_t* r, int32_t w) {
    int32_t c = sw_repair_class(r, w);
    if (c >= 0) return c;
    if (r->ncls >= SW_RCLS_MAX) return -1;
    int32_t i = r->ncls++;
    while (i > 0 && r->wc[i - 1] > w) {
        r->wc[i] = r->wc[i - 1];
        --i;
    }
    r->wc[i] = w;
    return i;
}

/* The repair itself on the filled-in profile; 0 on success, -1 when some
 * unplaced round finds no round to go to. */
SW_HD int32_t sw_profile_repair(sw_repair_t* r, int32_t T) {
    for (int32_t ci = r->ncls - 1; ci >= 0; --ci) {
        const int32_t c = r->wc[ci];
        for (int32_t d = 0; d < r->D[ci]; ++d) {
            int32_t ts = -1;
            for (int32_t t = 0; t < T; ++t)
                if (r->caps[ci][t] < r->M[ci] && (ts < 0 || r->L[t] >= r->L[ts])) ts = t;
            if (ts < 0) return -1;
            int32_t need = c - r->L[ts];
            for (int32_t c2 = 0; c2 < ci && need > 0; ++c2) {
                const int32_t w2 = r->wc[c2];
                while (need > 0 && r->caps[c2][ts] > 0) {
                    int32_t t2 = -1;
                    for (int32_t t = 0; t < T && t2 < 0; ++t)
                        if (t != ts && r->L[t] >= w2 && r->caps[c2][t] < r->M[c2]) t2 = t;
                    if (t2 < 0) break;
                    r->caps[c2][ts] -= 1;
                    r->L[ts] += w2;
                    r->caps[c2][t2] += 1;
                    r->L[t2] -= w2;
                    r->changed[c2] = 1;
                    need -= w2;
                }
            }
            if (r->L[ts] < c) return -1;
            r->caps[ci][ts] += 1;
            r->L[ts] -= c;
            r->changed[ci] = 1;
        }
    }
    return 0;
}

#endif /* SW_REPAIR_H */
