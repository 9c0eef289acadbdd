/*
 * oracle/shard_twin.c — TEST INFRASTRUCTURE, NOT PRODUCT CODE.
 *
 * CPU shard engine for the sharded plan-solve controller
 * (shockwave-replication_amd/csrc/sw_shard_ctl.h).  One process per rank
 * holds its slice of jobs (sw_shard_range) as plain host arrays; collectives
 * go through a caller-supplied sw_host_comm (gloo from Python in
 * tests/test_shard.py).  It exists so the multi-rank control flow of the
 * sharded solve — the lane-aligned deterministic sums, the rank-exclusive tie
 * prefix, the global width-tail arg-max, the gathered placement — is tested on
 * CPU at world sizes > 1, against the single-instance twin (plan_twin.c):
 * results must be bit-identical.  The product engine is sw_shard.hip; this
 * file is never linked into it.
 *
 * Per-step semantics follow plan_twin.c's select_level / feasible_level /
 * levels_between / pack / twin_plan_solve (the reference lines they restate
 * are cited there: shockwave.py:281-398).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/shockwave_amd.h"
#include "../shockwave-replication_amd/csrc/sw_arith.h"
#include "../shockwave-replication_amd/csrc/sw_repair.h"
#include "../shockwave-replication_amd/csrc/sw_shard_ctl.h"
#include "../shockwave-replication_amd/csrc/sw_validate.h"

void twin_pack_arrays_caps(int32_t N, int32_t T, int32_t G, const int32_t* w, const int32_t* nin,
                           const uint64_t* k1, const uint32_t* k2, uint8_t* y, int32_t* placed,
                           const int32_t* caps, int unit);

typedef struct {
    const sw_host_comm* comm;
    int32_t rank, world, LW;
    int64_t N, off, q, P; /* global jobs, slice offset, jobs per lane, padded slice */
    int32_t NL, T, G, nb;
    double k, A;
    const double* beta;
    const double* ell;
    double slope[SW_BMAX];
    const double* p;
    sw_jobc* jc;
    int32_t* Tj;
    float* key; /* [NL][T] */
    int32_t *l, *taken;
    int32_t* arr[SW_A_COUNT];
    uint64_t* y[SW_Y_COUNT];
    int32_t* w_all;
    int32_t scaps[SW_VSHARES][SW_TMAX]; /* this rank's shares of every round (pack_share) */
    int share;              /* the shares exist (sw_share_caps succeeded) */
    sw_result* res;
} eng_t;

#define KEY(E, i, n) ((E)->key[(size_t)(i) * (E)->T + (n)])

static int e_raise_stats(void* ctx, double M, int64_t out[3]);
static int e_raise_best(void* ctx, double M, int64_t i1, double M2, const int64_t* tried, int32_t ntried,
                        uint64_t* best);

static double fv(const eng_t* E, int32_t i, int32_t n) {
    return sw_f(&E->jc[i], n, E->nb, E->beta, E->ell, E->slope);
}

static int32_t lforce(const eng_t* E, int32_t i, double M) {
    int32_t c = 0;
    for (int32_t n = 0; n < E->Tj[i]; ++n) c += (sw_g(&E->jc[i], n) > M);
    return c;
}

static int32_t cnt(const eng_t* E, int32_t i, uint32_t rho, int ge) {
    int32_t c = 0;
    for (int32_t n = E->l[i]; n < E->Tj[i]; ++n) {
        uint32_t b = sw_fbits_of(KEY(E, i, n));
        c += ge ? (b >= rho) : (b > rho);
    }
    return c;
}

/* lane partials of v over this rank's lanes, gathered into out[SW_DET_LANES] */
static int lanes_gather(eng_t* E, const double* v, double* out) {
    double* mine = (double*)calloc((size_t)E->LW, sizeof(double));
    if (!mine) return -1;
    for (int32_t i = 0; i < E->NL; ++i) {
        const int64_t L = (E->off + i) / E->q - (int64_t)E->rank * E->LW;
        mine[L] = mine[L] + v[i];
    }
    int rc = E->comm->allgather(E->comm->ctx, mine, out, (int64_t)E->LW * (int64_t)sizeof(double));
    free(mine);
    return rc;
}

static int e_setup(void* ctx, double* A, double* lb, double* top) {
    eng_t* E = (eng_t*)ctx;
    double mx[3] = {0.0, 0.0, 0.0};
    for (int32_t i = 0; i < E->NL; ++i) mx[0] = sw_max(mx[0], E->jc[i].a);
    if (E->comm->allreduce_max_f64(E->comm->ctx, mx, 1)) return -1;
    E->A = mx[0];
    for (int32_t i = 0; i < E->NL; ++i) {
        const double ks = sw_key_scale(E->jc[i].w, E->A);
        double prev = fv(E, i, 0), vm = 0.0;
        for (int32_t n = 0; n < E->T; ++n) {
            double cur = fv(E, i, n + 1);
            double v = sw_pos(cur - prev);
            vm = (n == 0) ? v : sw_min(vm, v);
            KEY(E, i, n) = sw_key(vm, ks);
            prev = cur;
        }
        mx[1] = sw_max(mx[1], sw_g(&E->jc[i], E->Tj[i]));
        mx[2] = sw_max(mx[2], sw_g(&E->jc[i], 0));
    }
    if (E->comm->allreduce_max_f64(E->comm->ctx, mx + 1, 2)) return -1;
    *A = E->A;
    *lb = mx[1];
    *top = mx[2];
    /* widths of every job, gathered in padded per-rank blocks (the gathered
     * placements read them; the controller asks for them through e_widths) */
    int32_t* blk = (int32_t*)calloc((size_t)(E->P > 0 ? E->P : 1), sizeof(int32_t));
    int32_t* all = (int32_t*)calloc((size_t)(E->P > 0 ? E->P : 1) * E->world, sizeof(int32_t));
    if (!blk || !all) { free(blk); free(all); return -1; }
    for (int32_t i = 0; i < E->NL; ++i) blk[i] = E->jc[i].w;
    int rc = E->comm->allgather(E->comm->ctx, blk, all, E->P * (int64_t)sizeof(int32_t));
    /* rank r's block starts at r·P, which is also its first global job */
    for (int64_t j = 0; j < E->N; ++j) E->w_all[j] = all[j];
    free(blk); free(all);
    return rc;
}

static int e_widths(void* ctx, int32_t* w_all) {
    eng_t* E = (eng_t*)ctx;
    for (int64_t j = 0; j < E->N; ++j) w_all[j] = E->w_all[j];
    return 0;
}


static int e_force(void* ctx, double M, int32_t is_inf, int64_t out[2]) {
    eng_t* E = (eng_t*)ctx;
    out[0] = out[1] = 0;
    for (int32_t i = 0; i < E->NL; ++i) {
        E->l[i] = is_inf ? 0 : lforce(E, i, M);
        out[0] += (int64_t)E->jc[i].w * E->l[i];
        out[1] += (int64_t)E->jc[i].w * (E->Tj[i] - E->l[i]);
    }
    return E->comm->allreduce_sum_i64(E->comm->ctx, out, 2);
}

static int e_count_gt(void* ctx, const uint32_t* rho, int32_t K, uint64_t lo, int64_t* out) {
    eng_t* E = (eng_t*)ctx;
    for (int32_t k = 0; k < K; ++k) {
        out[k] = 0;
        for (int32_t i = 0; i < E->NL; ++i) out[k] += (int64_t)E->jc[i].w * cnt(E, i, rho[k], 0);
    }
    out[K] = 0; /* keys ≥ lo (lo < 2^32: a price bracket's end) */
    for (int32_t i = 0; i < E->NL; ++i) out[K] += (int64_t)E->jc[i].w * cnt(E, i, (uint32_t)lo, 1);
    return E->comm->allreduce_sum_i64(E->comm->ctx, out, K + 1);
}

static int e_feasible(void* ctx, const double* M, int32_t K, uint64_t lo, int64_t* out) {
    eng_t* E = (eng_t*)ctx;
    for (int32_t k = 0; k < K; ++k) {
        out[k] = 0;
        for (int32_t i = 0; i < E->NL; ++i) out[k] += (int64_t)E->jc[i].w * lforce(E, i, M[k]);
    }
    out[K] = 0; /* levels whose bits are ≥ lo */
    for (int32_t i = 0; i < E->NL; ++i)
        for (int32_t n = 0; n < E->Tj[i]; ++n) out[K] += sw_bits(sw_g(&E->jc[i], n)) >= lo ? E->jc[i].w : 0;
    return E->comm->allreduce_sum_i64(E->comm->ctx, out, K + 1);
}

/* the items of a search bracket [lo, hi] (sw_shard_ops.gather): this rank's
 * (v, w) pairs, all-gathered in blocks of 1 + 2·SW_GATHER_CAP words */
static int e_gather(void* ctx, int32_t kind, uint64_t lo, uint64_t hi, uint64_t* v, int64_t* w, int32_t* n) {
    eng_t* E = (eng_t*)ctx;
    const int64_t bw = 1 + 2 * (int64_t)SW_GATHER_CAP;
    int64_t* mine = (int64_t*)calloc((size_t)bw, sizeof(int64_t));
    int64_t* all = (int64_t*)calloc((size_t)bw * (size_t)E->world, sizeof(int64_t));
    if (!mine || !all) { free(mine); free(all); return -1; }
    int64_t m = 0;
    for (int32_t i = 0; i < E->NL; ++i)
        for (int32_t t = kind ? 0 : E->l[i]; t < E->Tj[i]; ++t) {
            const uint64_t b = kind ? sw_bits(sw_g(&E->jc[i], t)) : (uint64_t)sw_fbits_of(KEY(E, i, t));
            if (b < lo || b > hi) continue;
            if (m < SW_GATHER_CAP) {
                mine[1 + 2 * m] = (int64_t)b;
                mine[2 + 2 * m] = E->jc[i].w;
            }
            ++m;
        }
    mine[0] = m;
    int rc = E->comm->allgather(E->comm->ctx, mine, all, bw * (int64_t)sizeof(int64_t));
    int32_t k = 0;
    for (int32_t r = 0; !rc && r < E->world; ++r) {
        const int64_t* b = all + (size_t)r * bw;
        if (b[0] > SW_GATHER_CAP || k + b[0] > SW_GATHER_CAP) { rc = -3; break; }
        for (int64_t e = 0; e < b[0]; ++e, ++k) {
            v[k] = (uint64_t)b[1 + 2 * e];
            w[k] = b[2 + 2 * e];
        }
    }
    *n = k;
    free(mine); free(all);
    return rc;
}

static int e_between(void* ctx, double a, double b, int64_t* out) {
    eng_t* E = (eng_t*)ctx;
    int64_t c = 0;
    for (int32_t i = 0; i < E->NL; ++i)
        for (int32_t n = 0; n <= E->Tj[i]; ++n) {
            double v = sw_g(&E->jc[i], n);
            c += (v > a && v < b);
        }
    *out = c;
    return E->comm->allreduce_sum_i64(E->comm->ctx, out, 1);
}

static int e_take_all(void* ctx) {
    eng_t* E = (eng_t*)ctx;
    for (int32_t i = 0; i < E->NL; ++i) {
        E->arr[SW_A_N][i] = E->Tj[i];
        E->taken[i] = E->Tj[i] - E->l[i];
    }
    return 0;
}

static int e_take(void* ctx, uint32_t rho, int64_t* wt, int64_t* excl) {
    eng_t* E = (eng_t*)ctx;
    int64_t mine[2] = {0, 0};
    for (int32_t i = 0; i < E->NL; ++i) {
        E->taken[i] = cnt(E, i, rho, 0);
        mine[0] += (int64_t)E->jc[i].w * E->taken[i];
        mine[1] += (int64_t)E->jc[i].w * (cnt(E, i, rho, 1) - E->taken[i]);
    }
    int64_t* all = (int64_t*)malloc(sizeof(int64_t) * 2 * E->world);
    if (!all) return -1;
    int rc = E->comm->allgather(E->comm->ctx, mine, all, 2 * (int64_t)sizeof(int64_t));
    *wt = 0;
    *excl = 0;
    for (int32_t r = 0; r < E->world; ++r) {
        *wt += all[2 * r];
        if (r < E->rank) *excl += all[2 * r + 1];
    }
    free(all);
    return rc;
}

static int e_assign(void* ctx, uint32_t rho, int64_t rem, int64_t excl, int64_t* used) {
    eng_t* E = (eng_t*)ctx;
    int64_t u = 0;
    for (int32_t i = 0; i < E->NL; ++i) {
        const int32_t tie = cnt(E, i, rho, 1) - E->taken[i];
        const int64_t wj = E->jc[i].w;
        int32_t tt;
        if (excl + wj * tie <= rem) tt = tie;
        else if (excl <= rem) tt = (int32_t)((rem - excl) / wj);
        else tt = 0;
        E->arr[SW_A_N][i] = E->l[i] + E->taken[i] + tt;
        u += wj * tt;
        excl += wj * tie;
    }
    *used = u;
    return E->comm->allreduce_sum_i64(E->comm->ctx, used, 1);
}

static int e_tail_best(void* ctx, int64_t rem2, uint64_t* best) {
    eng_t* E = (eng_t*)ctx;
    uint64_t b = 0;
    for (int32_t i = 0; i < E->NL; ++i) {
        const int32_t n = E->arr[SW_A_N][i];
        if (n < E->Tj[i] && (int64_t)E->jc[i].w <= rem2) {
            const uint64_t kk = ((uint64_t)sw_fbits_of(KEY(E, i, n)) << 32) |
                                (uint64_t)(0xFFFFFFFFu - (uint32_t)(E->off + i));
            b = kk > b ? kk : b;
        }
    }
    *best = b;
    return E->comm->allreduce_max_u64(E->comm->ctx, best, 1);
}

static int e_tail_apply(void* ctx, int64_t jb) {
    eng_t* E = (eng_t*)ctx;
    if (jb >= E->off && jb < E->off + E->NL) E->arr[SW_A_N][jb - E->off] += 1;
    return 0;
}

static int e_fill_best(void* ctx, const int64_t* load, uint64_t* best) {
    eng_t* E = (eng_t*)ctx;
    uint64_t b = 0;
    for (int32_t i = 0; i < E->NL; ++i) {
        const int32_t n = E->arr[SW_A_NFIN][i];
        if (n >= E->Tj[i]) continue;
        const uint64_t m = E->y[SW_Y_BEST][i];
        const int64_t w = E->jc[i].w;
        int32_t tf = -1;
        for (int32_t t = 0; t < E->T; ++t)
            if (!((m >> t) & 1u) && w <= E->G - load[t]) { tf = t; break; }
        if (tf < 0) continue;
        const uint64_t kk = sw_fill_key(fv(E, i, n + 1) - fv(E, i, n), E->off + i, tf);
        b = kk > b ? kk : b;
    }
    *best = b;
    return E->comm->allreduce_max_u64(E->comm->ctx, best, 1);
}

static int e_fill_apply(void* ctx, int64_t jb, int32_t t) {
    eng_t* E = (eng_t*)ctx;
    if (jb >= E->off && jb < E->off + E->NL) {
        E->y[SW_Y_BEST][jb - E->off] |= (uint64_t)1 << t;
        E->arr[SW_A_NFIN][jb - E->off] += 1;
    }
    return 0;
}

static int e_eval(void* ctx, int32_t sel, int32_t arg, double* lanesA, double* lanesB, double* gm,
                  int64_t* isum) {
    eng_t* E = (eng_t*)ctx;
    const int32_t NL = E->NL;
    double* va = (double*)calloc((size_t)(NL > 0 ? NL : 1), sizeof(double));
    double* vb = (double*)calloc((size_t)(NL > 0 ? NL : 1), sizeof(double));
    if (!va || !vb) { free(va); free(vb); return -1; }
    double g = 0.0;
    int64_t s = 0;
    for (int32_t i = 0; i < NL; ++i) {
        const sw_jobc* c = &E->jc[i];
        if (sel == SW_EV_SELECT) {
            const int32_t n = E->arr[SW_A_N][i];
            va[i] = fv(E, i, n);
            vb[i] = fv(E, i, E->l[i] + E->taken[i]);
            g = sw_max(g, sw_g(c, n));
        } else if (sel == SW_EV_GMAX) {
            g = sw_max(g, sw_g(c, E->arr[arg][i]));
        } else if (sel == SW_EV_PACKED) {
            const int32_t pl = E->arr[arg][i];
            va[i] = fv(E, i, pl);
            g = sw_max(g, sw_g(c, pl));
            s += (int64_t)c->w * (E->arr[SW_A_NB][i] - pl);
        } else if (sel == SW_EV_P2OK) {
            s += E->arr[SW_A_PL][i] != E->arr[SW_A_NFIN][i];
        } else if (sel == SW_EV_UNPLACED) {
            s += E->arr[arg & 0xFF][i] != E->arr[arg >> 8][i];
        } else if (sel == SW_EV_UMAX) {
            va[i] = fv(E, i, E->Tj[i]);
        } else { /* SW_EV_FINAL */
            const uint64_t m = E->y[arg][i];
            int32_t cn = 0;
            int64_t S = 0;
            for (int32_t t = 0; t < E->T; ++t)
                if ((m >> t) & 1u) { cn += 1; S += t; }
            va[i] = fv(E, i, cn);
            vb[i] = cn > 0 ? ((double)S / (double)cn) * E->p[i] : 0.0;
            g = sw_max(g, sw_g(c, cn));
            s += cn > 0;
            if (E->res->plan)
                for (int32_t t = 0; t < E->T; ++t)
                    E->res->plan[(size_t)i * E->T + t] = (uint8_t)((m >> t) & 1u);
            if (E->res->planned_rounds) E->res->planned_rounds[i] = cn;
        }
    }
    int rc = lanes_gather(E, va, lanesA);
    if (!rc) rc = lanes_gather(E, vb, lanesB);
    *gm = g;
    *isum = s;
    if (!rc) rc = E->comm->allreduce_max_f64(E->comm->ctx, gm, 1);
    if (!rc) rc = E->comm->allreduce_sum_i64(E->comm->ctx, isum, 1);
    free(va); free(vb);
    return rc;
}

static int e_copy(void* ctx, int32_t dst, int32_t src) {
    eng_t* E = (eng_t*)ctx;
    if (E->NL) memcpy(E->arr[dst], E->arr[src], sizeof(int32_t) * (size_t)E->NL);
    return 0;
}

static int e_copy_y(void* ctx, int32_t dst, int32_t src) {
    eng_t* E = (eng_t*)ctx;
    if (E->NL) memcpy(E->y[dst], E->y[src], sizeof(uint64_t) * (size_t)E->NL);
    return 0;
}

/* gathered placement: every rank runs the twin's packer on all jobs */
typedef struct {
    uint64_t k1;
    uint32_t k2;
    int32_t nin;
} pk_t;

/* mode 1/3/2/4 = sw_shard_ops.pack; mode 5 = pack_class (jobs of width wc,
 * unit widths, per-round capacities caps, other jobs untouched) */
static int e_pack_any(eng_t* E, int32_t mode, int32_t src, double Mb, int32_t ydst, int32_t pdst,
                      int32_t wc, const int32_t* caps) {
    const int64_t P = E->P > 0 ? E->P : 1, N = E->N;
    pk_t* mine = (pk_t*)calloc((size_t)P, sizeof(pk_t));
    pk_t* all = (pk_t*)calloc((size_t)P * E->world, sizeof(pk_t));
    int32_t* nin = (int32_t*)calloc((size_t)(N > 0 ? N : 1), sizeof(int32_t));
    uint64_t* k1 = (uint64_t*)calloc((size_t)(N > 0 ? N : 1), sizeof(uint64_t));
    uint32_t* k2 = (uint32_t*)calloc((size_t)(N > 0 ? N : 1), sizeof(uint32_t));
    int32_t* placed = (int32_t*)calloc((size_t)(N > 0 ? N : 1), sizeof(int32_t));
    uint8_t* y = (uint8_t*)calloc((size_t)(N > 0 ? N : 1) * E->T, 1);
    int rc = -1;
    if (!mine || !all || !nin || !k1 || !k2 || !placed || !y) goto out;
    for (int32_t i = 0; i < E->NL; ++i) {
        const int32_t n = (mode == 5 && E->jc[i].w != wc) ? 0 : E->arr[src][i];
        mine[i].nin = n;
        if (n > 0) {
            if (mode == 4) {
                mine[i].k1 = sw_ratio_key(E->p[i] / (double)(n * E->jc[i].w));
                mine[i].k2 = 0;
            } else if (mode != 2 && mode != 5) {
                const double lvl = sw_g(&E->jc[i], n - 1);
                const int crit = E->k > 0.0 && lvl > Mb;
                mine[i].k1 = crit ? (SW_CRIT_BIT | sw_bits(lvl)) : (mode == 3 ? (uint64_t)E->jc[i].w : 0);
                mine[i].k2 = sw_fbits_of(KEY(E, i, n - 1));
            } else {
                mine[i].k1 = sw_ratio_key(E->p[i] / (double)n);
                mine[i].k2 = 0;
            }
        }
    }
    rc = E->comm->allgather(E->comm->ctx, mine, all, P * (int64_t)sizeof(pk_t));
    if (rc) goto out;
    for (int64_t j = 0; j < N; ++j) {
        nin[j] = all[j].nin; /* blocks are P long and contiguous: job j at j */
        k1[j] = all[j].k1;
        k2[j] = all[j].k2;
    }
    twin_pack_arrays_caps((int32_t)N, E->T, E->G, E->w_all, nin, k1, k2, y, placed,
                          mode == 5 ? caps : NULL, mode == 5);
    for (int32_t i = 0; i < E->NL; ++i) {
        const int64_t j = E->off + i;
        if (mode == 5 && !(E->jc[i].w == wc && E->arr[src][i] > 0)) continue;
        uint64_t m = 0;
        for (int32_t t = 0; t < E->T; ++t) m |= (uint64_t)y[(size_t)j * E->T + t] << t;
        E->y[ydst][i] = m;
        E->arr[pdst][i] = placed[j];
    }
out:
    free(mine); free(all); free(nin); free(k1); free(k2); free(placed); free(y);
    return rc;
}

static int e_pack(void* ctx, int32_t mode, int32_t src, double Mb, int32_t ydst, int32_t pdst) {
    return e_pack_any((eng_t*)ctx, mode, src, Mb, ydst, pdst, 0, NULL);
}

static int e_pack_class(void* ctx, int32_t src, int32_t wc, const int32_t* caps, int32_t ydst,
                        int32_t pdst) {
    return e_pack_any((eng_t*)ctx, 5, src, 0.0, ydst, pdst, wc, caps);
}

static int e_class_caps(void* ctx, int32_t src, int32_t ysrc, int32_t wc, int32_t psrc,
                        int32_t* caps, int32_t* next_w, int64_t* md) {
    eng_t* E = (eng_t*)ctx;
    int64_t buf[SW_TMAX + 2];
    uint64_t nx = 0; /* max of ~next: the min width above wc */
    for (int32_t t = 0; t < E->T + 2; ++t) buf[t] = 0;
    for (int32_t i = 0; i < E->NL; ++i) {
        if (E->arr[src][i] <= 0) continue;
        const int32_t w = E->jc[i].w;
        if (w == wc) {
            if (psrc == SW_CLASS_HIST) buf[E->arr[src][i] - 1] += 1; /* count histogram */
            else
                for (int32_t t = 0; t < E->T; ++t) buf[t] += (int64_t)((E->y[ysrc][i] >> t) & 1u);
            buf[E->T] += 1;
            if (psrc >= 0) buf[E->T + 1] += E->arr[src][i] - E->arr[psrc][i];
        }
        if (w > wc) {
            const uint64_t v = 0xFFFFFFFFull - (uint64_t)w;
            nx = v > nx ? v : nx;
        }
    }
    int rc = E->comm->allreduce_sum_i64(E->comm->ctx, buf, E->T + 2);
    if (!rc) rc = E->comm->allreduce_max_u64(E->comm->ctx, &nx, 1);
    if (rc) return -1;
    for (int32_t t = 0; t < E->T; ++t) caps[t] = (int32_t)buf[t];
    md[0] = buf[E->T];
    md[1] = buf[E->T + 1];
    *next_w = nx == 0 ? 0x7FFFFFFF : (int32_t)(0xFFFFFFFFull - nx);
    return 0;
}

/* this rank's shares (sw_share_count): S = V / W of them, share s holding the
 * local jobs [lo, hi) */
static int32_t e_shares(const eng_t* E, int32_t s, int32_t* lo, int32_t* hi) {
    const int32_t V = sw_share_count(E->N, E->G, E->world), S = V / E->world;
    int64_t a = 0, b = 0;
    if (s < S) sw_shard_range(E->N, V, E->rank * S + s, &a, &b);
    *lo = (int32_t)(a - E->off);
    *hi = (int32_t)(b - E->off);
    return S;
}

/* the share placement (sw_shard_ops.pack_share): the loads of every share
 * all-gathered, this rank's jobs of each of its shares packed alone into that
 * share of the rounds (density order, mixed widths, the tier rule over
 * non-uniform capacities: plan_twin.c pack) */
static int e_pack_share(void* ctx, int32_t src, int32_t ydst, int32_t pdst) {
    eng_t* E = (eng_t*)ctx;
    const int32_t NL = E->NL, T = E->T;
    const size_t NN = NL > 0 ? (size_t)NL : 1;
    int32_t lo, hi;
    const int32_t S = e_shares(E, 0, &lo, &hi), V = S * E->world;
    int64_t mine[SW_VSHARES];
    for (int32_t s = 0; s < S; ++s) {
        e_shares(E, s, &lo, &hi);
        mine[s] = 0;
        for (int32_t i = lo; i < hi; ++i) mine[s] += (int64_t)E->jc[i].w * E->arr[src][i];
    }
    int64_t* loads = (int64_t*)calloc((size_t)V, sizeof(int64_t));
    int32_t* w = (int32_t*)malloc(sizeof(int32_t) * NN);
    int32_t* nin = (int32_t*)malloc(sizeof(int32_t) * NN);
    uint64_t* k1 = (uint64_t*)malloc(sizeof(uint64_t) * NN);
    uint32_t* k2 = (uint32_t*)calloc(NN, sizeof(uint32_t));
    int32_t* placed = (int32_t*)calloc(NN, sizeof(int32_t));
    uint8_t* y = (uint8_t*)calloc(NN * (size_t)T, 1);
    int rc = -1;
    if (!loads || !w || !nin || !k1 || !k2 || !placed || !y) goto out;
    rc = E->comm->allgather(E->comm->ctx, mine, loads, (int64_t)sizeof(int64_t) * S);
    if (rc) goto out;
    E->share = 1;
    for (int32_t s = 0; s < S; ++s)
        E->share &= sw_share_caps(loads, V, E->rank * S + s, T, E->G, E->scaps[s]) == 0;
    for (int32_t i = 0; i < NL; ++i) {
        w[i] = E->jc[i].w;
        nin[i] = E->share ? E->arr[src][i] : 0;
        k1[i] = nin[i] > 0 ? sw_ratio_key(E->p[i] / (double)(nin[i] * w[i])) : 0;
    }
    if (E->share)
        for (int32_t s = 0; s < S; ++s) {
            e_shares(E, s, &lo, &hi);
            if (hi > lo)
                twin_pack_arrays_caps(hi - lo, T, E->G, w + lo, nin + lo, k1 + lo, k2 + lo,
                                      y + (size_t)lo * T, placed + lo, E->scaps[s], 0);
        }
    for (int32_t i = 0; i < NL; ++i) {
        uint64_t m = 0;
        for (int32_t t = 0; t < T; ++t) m |= (uint64_t)y[(size_t)i * T + t] << t;
        E->y[ydst][i] = m;
        E->arr[pdst][i] = placed[i];
    }
out:
    free(loads); free(w); free(nin); free(k1); free(k2); free(placed); free(y);
    return rc;
}

/* sw_shard_ops.share_repair: every share of this rank whose pack stranded
 * rounds has its width profile repaired inside the share (sw_profile_repair
 * with the share's free GPUs) and every changed class repacked alone (unit
 * widths, order p/n) — plan_twin.c repair_pack on the share's own jobs */
static int e_share_repair_one(eng_t* E, int32_t src, int32_t ydst, int32_t pdst, int32_t lo, int32_t hi,
                              const int32_t* scaps) {
    const int32_t T = E->T, NL = hi - lo;
    int64_t dfc = 0;
    for (int32_t i = lo; i < hi; ++i) dfc += (int64_t)E->jc[i].w * (E->arr[src][i] - E->arr[pdst][i]);
    if (dfc == 0) return 0;
    sw_repair_t R;
    memset(&R, 0, sizeof(R));
    for (int32_t i = lo; i < hi; ++i)
        if (E->arr[src][i] > 0 && sw_repair_add_class(&R, E->jc[i].w) < 0) return 0;
    for (int32_t t = 0; t < T; ++t) R.L[t] = scaps[t];
    for (int32_t i = lo; i < hi; ++i) {
        const uint64_t m = E->y[ydst][i];
        for (int32_t t = 0; t < T; ++t)
            if ((m >> t) & 1u) R.L[t] -= E->jc[i].w;
        if (E->arr[src][i] <= 0) continue;
        const int32_t c = sw_repair_class(&R, E->jc[i].w);
        R.M[c] += 1;
        R.D[c] += E->arr[src][i] - E->arr[pdst][i];
        for (int32_t t = 0; t < T; ++t) R.caps[c][t] += (int32_t)((m >> t) & 1u);
    }
    if (sw_profile_repair(&R, T) != 0) return 0;
    const size_t NN = NL > 0 ? (size_t)NL : 1;
    int32_t* w = (int32_t*)malloc(sizeof(int32_t) * NN);
    int32_t* nc = (int32_t*)malloc(sizeof(int32_t) * NN);
    uint64_t* k1 = (uint64_t*)malloc(sizeof(uint64_t) * NN);
    uint32_t* k2 = (uint32_t*)calloc(NN, sizeof(uint32_t));
    int32_t* pc = (int32_t*)calloc(NN, sizeof(int32_t));
    uint8_t* yc = (uint8_t*)calloc(NN * (size_t)T, 1);
    int rc = -1;
    if (!w || !nc || !k1 || !k2 || !pc || !yc) goto out;
    for (int32_t i = 0; i < NL; ++i) w[i] = E->jc[lo + i].w;
    for (int32_t c = 0; c < R.ncls; ++c) {
        if (!R.changed[c]) continue;
        for (int32_t i = 0; i < NL; ++i) {
            const int cls = E->arr[src][lo + i] > 0 && w[i] == R.wc[c];
            nc[i] = cls ? E->arr[src][lo + i] : 0;
            k1[i] = cls ? sw_ratio_key(E->p[lo + i] / (double)nc[i]) : 0;
        }
        twin_pack_arrays_caps(NL, T, E->G, w, nc, k1, k2, yc, pc, R.caps[c], 1);
        for (int32_t i = 0; i < NL; ++i) {
            if (nc[i] <= 0) continue;
            uint64_t m = 0;
            for (int32_t t = 0; t < T; ++t) m |= (uint64_t)yc[(size_t)i * T + t] << t;
            E->y[ydst][lo + i] = m;
            E->arr[pdst][lo + i] = pc[i];
        }
    }
    rc = 0;
out:
    free(w); free(nc); free(k1); free(k2); free(pc); free(yc);
    return rc;
}

static int e_share_repair(void* ctx, int32_t src, int32_t ydst, int32_t pdst) {
    eng_t* E = (eng_t*)ctx;
    if (!E->share) return 0;
    int32_t lo, hi;
    const int32_t S = e_shares(E, 0, &lo, &hi);
    for (int32_t s = 0; s < S; ++s) {
        e_shares(E, s, &lo, &hi);
        if (e_share_repair_one(E, src, ydst, pdst, lo, hi, E->scaps[s]) < 0) return -1;
    }
    return 0;
}

/* the P2 exchange step on the gathered placement (twin_p2x_run) */
int32_t twin_p2x_run(int32_t A, int32_t T, int32_t G, const int32_t* job, const int32_t* w,
                     const double* c, uint64_t* m);
typedef struct {
    uint64_t m;
    double p;
    int32_t n, pad;
} p2g_t;

static int e_p2x(void* ctx, int32_t ysrc, int32_t nsrc, int32_t* cancels) {
    eng_t* E = (eng_t*)ctx;
    const int64_t P = E->P > 0 ? E->P : 1, N = E->N;
    p2g_t* mine = (p2g_t*)calloc((size_t)P, sizeof(p2g_t));
    p2g_t* all = (p2g_t*)calloc((size_t)P * E->world, sizeof(p2g_t));
    int32_t* job = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
    int32_t* w = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
    double* c = (double*)malloc(sizeof(double) * (size_t)(N > 0 ? N : 1));
    uint64_t* m = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(N > 0 ? N : 1));
    int rc = -1;
    if (!mine || !all || !job || !w || !c || !m) goto out;
    for (int32_t i = 0; i < E->NL; ++i) {
        mine[i].n = E->arr[nsrc][i];
        mine[i].p = E->p[i];
        mine[i].m = E->y[ysrc][i];
    }
    rc = E->comm->allgather(E->comm->ctx, mine, all, P * (int64_t)sizeof(p2g_t));
    if (rc) goto out;
    int32_t A = 0;
    for (int64_t j = 0; j < N; ++j) { /* blocks are P long and contiguous: job j at j */
        if (all[j].n <= 0) continue;
        job[A] = (int32_t)j;
        w[A] = E->w_all[j];
        c[A] = all[j].p / (double)all[j].n;
        m[A] = all[j].m;
        ++A;
    }
    *cancels = twin_p2x_run(A, E->T, E->G, job, w, c, m);
    for (int32_t a = 0; a < A; ++a)
        if (job[a] >= E->off && job[a] < E->off + E->NL) E->y[ysrc][job[a] - E->off] = m[a];
out:
    free(mine); free(all); free(job); free(w); free(c); free(m);
    return rc;
}

/* the per-round re-optimisation on the gathered P1 plan (twin_reround_arrays) */
int32_t twin_reround_arrays(int32_t N, int32_t T, int32_t G, double k, int32_t nb,
                            const double* beta, const double* ell, const sw_jobc* jc,
                            int32_t* n, uint8_t* y, int64_t* passes);
typedef struct {
    sw_jobc c;
    uint64_t m;
    int32_t n, pad;
} rrg_t;

static int e_reround(void* ctx, int32_t* moves) {
    eng_t* E = (eng_t*)ctx;
    const int64_t P = E->P > 0 ? E->P : 1, N = E->N;
    const size_t NN = N > 0 ? (size_t)N : 1;
    rrg_t* mine = (rrg_t*)calloc((size_t)P, sizeof(rrg_t));
    rrg_t* all = (rrg_t*)calloc((size_t)P * E->world, sizeof(rrg_t));
    sw_jobc* jc = (sw_jobc*)malloc(sizeof(sw_jobc) * NN);
    int32_t* n = (int32_t*)malloc(sizeof(int32_t) * NN);
    uint8_t* y = (uint8_t*)malloc(NN * (size_t)E->T);
    int rc = -1;
    if (!mine || !all || !jc || !n || !y) goto out;
    for (int32_t i = 0; i < E->NL; ++i) {
        mine[i].c = E->jc[i];
        mine[i].m = E->y[SW_Y_BEST][i];
        mine[i].n = E->arr[SW_A_NFIN][i];
    }
    rc = E->comm->allgather(E->comm->ctx, mine, all, P * (int64_t)sizeof(rrg_t));
    if (rc) goto out;
    for (int64_t j = 0; j < N; ++j) { /* blocks are P long and contiguous: job j at j */
        jc[j] = all[j].c;
        n[j] = all[j].n;
        for (int32_t t = 0; t < E->T; ++t) y[(size_t)j * E->T + t] = (uint8_t)((all[j].m >> t) & 1u);
    }
    int64_t passes = 0;
    *moves = twin_reround_arrays((int32_t)N, E->T, E->G, E->k, E->nb, E->beta, E->ell, jc, n, y,
                                 &passes);
    for (int32_t i = 0; i < E->NL; ++i) {
        const int64_t j = E->off + i;
        uint64_t m = 0;
        for (int32_t t = 0; t < E->T; ++t) m |= (uint64_t)y[(size_t)j * E->T + t] << t;
        E->y[SW_Y_BEST][i] = m;
        E->arr[SW_A_NFIN][i] = n[j];
    }
out:
    free(mine); free(all); free(jc); free(n); free(y);
    return rc;
}

/*
 * One rank's sharded solve (same contract as sw_dist_plan_solve): `local`
 * holds this rank's jobs, [job_offset, job_offset + local->num_jobs) of
 * total_jobs, which must be sw_shard_range(total_jobs, world, rank).
 */
int shard_twin_solve(const sw_host_comm* comm, int32_t rank, int32_t world, const sw_problem* local,
                     int64_t job_offset, int64_t total_jobs, sw_result* res) {
    int64_t lo, hi;
    if (sw_validate_problem(local) != 0) return SW_ERR_INVALID;
    if (sw_shard_range(total_jobs, world, rank, &lo, &hi) != 0) return SW_ERR_INVALID;
    if (lo != job_offset || hi - lo != local->num_jobs) return SW_ERR_INVALID;
    eng_t E;
    memset(&E, 0, sizeof(E));
    E.comm = comm;
    E.rank = rank;
    E.world = world;
    E.LW = SW_DET_LANES / world;
    E.N = total_jobs;
    E.off = job_offset;
    E.q = (total_jobs + SW_DET_LANES - 1) / SW_DET_LANES;
    if (E.q == 0) E.q = 1;
    E.P = (int64_t)E.LW * E.q;
    E.NL = local->num_jobs;
    E.T = local->future_rounds;
    E.G = local->num_gpus;
    E.nb = local->num_bases;
    E.k = local->regularizer;
    E.beta = local->bases;
    E.ell = local->log_bases;
    sw_pwl_slopes(E.nb, E.beta, E.ell, E.slope);
    E.p = local->priority;
    E.res = res;
    const size_t NN = E.NL > 0 ? (size_t)E.NL : 1;
    E.jc = (sw_jobc*)malloc(sizeof(sw_jobc) * NN);
    E.Tj = (int32_t*)malloc(sizeof(int32_t) * NN);
    E.key = (float*)malloc(sizeof(float) * NN * E.T);
    E.l = (int32_t*)calloc(NN, sizeof(int32_t));
    E.taken = (int32_t*)calloc(NN, sizeof(int32_t));
    for (int a = 0; a < SW_A_COUNT; ++a) E.arr[a] = (int32_t*)calloc(NN, sizeof(int32_t));
    for (int a = 0; a < SW_Y_COUNT; ++a) E.y[a] = (uint64_t*)calloc(NN, sizeof(uint64_t));
    E.w_all = (int32_t*)calloc(total_jobs > 0 ? (size_t)total_jobs : 1, sizeof(int32_t));
    for (int32_t i = 0; i < E.NL; ++i) {
        E.jc[i] = sw_make_jobc((int32_t)total_jobs, E.T, local->round_duration, local->nworkers[i],
                               local->epoch_duration[i], local->completed_epochs[i],
                               local->total_epochs[i], local->remaining_runtime[i],
                               local->priority[i]);
        E.Tj[i] = local->nworkers[i] <= E.G ? E.T : 0;
    }
    sw_shard_ops ops;
    ops.ctx = &E;
    ops.setup = e_setup;
    ops.widths = e_widths;
    ops.force = e_force;
    ops.count_gt = e_count_gt;
    ops.feasible = e_feasible;
    ops.gather = e_gather;
    ops.between = e_between;
    ops.take_all = e_take_all;
    ops.take = e_take;
    ops.assign = e_assign;
    ops.tail_best = e_tail_best;
    ops.tail_apply = e_tail_apply;
    ops.eval = e_eval;
    ops.copy = e_copy;
    ops.copy_y = e_copy_y;
    ops.pack = e_pack;
    ops.class_caps = e_class_caps;
    ops.pack_class = e_pack_class;
    ops.fill_best = e_fill_best;
    ops.fill_apply = e_fill_apply;
    ops.p2x = e_p2x;
    ops.reround = e_reround;
    ops.search = NULL; /* the controller's own K-ary loop */
    ops.pack_share = e_pack_share;
    ops.share_repair = e_share_repair;
    ops.raise_stats = e_raise_stats;
    ops.raise_best = e_raise_best;
    int rc = sw_shard_solve(&ops, total_jobs, E.T, E.G, E.k, &res->objective, &res->utility,
                            &res->makespan, &res->p2_objective, &res->bound, &res->iters,
                            &res->status);
    free(E.jc); free(E.Tj); free(E.key); free(E.l); free(E.taken); free(E.w_all);
    for (int a = 0; a < SW_A_COUNT; ++a) free(E.arr[a]);
    for (int a = 0; a < SW_Y_COUNT; ++a) free(E.y[a]);
    return rc < 0 ? SW_ERR_RCCL : rc;
}

/* raises (sw_shard_ops.raise_stats / raise_best) */
static int e_raise_stats(void* ctx, double M, int64_t out[3]) {
    eng_t* E = (eng_t*)ctx;
    /* this rank: the first job at M (global index, or INT64_MAX), #{g = M},
     * max{g < M}, max g, Σ w·nfin — gathered, merged in rank order */
    int64_t mine[5] = {INT64_MAX, 0, 0, 0, 0};
    double mlt = 0.0, mall = 0.0;
    for (int32_t i = 0; i < E->NL; ++i) {
        const int32_t n = E->arr[SW_A_NFIN][i];
        const double g = sw_g(&E->jc[i], n);
        if (g == M) { if (mine[0] == INT64_MAX) mine[0] = E->off + i; mine[1] += 1; }
        else if (g < M) mlt = sw_max(mlt, g);
        mall = sw_max(mall, g);
        mine[4] += (int64_t)E->jc[i].w * n;
    }
    mine[2] = (int64_t)sw_bits(mlt);
    mine[3] = (int64_t)sw_bits(mall);
    int64_t* all = (int64_t*)calloc((size_t)5 * E->world, sizeof(int64_t));
    if (!all) return -1;
    int rc = E->comm->allgather(E->comm->ctx, mine, all, 5 * (int64_t)sizeof(int64_t));
    if (!rc) {
        int32_t owner = -1;
        out[0] = INT64_MAX;
        out[2] = 0;
        for (int32_t r = 0; r < E->world; ++r) {
            const int64_t* b = all + (size_t)5 * r;
            if (owner < 0 && b[0] != INT64_MAX) { owner = r; out[0] = b[0]; }
            out[2] += b[4];
        }
        double M2 = 0.0;
        for (int32_t r = 0; r < E->world; ++r) {
            const int64_t* b = all + (size_t)5 * r;
            const double v = r == owner ? (b[1] >= 2 ? M : sw_from_bits((uint64_t)b[2]))
                                        : sw_from_bits((uint64_t)b[3]);
            M2 = sw_max(M2, v);
        }
        out[1] = (int64_t)sw_bits(M2);
    }
    free(all);
    return rc;
}

static int e_raise_best(void* ctx, double M, int64_t i1, double M2, const int64_t* tried, int32_t ntried,
                        uint64_t* best) {
    eng_t* E = (eng_t*)ctx;
    uint64_t b = 0;
    for (int32_t i = 0; i < E->NL; ++i) {
        const int64_t j = E->off + i;
        const int32_t n = E->arr[SW_A_NFIN][i];
        if (n >= E->Tj[i]) continue;
        int skip = 0;
        for (int32_t q = 0; q < ntried; ++q) skip |= tried[q] == j;
        if (skip) continue;
        const double Mo = j == i1 ? M2 : M;
        const uint64_t key = sw_fill_key(sw_raise_gain(fv(E, i, n), fv(E, i, n + 1), sw_g(&E->jc[i], n + 1),
                                                       Mo, M, E->k), j, 0);
        b = key > b ? key : b;
    }
    *best = b;
    return E->comm->allreduce_max_u64(E->comm->ctx, best, 1);
}

/* sw_share_caps (sw_shard_ctl.h) for tests/test_shard.py's property test. */
int shard_share_caps(const int64_t* loads, int32_t W, int32_t rank, int32_t T, int64_t G, int32_t* caps) {
    return sw_share_caps(loads, W, rank, T, G, caps);
}

/* sw_search_resolve (sw_shard_ctl.h) for tests/test_shard.py's property test. */
uint64_t shard_search_resolve(uint64_t lo, uint64_t hi, int64_t chi, int64_t bud, const uint64_t* v,
                              const int64_t* w, int32_t n) {
    return sw_search_resolve(lo, hi, chi, bud, v, w, n);
}
