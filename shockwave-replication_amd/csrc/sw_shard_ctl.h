/*
 * sw_shard_ctl.h — controller of the SHARDED single-instance plan solve
 * (jobs split across ranks, one process per GPU).
 *
 * Plain C99 (compiled by hipcc into the product library and by gcc into the
 * CPU test engine oracle/shard_twin.c).  The controller is the algorithm of
 * oracle/plan_twin.c rewritten as a sequence of STEPS; every
 * step is a local pass over this rank's jobs followed by one collective, done
 * by a "shard engine" behind the sw_shard_ops table:
 *
 *   product engine  sw_shard.hip   — HIP kernels over the rank's jobs in HBM,
 *                                    RCCL (xGMI) or host collectives
 *   CPU engine      oracle/shard_twin.c — test infrastructure only
 *
 * Every engine returns GLOBAL values (after its collective), so the control
 * flow is identical on every rank.
 *
 * Bit-identity with the single-instance solve.  Jobs are sharded along the
 * SW_DET_LANES lanes of the deterministic sum (sw_detsum: lane L sums jobs
 * [L·q, (L+1)·q), q = ⌈N/512⌉): rank r owns lanes [r·512/W, (r+1)·512/W) and
 * therefore jobs [r·(512/W)·q, (r+1)·(512/W)·q) (sw_shard_range).  Engines
 * return the per-lane partial sums of their own lanes, gathered in rank
 * order, and the controller runs the same halving tree as sw_detsum.  Integer
 * sums and maxima are order free, the tie group's job-ordered prefix becomes
 * a rank-exclusive prefix, and the width tail's arg-max is a global max of
 * (key, ~job).  So for every world size W | 512 the sharded solve returns the
 * same plan, counts and objective bits as sw_plan_solve / plan_twin.c on the
 * whole instance (tests/test_shard.py).
 *
 * Fewer collectives.  The two bisections of the twin (the fp32 price bits in
 * SELECT, the fp64 makespan bits of the feasibility search) become K-ary
 * searches: one step evaluates up to SW_SHARD_K thresholds and one
 * all-reduce carries all K counts.  The predicate is monotone, so the K-ary
 * search returns exactly the bisection's answer in ⌈bits / log2(K+1)⌉ steps
 * (K = 255: 31 → 4 for the price, ≤ 64 → 8 for the level; 63 thresholds took
 * 6 and 11).  Once a probe round has left a bracket whose items weigh at
 * most SW_GATHER_CAP (its two ends' counts are known), the next step gathers
 * those items instead of probing again and the answer is read off them
 * (sw_search_resolve): the same answer, as the predicate only changes at item
 * values.  The C4 level search takes 2 steps instead of 7 (706 items lie in
 * its first bracket, 5 in the second), its price search 3 instead of 4.
 */
#ifndef SW_SHARD_CTL_H
#define SW_SHARD_CTL_H

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "sw_arith.h"
#include "sw_bnb.h"
#include "sw_repair.h"

#define SW_SHARD_K 255 /* thresholds evaluated per search step (≤ 255: one per thread of a probe block) */
#define SW_GATHER_CAP 512 /* items a search's gathering step may collect (w ≥ 1: weight bounds the count) */
#define SW_CLASS_HIST (-2) /* class_caps: the class's count histogram */

/* per-job count arrays an engine keeps for its jobs */
enum {
    SW_A_N = 0,     /* current SELECT counts (twin: n)             */
    SW_A_NB = 1,    /* best level-search counts (twin: nb)         */
    SW_A_NFIN = 2,  /* best packed P1 counts (twin: nbest)         */
    SW_A_PL = 3,    /* placed counts of the last pack (twin: placed) */
    SW_A_PL2 = 4,   /* placed counts of pack order B (placed2)     */
    SW_A_COUNT = 5
};
/* per-job round bitmasks (bit t = runs in future round t) */
enum { SW_Y_CUR = 0, SW_Y_BEST = 1, SW_Y_2 = 2, SW_Y_COUNT = 3 };

/* eval selectors: which per-job quantities a reduction step sums */
enum {
    SW_EV_SELECT = 0, /* A: f(n)  B: f(l + taken)  gm: g(n)                        */
    SW_EV_GMAX = 1,   /* gm: g(arr[arg])                                             */
    SW_EV_PACKED = 2, /* A: f(arr[arg])  gm: g(arr[arg])  isum: Σ w·(nb − arr[arg])  */
    SW_EV_P2OK = 3,   /* isum: #{j : placed ≠ nfin}                                  */
    SW_EV_FINAL = 4,  /* y = Y[arg]: c = popcount(y); A: f(c)  B: S(y)/c·p  gm: g(c)
                         isum: #{c > 0}; also writes the plan rows and counts        */
    SW_EV_UNPLACED = 5, /* isum: #{j : arr[arg & 0xFF]_j ≠ arr[arg >> 8]_j}          */
    SW_EV_UMAX = 6      /* A: f(T_j) (every job all its rounds)                       */
};

typedef struct sw_shard_ops {
    void* ctx;
    /* constants, key rows; A = max_j a_j, lb = max_j g_j(T_j), top = max_j
     * g_j(0) */
    int (*setup)(void* ctx, double* A, double* lb, double* top);
    /* w_all[N] = every job's width (gathered) — only the width tail and the
     * fill need it, so it is gathered when one of them first runs */
    int (*widths)(void* ctx, int32_t* w_all);
    /* l_j := #{n < T_j : g_j(n) > M} (0 if is_inf); out = (Σ w·l, Σ w·(T_j − l)) */
    int (*force)(void* ctx, double M, int32_t is_inf, int64_t out[2]);
    /* out[i] = Σ w·#{n ∈ [l_j, T_j) : key_j(n) > rho[i]}, and out[K] = the
     * same count of keys ≥ lo (the bracket's lower end: bits ≥ lo) */
    int (*count_gt)(void* ctx, const uint32_t* rho, int32_t K, uint64_t lo, int64_t* out);
    /* out[i] = Σ w·#{n < T_j : g_j(n) > M[i]}, out[K] = #{bits(g) ≥ lo} alike */
    int (*feasible)(void* ctx, const double* M, int32_t K, uint64_t lo, int64_t* out);
    /* out = #{(j, n ≤ T_j) : a < g_j(n) < b} */
    int (*between)(void* ctx, double a, double b, int64_t* out);
    /* n := T_j, taken := T_j − l */
    int (*take_all)(void* ctx);
    /* taken_j := count(key > rho), tie_j := count(key ≥ rho) − taken_j;
     * wt = Σ_all w·taken, excl = Σ over ranks before this one of w·tie */
    int (*take)(void* ctx, uint32_t rho, int64_t* wt, int64_t* excl);
    /* tie group in job order; n := l + taken + tt; used = Σ_all w·tt */
    int (*assign)(void* ctx, uint32_t rho, int64_t rem, int64_t excl, int64_t* used);
    /* max over jobs with n < T_j and w ≤ rem2 of key(n) << 32 | ~j (0 if none) */
    int (*tail_best)(void* ctx, int64_t rem2, uint64_t* best);
    /* n[jb] += 1 on the rank owning global job jb */
    int (*tail_apply)(void* ctx, int64_t jb);
    /* reductions: lanesA/lanesB receive all SW_DET_LANES lane partials (rank
     * order), gm the max, isum the integer sum */
    int (*eval)(void* ctx, int32_t sel, int32_t arg, double* lanesA, double* lanesB, double* gm,
                int64_t* isum);
    int (*copy)(void* ctx, int32_t dst, int32_t src);   /* count arrays */
    int (*copy_y)(void* ctx, int32_t dst, int32_t src); /* bitmask arrays */
    /* place arr[src] rounds per job (twin: pack); mode 1/3 = P1 orders A/B
     * (Mb = makespan of arr[src]), 2 = P2 weight order p/n, 4 = P2 density
     * order p/(n·w).  Writes Y[ydst], arr[pdst] */
    int (*pack)(void* ctx, int32_t mode, int32_t src, double Mb, int32_t ydst, int32_t pdst);
    /* width-class profile (twin: the (c) placement and repair_pack).
     * caps[t] = #{j : arr[src]_j > 0, w_j = wc, bit t of Y[ysrc]_j} summed over
     * all ranks; next_w = the smallest width > wc among jobs with
     * arr[src]_j > 0 (0x7FFFFFFF if none); with psrc ≥ 0 also md[0] = #{j :
     * arr[src]_j > 0, w_j = wc} and md[1] = Σ over them of arr[src]_j −
     * arr[psrc]_j (the class's unplaced rounds) */
    int (*class_caps)(void* ctx, int32_t src, int32_t ysrc, int32_t wc, int32_t psrc,
                      int32_t* caps, int32_t* next_w, int64_t* md);
    /* (psrc = SW_CLASS_HIST: caps[v − 1] = #{j : arr[src]_j = v, w_j = wc}
     * for v = 1..T instead, the count histogram of the class; md[0] as above) */
    /* pack the jobs of width wc (arr[src] rounds, order p/n, unit widths) into
     * per-round capacities caps; writes their rows of Y[ydst] and arr[pdst]
     * and leaves every other job untouched */
    int (*pack_class)(void* ctx, int32_t src, int32_t wc, const int32_t* caps, int32_t ydst,
                      int32_t pdst);
    /* fill of stranded capacity (twin: fill_stranded): best = max over jobs
     * with arr[SW_A_NFIN]_j < T_j of sw_fill_key(f(n+1) − f(n), j, t), t the
     * first round without j in Y[SW_Y_BEST] with w_j ≤ G − load[t] (0 if
     * none); fill_apply sets bit t of job jb's Y[SW_Y_BEST] row and adds one
     * to its arr[SW_A_NFIN] on the owning rank */
    int (*fill_best)(void* ctx, const int64_t* load, uint64_t* best);
    int (*fill_apply)(void* ctx, int64_t jb, int32_t t);
    /* the P2 exchange step (sw_p2x.h) on the placement Y[ysrc] of the counts
     * arr[nsrc]: the active jobs' rows are gathered, the step runs on every
     * rank alike and each rank keeps its own rows; *cancels = cycles applied */
    int (*p2x)(void* ctx, int32_t ysrc, int32_t nsrc, int32_t* cancels);
    /* per-round exact re-optimisation (sw_reround.h) of the re-solved P1
     * plan Y[SW_Y_BEST] / arr[SW_A_NFIN]: every job's constants, row and
     * count are gathered, the step runs on every rank alike and each rank
     * keeps its own rows and counts; *moves = rounds whose set changed */
    int (*reround)(void* ctx, int32_t* moves);
    /* the items of a search bracket, over all ranks (rank order): value bits
     * in [lo, hi] — kind 0 the key bits of n ∈ [l_j, T_j), kind 1 the bits
     * of g_j(n), n < T_j — as (v, w_j) pairs; *n ≤ SW_GATHER_CAP (asked only
     * when the bracket's weight says so) */
    int (*gather)(void* ctx, int32_t kind, uint64_t lo, uint64_t hi, uint64_t* v, int64_t* w, int32_t* n);
    /* optional (NULL = the controller drives count_gt / feasible / gather
     * itself): the whole search of swc_search inside the engine — kind 0 over
     * count_gt, 1 over feasible; chi = Σ w·#{v > hi} when known, else −1 —
     * returning its answer and the number of rounds (collective steps) it
     * took, which must equal swc_search's */
    int (*search)(void* ctx, int32_t kind, uint64_t lo, uint64_t hi, int64_t bud, int64_t chi, uint64_t* out,
                  int32_t* rounds);
    /* the share placement: the ranks' loads Σ w·arr[src]
     * are all-gathered, sw_share_caps gives this rank its share of every
     * round's capacity, and the rank places its own jobs there alone
     * (density order p/(n·w), the tier rule over its per-round shares) into
     * Y[ydst] / arr[pdst] — no gathered placement.  share_repair repairs
     * this rank's width profile inside its shares (sw_profile_repair) when
     * the pack stranded rounds of its own jobs; no collective. */
    int (*pack_share)(void* ctx, int32_t src, int32_t ydst, int32_t pdst);
    int (*share_repair)(void* ctx, int32_t src, int32_t ydst, int32_t pdst);
    /* raises (sw_arith.h SW_RAISE_ITERS) on the plan arr[SW_A_NFIN], M its
     * makespan: out[0] = the first job j with g_j(nfin_j) = M, out[1] = the
     * bits of max_{j ≠ out[0]} g_j(nfin_j), out[2] = Σ w·nfin, all ranks */
    int (*raise_stats)(void* ctx, double M, int64_t out[3]);
    /* max over jobs with nfin_j < T_j not in tried[0..ntried) of
     * sw_fill_key(sw_raise_gain(…), j, 0), Mo = M2 for job i1 and M else */
    int (*raise_best)(void* ctx, double M, int64_t i1, double M2, const int64_t* tried, int32_t ntried,
                      uint64_t* best);
} sw_shard_ops;

/* Job range of `rank` (sw_dist_shard_range in include/shockwave_amd.h). */
static inline int sw_shard_range(int64_t N, int32_t world, int32_t rank, int64_t* lo, int64_t* hi) {
    if (world < 1 || world > SW_DET_LANES || (SW_DET_LANES % world) != 0 || rank < 0 ||
        rank >= world || N < 0)
        return -1;
    const int64_t q = (N + SW_DET_LANES - 1) / SW_DET_LANES;
    const int64_t per = (int64_t)(SW_DET_LANES / world) * q;
    int64_t a = (int64_t)rank * per, b = a + per;
    *lo = a < N ? a : N;
    *hi = b < N ? b : N;
    return 0;
}

/*
 * The share placement's per-round capacities of rank `rank`.
 * loads[r] = Σ w_j·n_j over rank r's jobs, L = Σ_r loads[r] ≤ G·T.  Rank r's
 * budget is B_r = loads[r] + its share of the slack S = G·T − L: ⌊S·L_r/L⌋,
 * and one more unit for each of the first S − Σ_r ⌊S·L_r/L⌋ ranks.  It gets
 * ⌊B_r/T⌋ GPUs in every round and one more in B_r mod T rounds; those
 * extras are one stream over the ranks in rank order (rank r's start at
 * round Σ_{r' < r} (B_r' mod T) mod T and wrap), and Σ_r B_r = G·T, so every
 * round's shares sum to exactly G.  Each rank then holds at least its own
 * load, spread like the whole instance's capacity (flat, so its density
 * order front-loads its jobs as the whole instance's would).  At world 1 the
 * share is G in every round: the single-instance pack.  Returns 0, or -1
 * when L = 0, L > G·T or G·T ≥ 2^31 (no share placement).  "Rank" here is a
 * share (sw_share_count).
 */
static inline int sw_share_caps(const int64_t* loads, int32_t W, int32_t rank, int32_t T, int64_t G,
                                int32_t* caps) {
    __int128 L = 0;
    for (int32_t r = 0; r < W; ++r) L += loads[r];
    const __int128 C = (__int128)G * T;
    /* C < 2^31: the engines' 64-bit restatement (k_share_caps) is exact */
    if (L <= 0 || L > C || T < 1 || C >= ((__int128)1 << 31)) return -1;
    const __int128 S = C - L;
    __int128 given = 0;
    for (int32_t r = 0; r < W; ++r) given += S * loads[r] / L;
    const int64_t rest = (int64_t)(S - given); /* < W */
    int64_t cursor = 0, Bme = 0;
    for (int32_t r = 0; r <= rank; ++r) {
        const int64_t B = loads[r] + (int64_t)(S * loads[r] / L) + (r < rest ? 1 : 0);
        if (r < rank) cursor = (cursor + B % T) % T;
        else Bme = B;
    }
    const int64_t base = Bme / T, ext = Bme % T;
    for (int32_t t = 0; t < T; ++t) {
        const int64_t d = ((int64_t)t - cursor + T) % T; /* position in this rank's extras */
        caps[t] = (int32_t)(base + (d < ext ? 1 : 0));
    }
    return 0;
}

/*
 * Shares of the share placement.  A large instance (at least
 * SW_VSHARE_MIN_JOBS jobs on at least SW_VSHARE_MIN_GPUS GPUs) is placed in
 * SW_VSHARES lane-aligned shares whatever the world size: share v holds the
 * jobs sw_shard_range(N, SW_VSHARES, v) and rank r of W (W | SW_VSHARES)
 * places shares r·S … r·S + S − 1, S = SW_VSHARES / W, one workgroup each.
 * So the placement — and with it the whole solve — is the same at W = 1, 2,
 * 4 and 8, and a rank's round loops run side by side on S workgroups instead
 * of one loop over all its jobs.  Smaller instances, and worlds above
 * SW_VSHARES, keep one share per rank (at W = 1 the single-instance pack).
 */
#define SW_VSHARES 8
#define SW_VSHARE_MIN_JOBS 4096
#define SW_VSHARE_MAX_JOBS 65536 /* a share's round loop: at most 20·512 entries */
#define SW_VSHARE_MIN_GPUS 512
static inline int32_t sw_share_count(int64_t N, int64_t G, int32_t W) {
    return (W < SW_VSHARES && N >= SW_VSHARE_MIN_JOBS && N <= SW_VSHARE_MAX_JOBS && G >= SW_VSHARE_MIN_GPUS)
               ? SW_VSHARES
               : W;
}

/* The combining phase of sw_detsum (oracle/plan_twin.c) over the lane partials. */
static inline double sw_shard_tree(const double* lanes) {
    double part[SW_DET_LANES];
    double wsum[SW_DET_LANES / 64];
    memcpy(part, lanes, sizeof(part));
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

typedef struct {
    const sw_shard_ops* ops;
    int64_t N;
    int32_t T, G;
    int64_t C;
    double k, A, lb, top;
    int32_t* w_all;
    int w_ok;      /* w_all gathered */
    int64_t steps; /* collective steps taken (reported as iters) */
    double lanesA[SW_DET_LANES], lanesB[SW_DET_LANES];
} sw_shard_ctl;

typedef struct {
    double U, Mact, J, ubound;
    uint32_t rho; /* price ρ* bits (0 when every item fits) */
} sw_shard_eval;

#define SWC_TRY(x)              \
    do {                        \
        int rc_ = (x);          \
        if (rc_ < 0) return rc_; \
    } while (0)

/*
 * A search step's kind (swc_search, and the engines' device-chained rounds):
 * 0 = the bracket [lo, hi) is closed, 2 = gather its items (both ends'
 * counts known: clo = Σ w·#{v ≥ lo}, chi = Σ w·#{v > hi}, and clo − chi ≤
 * SW_GATHER_CAP), 1 = probe K thresholds.
 */
SW_HD int sw_search_mode(uint64_t lo, uint64_t hi, int64_t clo, int64_t chi) {
    if (lo >= hi) return 0;
    return (clo >= 0 && chi >= 0 && clo - chi <= SW_GATHER_CAP) ? 2 : 1;
}

/*
 * The answer of a gathered bracket: the smallest x in [lo, hi) with chi +
 * Σ_{v_i > x} w_i ≤ bud, else hi.  The sum only changes at the items' values,
 * so x is lo or one of them (the engines compute the same integers in
 * parallel: each item's sum over all items, then a minimum).
 */
static inline uint64_t sw_search_resolve(uint64_t lo, uint64_t hi, int64_t chi, int64_t bud, const uint64_t* v,
                                         const int64_t* w, int32_t n) {
    uint64_t best = hi;
    int64_t s = chi;
    for (int32_t k = 0; k < n; ++k) s += v[k] > lo ? w[k] : 0;
    if (s <= bud) best = lo;
    for (int32_t i = 0; i < n; ++i) {
        int64_t si = chi;
        for (int32_t k = 0; k < n; ++k) si += v[k] > v[i] ? w[k] : 0;
        if (si <= bud && v[i] < best) best = v[i];
    }
    return best;
}

/*
 * K-ary search for the smallest x in [lo, hi) with pred(x) true, else hi —
 * the twin's bisection `while (lo < hi) { mid; pred(mid) ? hi = mid : lo =
 * mid + 1; }` for a monotone predicate.  kind 0: pred(x) = Σ w·cnt_gt(x) ≤
 * bud (price bits); kind 1: pred(x) = Σ w·lforce(bits→double x) ≤ bud.  chi
 * = Σ w·#{v > hi} when the caller knows it (no item lies above the level
 * search's top, no key above SW_KEY_INF_BITS), else −1.  A probe round keeps
 * its counts at the new bracket's ends; a bracket of small weight is then
 * gathered and resolved in one step (sw_search_mode).
 */
static inline int swc_search(sw_shard_ctl* c, int kind, uint64_t lo, uint64_t hi, int64_t bud, int64_t chi,
                             uint64_t* out) {
    uint64_t pts[SW_SHARD_K];
    uint32_t rho[SW_SHARD_K];
    double Ms[SW_SHARD_K];
    int64_t cnt[SW_SHARD_K + 1];
    uint64_t gv[SW_GATHER_CAP];
    int64_t gw[SW_GATHER_CAP];
    if (c->ops->search) {
        int32_t rounds = 0;
        SWC_TRY(c->ops->search(c->ops->ctx, kind, lo, hi, bud, chi, out, &rounds));
        c->steps += rounds;
        return 0;
    }
    int64_t clo = -1;
    while (lo < hi) {
        if (sw_search_mode(lo, hi, clo, chi) == 2) {
            int32_t n = 0;
            SWC_TRY(c->ops->gather(c->ops->ctx, kind, lo, hi, gv, gw, &n));
            c->steps++;
            if (n < 0 || n > SW_GATHER_CAP) return -3;
            lo = sw_search_resolve(lo, hi, chi, bud, gv, gw, n);
            break;
        }
        const uint64_t span = hi - lo;
        const int32_t K = span < (uint64_t)SW_SHARD_K ? (int32_t)span : SW_SHARD_K;
        const uint64_t d = (uint64_t)K + 1u, a = span / d, b = span % d;
        for (int32_t i = 0; i < K; ++i) {
            const uint64_t m = (uint64_t)(i + 1);
            pts[i] = lo + a * m + (b * m) / d;
            rho[i] = (uint32_t)pts[i];
            Ms[i] = sw_from_bits(pts[i]);
        }
        if (kind == 0) SWC_TRY(c->ops->count_gt(c->ops->ctx, rho, K, lo, cnt));
        else SWC_TRY(c->ops->feasible(c->ops->ctx, Ms, K, lo, cnt));
        c->steps++;
        int32_t f = K;
        for (int32_t i = 0; i < K; ++i)
            if (cnt[i] <= bud) { f = i; break; }
        if (f < K) {
            hi = pts[f];
            chi = cnt[f];
            if (f > 0) { lo = pts[f - 1] + 1u; clo = cnt[f - 1]; }
            else clo = cnt[K]; /* lo stays: its count from this round */
        } else {
            lo = pts[K - 1] + 1u;
            clo = cnt[K - 1];
        }
    }
    *out = lo;
    return 0;
}

/* job j's width, the widths gathered on first use (one collective step) */
static inline int swc_width(sw_shard_ctl* c, int64_t j, int32_t* w) {
    if (!c->w_ok) {
        SWC_TRY(c->ops->widths(c->ops->ctx, c->w_all));
        c->steps++;
        c->w_ok = 1;
    }
    *w = c->w_all[j];
    return 0;
}

/* twin: select_level ([plo, phi] brackets ρ*(M), see there) */
static inline int swc_select(sw_shard_ctl* c, double M, int is_inf, sw_shard_eval* ev,
                             uint32_t plo, uint32_t phi) {
    const sw_shard_ops* o = c->ops;
    int64_t wfa[2];
    SWC_TRY(o->force(o->ctx, M, is_inf, wfa));
    c->steps++;
    const int64_t Wf = wfa[0], Wall = wfa[1];
    ev->rho = 0;
    if (Wf > c->C) {
        ev->U = 0.0; ev->Mact = 0.0; ev->J = -1e308; ev->ubound = 0.0;
        return 0;
    }
    const int64_t bud = c->C - Wf;
    double rho_d = 0.0;
    int64_t wgt_star;
    if (Wall <= bud) {
        SWC_TRY(o->take_all(o->ctx));
        wgt_star = Wall;
    } else {
        uint64_t r64;
        SWC_TRY(swc_search(c, 0, plo, phi, bud, phi == SW_KEY_INF_BITS ? 0 : -1, &r64));
        const uint32_t rho = (uint32_t)r64;
        ev->rho = rho;
        rho_d = (double)sw_float_of(rho);
        int64_t wt, excl, used;
        SWC_TRY(o->take(o->ctx, rho, &wt, &excl));
        c->steps++;
        wgt_star = wt;
        const int64_t rem = bud - wt;
        SWC_TRY(o->assign(o->ctx, rho, rem, excl, &used));
        c->steps++;
        int64_t rem2 = rem - used;
        while (rem2 > 0) {
            uint64_t best;
            SWC_TRY(o->tail_best(o->ctx, rem2, &best));
            c->steps++;
            if (best == 0) break;
            const int64_t jb = (int64_t)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu));
            SWC_TRY(o->tail_apply(o->ctx, jb));
            int32_t wb;
            SWC_TRY(swc_width(c, jb, &wb));
            rem2 -= wb;
        }
    }
    double gm;
    int64_t isum;
    SWC_TRY(o->eval(o->ctx, SW_EV_SELECT, 0, c->lanesA, c->lanesB, &gm, &isum));
    c->steps++;
    ev->U = sw_shard_tree(c->lanesA);
    ev->Mact = gm;
    ev->J = ev->U - c->k * gm;
    ev->ubound = sw_shard_tree(c->lanesB) + (rho_d * c->A) * (double)(bud - wgt_star);
    return 0;
}

static inline int swc_keep(sw_shard_ctl* c, const sw_shard_eval* e, sw_shard_eval* best) {
    if (e->J > best->J || (e->J == best->J && e->Mact < best->Mact)) {
        *best = *e;
        SWC_TRY(c->ops->copy(c->ops->ctx, SW_A_NB, SW_A_N));
    }
    return 0;
}

/* twin: level_search — best counts in SW_A_NB; *bound as the twin; *mk =
 * the makespan max_j g_j(nb_j) of those counts, which the winning level's
 * SELECT evaluation already reduced (so the solve needs no GMAX step) */
static inline int swc_level_search(sw_shard_ctl* c, double* bound, double* mk) {
    const sw_shard_ops* o = c->ops;
    sw_shard_eval ev, best, elo;
    if (!(c->N > 0 && c->k > 0.0)) { /* no makespan term: the utility optimum */
        SWC_TRY(swc_select(c, 0.0, 1, &ev, 0, SW_KEY_INF_BITS));
        SWC_TRY(o->copy(o->ctx, SW_A_NB, SW_A_N));
        *bound = ev.ubound - c->k * ev.Mact;
        *mk = ev.Mact;
        return 0;
    }
    uint64_t lo;
    /* no item lies above top = max_j g_j(0): chi = 0 */
    SWC_TRY(swc_search(c, 1, sw_bits(c->lb), sw_bits(c->top), c->C, 0, &lo));
    const double M_lo = sw_from_bits(lo);
    SWC_TRY(swc_select(c, M_lo, 0, &elo, 0, SW_KEY_INF_BITS));
    best = elo;
    SWC_TRY(o->copy(o->ctx, SW_A_NB, SW_A_N));
    /* a higher level can win only below M_lo + (U_max − U(M_lo))/k (twin) */
    double gm;
    int64_t isum, nbw = 0;
    SWC_TRY(o->eval(o->ctx, SW_EV_UMAX, 0, c->lanesA, c->lanesB, &gm, &isum));
    c->steps++;
    const double U_max = sw_shard_tree(c->lanesA);
    const double wmax = (U_max - elo.U) / c->k;
    if (wmax > 0.0) {
        SWC_TRY(o->between(o->ctx, M_lo, M_lo + wmax, &nbw));
        c->steps++;
    }
    if (nbw == 0) {
        *bound = elo.ubound - c->k * M_lo;
        *mk = best.Mact;
        return 0;
    }
    SWC_TRY(swc_select(c, 0.0, 1, &ev, 0, elo.rho));
    SWC_TRY(swc_keep(c, &ev, &best));
    /* branch and bound over the levels in (M_lo, M_free] (twin; sw_bnb.h) */
    const double kk = c->k, M_free = ev.Mact;
    double cert = sw_max(elo.ubound - kk * M_lo, ev.ubound - kk * M_free);
    sw_bnb_ivl L[SW_BNB_CAP];
    int32_t nL = 0, probes = 0;
    if (M_lo < M_free) L[nL++] = sw_bnb_make(M_lo, M_free, ev.ubound, elo.rho, ev.rho);
    while (nL > 0) {
        double kb;
        const int32_t i = sw_bnb_pick(L, nL, kk, &kb);
        if (kb <= best.J) break;
        if (probes == SW_BNB_PROBES) { cert = sw_max(cert, kb); break; }
        const sw_bnb_ivl I = L[i];
        L[i] = L[--nL];
        SWC_TRY(o->between(o->ctx, I.a, I.b, &nbw));
        c->steps++;
        if (nbw == 0) {
            cert = sw_max(cert, I.vb - kk * I.b);
            continue;
        }
        const double m = sw_bnb_mid(I.a, I.b);
        sw_shard_eval e;
        SWC_TRY(swc_select(c, m, 0, &e, I.rb, I.ra));
        ++probes;
        SWC_TRY(swc_keep(c, &e, &best));
        if (sw_bnb_key(e.ubound, kk, I.a) > best.J) L[nL++] = sw_bnb_make(I.a, m, e.ubound, I.ra, e.rho);
        if (sw_bnb_key(I.vb, kk, m) > best.J) L[nL++] = sw_bnb_make(m, I.b, I.vb, e.rho, I.rb);
    }
    *bound = sw_max(cert, best.J);
    *mk = best.Mact;
    return 0;
}

/* twin: repair_pack — the density pack (Y[ysrc], arr[psrc]) of arr[nin]
 * stranded rounds: gather the width-class profile, repair it on the host
 * (sw_repair.h, identical on every rank), repack every changed class into
 * Y[ydst] / arr[pdst] (the rest copied from the density pack).  *ok = every
 * round placed. */
static inline int swc_repair(sw_shard_ctl* c, int32_t nin, int32_t ysrc, int32_t psrc,
                             int32_t ydst, int32_t pdst, int* ok) {
    const sw_shard_ops* o = c->ops;
    sw_repair_t R;
    int32_t caps[SW_TMAX];
    int32_t next_w = 0, wc;
    int64_t md[2] = {0, 0};
    int over = 0;
    memset(&R, 0, sizeof(R));
    *ok = 0;
    SWC_TRY(o->class_caps(o->ctx, nin, ysrc, 0, -1, caps, &next_w, md));
    c->steps++;
    for (int32_t t = 0; t < c->T; ++t) R.L[t] = c->G;
    while (next_w != 0x7FFFFFFF) {
        wc = next_w;
        SWC_TRY(o->class_caps(o->ctx, nin, ysrc, wc, psrc, caps, &next_w, md));
        c->steps++;
        const int32_t ci = sw_repair_add_class(&R, wc);
        if (ci < 0) { over = 1; continue; }
        R.M[ci] = (int32_t)md[0];
        R.D[ci] = (int32_t)md[1];
        for (int32_t t = 0; t < c->T; ++t) {
            R.caps[ci][t] = caps[t];
            R.L[t] -= wc * caps[t];
        }
    }
    if (over || sw_profile_repair(&R, c->T) != 0) return 0;
    SWC_TRY(o->copy_y(o->ctx, ydst, ysrc));
    SWC_TRY(o->copy(o->ctx, pdst, psrc));
    for (int32_t ci = 0; ci < R.ncls; ++ci) {
        if (!R.changed[ci]) continue;
        SWC_TRY(o->pack_class(o->ctx, nin, R.wc[ci], R.caps[ci], ydst, pdst));
        c->steps++;
    }
    double gm;
    int64_t bad;
    SWC_TRY(o->eval(o->ctx, SW_EV_UNPLACED, pdst | (nin << 8), c->lanesA, c->lanesB, &gm, &bad));
    c->steps++;
    *ok = bad == 0;
    return 0;
}

/* twin: pattern_pack — an exact width-class profile over round patterns
 * (sw_profile_search) for arr[nin], from the classes' count histograms
 * (class_caps with psrc = SW_CLASS_HIST); every class is packed inside it
 * into Y[ydst] / arr[pdst], which hold a pack of arr[nin] (every row with a
 * count is rewritten).  *ok = every round placed. */
static inline int swc_pattern(sw_shard_ctl* c, int32_t nin, int32_t ydst, int32_t pdst, int* ok) {
    const sw_shard_ops* o = c->ops;
    sw_repair_t R;
    int32_t hist[SW_RCLS_MAX * (SW_TMAX + 1)];
    int32_t caps[SW_TMAX];
    int32_t next_w = 0, over = 0;
    int64_t md[2] = {0, 0}, A = 0;
    memset(&R, 0, sizeof(R));
    *ok = 0;
    SWC_TRY(o->class_caps(o->ctx, nin, SW_Y_CUR, 0, SW_CLASS_HIST, caps, &next_w, md));
    c->steps++;
    while (next_w != 0x7FFFFFFF) {
        const int32_t wc = next_w;
        SWC_TRY(o->class_caps(o->ctx, nin, SW_Y_CUR, wc, SW_CLASS_HIST, caps, &next_w, md));
        c->steps++;
        const int32_t ci = R.ncls < SW_RCLS_MAX ? sw_repair_add_class(&R, wc) : -1;
        if (ci < 0) { over = 1; break; }
        R.M[ci] = (int32_t)md[0];
        A += md[0];
        hist[ci * (c->T + 1)] = 0;
        for (int32_t v = 1; v <= c->T; ++v) hist[ci * (c->T + 1) + v] = caps[v - 1];
    }
    if (over || A == 0) return 0;
    int32_t* scratch = (int32_t*)malloc(sizeof(int32_t) * (size_t)SW_PAT_SCRATCH(A));
    if (!scratch) return -1;
    const int32_t found = sw_profile_search(&R, c->T, c->G, hist, scratch, NULL);
    free(scratch);
    if (!found) return 0;
    for (int32_t ci = 0; ci < R.ncls; ++ci) {
        SWC_TRY(o->pack_class(o->ctx, nin, R.wc[ci], R.caps[ci], ydst, pdst));
        c->steps++;
    }
    double gm;
    int64_t bad;
    SWC_TRY(o->eval(o->ctx, SW_EV_UNPLACED, pdst | (nin << 8), c->lanesA, c->lanesB, &gm, &bad));
    c->steps++;
    *ok = bad == 0;
    return 0;
}

/*
 * The whole sharded plan solve (twin: twin_plan_solve).  Scalar results are
 * global; the engine's SW_EV_FINAL step wrote this rank's plan rows.
 * Returns SW_OK / SW_FALLBACK (1) or a negative engine error.
 */
static inline int sw_shard_solve(const sw_shard_ops* o, int64_t N, int32_t T, int32_t G, double k,
                                 double* objective, double* utility, double* makespan,
                                 double* p2_objective, double* bound_out, int32_t* iters,
                                 int32_t* status_out) {
    sw_shard_ctl* c = (sw_shard_ctl*)malloc(sizeof(sw_shard_ctl));
    if (!c) return -1;
    c->ops = o;
    c->N = N;
    c->T = T;
    c->G = G;
    c->C = (int64_t)G * T;
    c->k = k;
    c->steps = 0;
    c->w_ok = 0;
    c->w_all = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
    int rc = 0;
    if (!c->w_all) { free(c); return -1; }
#define SWC_RUN(x)                   \
    do {                             \
        rc = (x);                    \
        if (rc < 0) goto done;       \
    } while (0)
    {
        SWC_RUN(o->setup(o->ctx, &c->A, &c->lb, &c->top));
        c->steps++;
        int32_t status = 0;
        double bound = 0.0, Jbest = 0.0, gm;
        int dens_best = 0, dskip_best = 0, rep_best = 0;
        for (int it = 0; it < SW_REPACK_ITERS; ++it) {
            double b0, Mb;
            SWC_RUN(swc_level_search(c, &b0, &Mb));
            if (it == 0) bound = b0;
            int64_t deficit = 0;
            double Jp = 0.0;
            int dens = 0, rep = 0;
            /* the share placement: every rank places its own jobs in its share
             * of each round (no gathered placement); it is P1's and, in density
             * order, P2's.  When it strands rounds on some rank, that rank
             * repairs its profile; if rounds stay unplaced, the gathered orders
             * below decide (the single-instance flow) */
            int ord0 = -1;
            if (o->pack_share) {
                int64_t dfc;
                SWC_RUN(o->pack_share(o->ctx, SW_A_NB, SW_Y_CUR, SW_A_PL));
                c->steps++;
                SWC_RUN(o->eval(o->ctx, SW_EV_PACKED, SW_A_PL, c->lanesA, c->lanesB, &gm, &dfc));
                c->steps++;
                const int repaired = dfc != 0; /* twin: the density pack's repair */
                if (dfc != 0) {
                    SWC_RUN(o->share_repair(o->ctx, SW_A_NB, SW_Y_CUR, SW_A_PL));
                    SWC_RUN(o->eval(o->ctx, SW_EV_PACKED, SW_A_PL, c->lanesA, c->lanesB, &gm, &dfc));
                    c->steps++;
                }
                if (dfc == 0) {
                    Jp = sw_shard_tree(c->lanesA) - c->k * gm;
                    dens = 1;
                    rep = repaired;
                    ord0 = 2; /* placed: no gathered order */
                }
            }
            for (int ord = ord0; ord < 2; ++ord) {
                const int32_t pdst = ord == 1 ? SW_A_PL2 : SW_A_PL;
                const int32_t pm = ord < 0 ? 4 : ord ? 3 : 1;
                SWC_RUN(o->pack(o->ctx, pm, SW_A_NB, Mb, ord == 1 ? SW_Y_2 : SW_Y_CUR, pdst));
                c->steps++;
                int64_t dfc;
                SWC_RUN(o->eval(o->ctx, SW_EV_PACKED, pdst, c->lanesA, c->lanesB, &gm, &dfc));
                c->steps++;
                double Jo = sw_shard_tree(c->lanesA) - c->k * gm;
                if (ord < 0) { /* density order: also the P2 placement when it packs */
                    int rok = 0;
                    if (dfc != 0) SWC_RUN(swc_repair(c, SW_A_NB, SW_Y_CUR, SW_A_PL, SW_Y_2, SW_A_PL2, &rok));
                    if (rok) { /* the repaired placement places every count */
                        SWC_RUN(o->copy_y(o->ctx, SW_Y_CUR, SW_Y_2));
                        SWC_RUN(o->copy(o->ctx, SW_A_PL, SW_A_PL2));
                        SWC_RUN(o->eval(o->ctx, SW_EV_PACKED, SW_A_PL, c->lanesA, c->lanesB, &gm, &dfc));
                        c->steps++;
                        Jo = sw_shard_tree(c->lanesA) - c->k * gm;
                        rep = 1;
                    }
                    if (dfc == 0) { Jp = Jo; dens = 1; break; }
                    continue;
                }
                if (ord == 0 || Jo > Jp) {
                    Jp = Jo;
                    deficit = dfc;
                    if (ord == 1) {
                        SWC_RUN(o->copy(o->ctx, SW_A_PL, SW_A_PL2));
                        SWC_RUN(o->copy_y(o->ctx, SW_Y_CUR, SW_Y_2));
                    }
                }
                if (ord == 0 && dfc == 0) break;
            }
            if (deficit != 0) { /* twin: pattern_pack — the counts as they are */
                int pok = 0;
                SWC_RUN(swc_pattern(c, SW_A_NB, SW_Y_CUR, SW_A_PL, &pok));
                if (pok) {
                    int64_t dfc;
                    SWC_RUN(o->eval(o->ctx, SW_EV_PACKED, SW_A_PL, c->lanesA, c->lanesB, &gm, &dfc));
                    c->steps++;
                    Jp = sw_shard_tree(c->lanesA) - c->k * gm;
                    deficit = 0;
                }
            }
            if (it == 0 || Jp > Jbest) {
                Jbest = Jp;
                dens_best = dens;
                rep_best = rep;
                dskip_best = !dens && deficit == 0;
                SWC_RUN(o->copy(o->ctx, SW_A_NFIN, SW_A_PL));
                SWC_RUN(o->copy_y(o->ctx, SW_Y_BEST, SW_Y_CUR));
            }
            if (deficit == 0) break;
            status |= SW_STATUS_P1_REPACKED;
            c->C -= deficit;
        }
        /* a re-solved P1 can strand capacity: fill it (twin: fill_stranded);
         * the per-round load comes from the width classes' round counts */
        if (status & SW_STATUS_P1_REPACKED) {
            int64_t load[SW_TMAX];
            int32_t caps[SW_TMAX];
            int32_t next_w = 0;
            int64_t md[2];
            for (int32_t t = 0; t < T; ++t) load[t] = 0;
            SWC_RUN(o->class_caps(o->ctx, SW_A_NFIN, SW_Y_BEST, 0, -1, caps, &next_w, md));
            c->steps++;
            while (next_w != 0x7FFFFFFF) {
                const int32_t wc = next_w;
                SWC_RUN(o->class_caps(o->ctx, SW_A_NFIN, SW_Y_BEST, wc, -1, caps, &next_w, md));
                c->steps++;
                for (int32_t t = 0; t < T; ++t) load[t] += (int64_t)wc * caps[t];
            }
            int added = 0;
            for (int step = 0; step < SW_FILL_MAX; ++step) {
                uint64_t best;
                SWC_RUN(o->fill_best(o->ctx, load, &best));
                c->steps++;
                if (best == 0) break;
                const int64_t jb = sw_fill_job(best);
                const int32_t tb = sw_fill_round(best);
                SWC_RUN(o->fill_apply(o->ctx, jb, tb));
                int32_t wb;
                SWC_RUN(swc_width(c, jb, &wb));
                load[tb] += wb;
                ++added;
            }
            if (added > 0) {
                dens_best = 0;
                rep_best = 0;
                dskip_best = 0;
            }
            /* ... and re-optimise it round by round (twin_reround_arrays) */
            int32_t moves = 0;
            SWC_RUN(o->reround(o->ctx, &moves));
            c->steps++;
            if (moves > 0) {
                dens_best = 0;
                rep_best = 0;
                dskip_best = 0;
            }
            /* ... and try raises (twin: raise_counts): one job one more round,
             * the plan re-placed by the pattern search (on arr[SW_A_N], its rows
             * first reset by a density pack) */
            for (int rit = 0; rit < SW_RAISE_ITERS; ++rit) {
                int64_t isum, rs[3];
                SWC_RUN(o->eval(o->ctx, SW_EV_PACKED, SW_A_NFIN, c->lanesA, c->lanesB, &gm, &isum));
                c->steps++;
                const double J = sw_shard_tree(c->lanesA) - c->k * gm, M = gm;
                SWC_RUN(o->raise_stats(o->ctx, M, rs));
                c->steps++;
                const double M2 = sw_from_bits((uint64_t)rs[1]);
                int64_t tried[SW_RAISE_TRIES];
                int took = 0;
                for (int tr = 0; tr < SW_RAISE_TRIES && !took; ++tr) {
                    uint64_t best;
                    SWC_RUN(o->raise_best(o->ctx, M, rs[0], M2, tried, tr, &best));
                    c->steps++;
                    if (best == 0) break;
                    const int64_t b = sw_fill_job(best);
                    tried[tr] = b;
                    int32_t wb;
                    SWC_RUN(swc_width(c, b, &wb));
                    if (rs[2] + wb > (int64_t)c->G * c->T) continue;
                    SWC_RUN(o->copy(o->ctx, SW_A_N, SW_A_NFIN));
                    SWC_RUN(o->tail_apply(o->ctx, b));
                    SWC_RUN(o->pack(o->ctx, 4, SW_A_N, 0.0, SW_Y_CUR, SW_A_PL));
                    c->steps++;
                    int pok = 0;
                    SWC_RUN(swc_pattern(c, SW_A_N, SW_Y_CUR, SW_A_PL, &pok));
                    if (!pok) continue;
                    int64_t dfc;
                    SWC_RUN(o->eval(o->ctx, SW_EV_PACKED, SW_A_PL, c->lanesA, c->lanesB, &gm, &dfc));
                    c->steps++;
                    if (sw_shard_tree(c->lanesA) - c->k * gm > J) {
                        SWC_RUN(o->copy(o->ctx, SW_A_NFIN, SW_A_PL));
                        SWC_RUN(o->copy_y(o->ctx, SW_Y_BEST, SW_Y_CUR));
                        took = 1;
                    }
                }
                if (!took) break;
                dens_best = 0;
                rep_best = 0;
                dskip_best = 0;
            }
        }
        /* P2: priority placement of the best packed counts (shockwave.py:281-328);
         * (a) density order, (b) weight order, (c) class-wise inside the P1
         * profile — first that places every round (twin: the P2 block) */
        int ok2 = 0;
        int64_t bad;
        if (dens_best) { /* (a) is the P1 placement itself */
            SWC_RUN(o->copy_y(o->ctx, SW_Y_2, SW_Y_BEST));
            ok2 = 1;
            if (rep_best) status |= SW_STATUS_P2_REPAIRED;
        }
        for (int att = 0; att < 2 && !ok2; ++att) {
            if (att == 0 && dskip_best) continue;
            SWC_RUN(o->pack(o->ctx, att == 0 ? 4 : 2, SW_A_NFIN, 0.0, SW_Y_2, SW_A_PL));
            c->steps++;
            SWC_RUN(o->eval(o->ctx, SW_EV_P2OK, 0, c->lanesA, c->lanesB, &gm, &bad));
            c->steps++;
            ok2 = bad == 0;
            if (!ok2 && att == 0) { /* (a') density with its width profile repaired */
                SWC_RUN(swc_repair(c, SW_A_NFIN, SW_Y_2, SW_A_PL, SW_Y_CUR, SW_A_PL2, &ok2));
                if (ok2) {
                    SWC_RUN(o->copy_y(o->ctx, SW_Y_2, SW_Y_CUR));
                    status |= SW_STATUS_P2_REPAIRED;
                }
            }
            if (ok2 && att == 1) status |= SW_STATUS_P2_WEIGHT_ORDER;
        }
        if (!ok2) {
            int32_t caps[SW_TMAX];
            int32_t wc = 0, next_w = 0;
            int64_t md[2];
            SWC_RUN(o->class_caps(o->ctx, SW_A_NFIN, SW_Y_BEST, 0, -1, caps, &next_w, md));
            c->steps++;
            while (next_w != 0x7FFFFFFF) {
                wc = next_w;
                SWC_RUN(o->class_caps(o->ctx, SW_A_NFIN, SW_Y_BEST, wc, -1, caps, &next_w, md));
                c->steps++;
                SWC_RUN(o->pack_class(o->ctx, SW_A_NFIN, wc, caps, SW_Y_2, SW_A_PL));
                c->steps++;
            }
            SWC_RUN(o->eval(o->ctx, SW_EV_P2OK, 0, c->lanesA, c->lanesB, &gm, &bad));
            c->steps++;
            ok2 = bad == 0;
            if (ok2) status |= SW_STATUS_P2_CLASSWISE;
        }
        if (!ok2) status |= SW_STATUS_P2_FALLBACK;
        if (ok2) { /* the exchange step (twin: twin_p2x_plan) */
            int32_t nc = 0;
            SWC_RUN(o->p2x(o->ctx, SW_Y_2, SW_A_NFIN, &nc));
            c->steps++;
            if (nc > 0) status |= SW_STATUS_P2_EXCHANGED;
        }
        int64_t any;
        SWC_RUN(o->eval(o->ctx, SW_EV_FINAL, ok2 ? SW_Y_2 : SW_Y_BEST, c->lanesA, c->lanesB, &gm,
                        &any));
        c->steps++;
        if (any == 0) status |= SW_STATUS_NO_PLANNED;
        const double U = sw_shard_tree(c->lanesA);
        *p2_objective = sw_shard_tree(c->lanesB);
        *utility = U;
        *makespan = gm;
        *objective = U - k * gm;
        *bound_out = bound;
        if (sw_p1_uncertified(*objective, bound)) status |= SW_STATUS_P1_UNCERTIFIED;
        *iters = (int32_t)c->steps;
        *status_out = status;
        rc = (status & SW_STATUS_P2_FALLBACK) ? SW_FALLBACK : SW_OK;
    }
done:
#undef SWC_RUN
    free(c->w_all);
    free(c);
    return rc;
}

#endif /* SW_SHARD_CTL_H */
