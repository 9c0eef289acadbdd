/*
 * sw_kernels.hip — the MI355X (gfx950) plan-solve kernel.
 *
 * One 512-thread workgroup (8 wave64, SW_BLOCK in sw_block.h) solves one
 * instance end to end:
 *   setup     per-job constants and fp32 ranking-key rows — the fused
 *             log-utility-gradient × fairness-weight step — and A = max_j a_j
 *   P1        level search over the makespan M; at each level a price
 *             bisection over the fp32 key bits (the price of a GPU-round),
 *             a job-ordered tie group and a width tail; then packing into
 *             rounds, re-solved on a smaller budget when widths fragment
 *             the rounds                                  (shockwave.py:330-388)
 *   P2        priority placement of the planned rounds    (shockwave.py:281-328)
 *   emit      plan bytes, planned-round counts, objective  (shockwave.py:390-398)
 * The algorithm is specified by, and bit-identical to, oracle/plan_twin.c;
 * functions below name the twin function they mirror.  DESIGN.md §3
 * describes the algorithm, §4 the mapping onto CDNA4.
 *
 * Mapping.  N ≤ 1024 (every reference configuration): two jobs per thread
 * (SW_JPT), their fp32 key rows in VGPRs, per-job state in LDS, every block
 * reduction one barrier (sw_block.h).  Packing sorts the jobs with a
 * register bitonic sort (shuffles for strides < 128, LDS beyond), then the
 * whole block runs the round loop of sw_pack.h: each thread keeps its two
 * sorted positions in VGPRs, tiers and fills are block scans.
 * N > 1024 (the 10k-job C4 shape): several jobs per thread, per-job state
 * and key rows in an HBM workspace (L2-resident), sort through the
 * workspace, and wave 0 runs the round loop over workspace position state.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shockwave_amd.h"
#include "sw_arith.h"
#include "sw_block.h"
#include "sw_device.h"
#include "sw_pack.h"
#include "sw_bnb.h"
#include "sw_repair.h"
#include "sw_reround_dev.h"
#include "sw_p2x_inst.h"

namespace {

#ifdef SW_STAMPS
#define SW_STAMP(slot)                                                            \
    do {                                                                          \
        __syncthreads();                                                          \
        if (threadIdx.x == 0 && B.stamps) {                                       \
            uint64_t now_ = __builtin_amdgcn_s_memtime();                         \
            B.stamps[(size_t)inst_ * SW_STAMP_SLOTS + (slot)] += now_ - stamp_prev_;      \
            stamp_prev_ = now_;                                                   \
        }                                                                         \
    } while (0)
#else
#define SW_STAMP(slot) \
    do {               \
    } while (0)
#endif

#ifdef SW_STAMPS
/* level-search breakdown (thread 0's view), slots 16 + k: 0 force pass,
 * 1 price probes, 2 tie group, 3 width tail, 4 evaluation, 5 M_lo search,
 * 6 levels_between; 7 / 8 count price probes / M_lo passes.  Accumulated in
 * registers (lsa) and added to the slots when the search returns. */
#define LS_STAMP(k)                                            \
    do {                                                       \
        const uint64_t now_ = __builtin_amdgcn_s_memtime();    \
        lsa[k] += now_ - ls_t;                                 \
        ls_t = now_;                                           \
    } while (0)
#else
#define LS_STAMP(k) \
    do {            \
    } while (0)
#endif

struct SelEval {
    double U, Mact, J, ubound;
    uint32_t rho; /* price ρ* bits of the level (0 when every item fits) */
};

/* Workgroup-uniform values (block-reduction results and what the level
 * search derives from them) moved to SGPRs: held in VGPRs, the level
 * search's four evaluations and its bracket took ~40 VGPRs of uniform data,
 * which the 128-VGPR level kernel spilled to scratch — 2.6 GB of scratch
 * write-backs per 32768-instance launch (profiles/r6z1_summary.json). */
__device__ __forceinline__ double sw_uni(double x) { return sw_f64u(x); }
__device__ __forceinline__ uint32_t sw_uni(uint32_t x) { return (uint32_t)sw_u32((int32_t)x); }
__device__ __forceinline__ SelEval sw_uni(const SelEval& e) {
    SelEval r;
    r.U = sw_uni(e.U);
    r.Mact = sw_uni(e.Mact);
    r.J = sw_uni(e.J);
    r.ubound = sw_uni(e.ubound);
    r.rho = sw_uni(e.rho);
    return r;
}

/* packed per-position packer state: r | w << 8 | sel << 16 */
__device__ __forceinline__ uint32_t st_r(uint32_t s) { return s & 0xFFu; }
__device__ __forceinline__ uint32_t st_w(uint32_t s) { return (s >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t st_sel(uint32_t s) { return (s >> 16) & 1u; }

/* Per-job constants of the on-chip path as structure-of-arrays in LDS: a
 * thread's two jobs sit side by side, so one field of both is one 16-byte LDS
 * read, and the 34 VGPRs a register copy would pin stay free for the
 * searches and the packer. */
struct sw_job_lds {
    double *rate, *cap, *d, *R, *a, *Fd, *Ed, *invE;
    int32_t* w;
    template <class Carve>
    __device__ __forceinline__ void carve(Carve&& cv) {
        rate = (double*)cv(8 * SW_LDS_JOBS);
        cap = (double*)cv(8 * SW_LDS_JOBS);
        d = (double*)cv(8 * SW_LDS_JOBS);
        R = (double*)cv(8 * SW_LDS_JOBS);
        a = (double*)cv(8 * SW_LDS_JOBS);
        Fd = (double*)cv(8 * SW_LDS_JOBS);
        Ed = (double*)cv(8 * SW_LDS_JOBS);
        invE = (double*)cv(8 * SW_LDS_JOBS);
        w = (int32_t*)cv(4 * SW_LDS_JOBS);
    }
    __device__ __forceinline__ sw_jobc get(int j) const {
        sw_jobc c;
        c.rate = rate[j]; c.cap = cap[j]; c.d = d[j]; c.R = R[j]; c.a = a[j];
        c.Fd = Fd[j]; c.Ed = Ed[j]; c.invE = invE[j]; c.w = w[j];
        return c;
    }
    __device__ __forceinline__ void put(int j, const sw_jobc& c) const {
        rate[j] = c.rate; cap[j] = c.cap; d[j] = c.d; R[j] = c.R; a[j] = c.a;
        Fd[j] = c.Fd; Ed[j] = c.Ed; invE[j] = c.invE; w[j] = c.w;
    }
};
#define SW_JOB_LDS_BYTES (8 * 8 * SW_LDS_JOBS + 4 * SW_LDS_JOBS)

/* jobs per thread on the on-chip path (N ≤ SW_LDS_JOBS = SW_JPT · SW_BLOCK) */
#define SW_JPT 2
/* keys per job per staging chunk of the key-row setup: the level kernel's
 * staging window is SW_JPT · SW_SETUP_CH · SW_BLOCK floats (8 KB), which its
 * level search reuses for five per-job byte arrays (5 KB) */
#define SW_SETUP_CH 2

/* SMALL: the pack kernel's context — every pack has at most SW_BLOCK active
 * jobs (one position per thread), so the 1024-position paths compile out. */
template <int KT, bool ONE, bool SMALL = false>
struct Ctx {
    /* instance scalars (uniform) */
    int32_t N, T, G, nb, q;
    int64_t C;
    double k, A;
    double inv_delta; /* 1 / Δ: the slope of g(n) ≈ R − Δ·n (d·rate = Δ) */
    int64_t passes;
    double lsU, lsM; /* utility / makespan of the level search's best counts */
    const sw_inst_dev* inst;
    const double* beta; /* LDS */
    const double* ell;  /* LDS */
    const double* slope; /* LDS: segment slopes (sw_pwl_slopes) */
    sw_blk blk;
    /* inputs (instance-relative) */
    const int32_t* w_in;
    const double* p_in;
#ifdef SW_STAMPS
    uint64_t* swp; /* pack phase stamps of this instance */
    uint64_t* lsp; /* level-search stamps */
    uint64_t ls_t;
    uint64_t lsa[9];
#endif
    /* per-job state (LDS when ONE, HBM workspace otherwise) */
    uint8_t *ncur, *lcur, *tkcur, *nbest, *placed, *placed2, *nfin;
    uint8_t* tiecur; /* the take pass's tie counts, read by the tie group */
    uint64_t *ycur, *ybest, *y2;
    /* packer: transposed position state, masks, order, sort buffers */
    uint32_t* pst;
    uint64_t* pmask;
    int32_t* pord;
    uint64_t* sbuf; /* ONE: [2][2][1024] bitonic exchange; else [2][NP] keys */
    int32_t *H, *SH;
    sw_pack_lds* PL;
    /* class-wise P2 (MODE 5): the class width and its per-round capacity (LDS) */
    int32_t pwc;
    int32_t* caps;
    int64_t* misc;
    sw_repair_t* rep; /* LDS: the width profile of repair_pack */
    sw_bnb_ivl* bnb;  /* the level search's interval list (SW_BNB_CAP entries, sw_bnb.h) */
    /* this thread's jobs (ONE): slot s ↔ job jlo() + s */
    sw_job_lds JL; /* ONE: per-job constants, SoA in LDS (not VGPRs) */
    float kr[SW_JPT][KT];
    /* per-job data in HBM (!ONE) */
    float* gkeys;
    sw_jobc* gjc;

    __device__ __forceinline__ int jlo() const { return (int)threadIdx.x * q; }
    __device__ __forceinline__ int jhi() const {
        int h = jlo() + q;
        return h < N ? h : N;
    }
    /* Visit this thread's jobs in order; s is a compile-time slot on the
     * on-chip path, 0 otherwise. */
    template <class F>
    __device__ __forceinline__ void for_jobs(F&& f) const {
        if constexpr (ONE) {
#pragma unroll
            for (int s = 0; s < SW_JPT; ++s) {
                const int j = jlo() + s;
                if (s < q && j < N) f(j, s);
            }
        } else {
            for (int j = jlo(); j < jhi(); ++j) f(j, 0);
        }
    }
    __device__ __forceinline__ sw_jobc jc(int j, int s) const {
        if constexpr (ONE) {
            (void)s;
            return JL.get(j);
        } else {
            (void)s;
            return gjc[j];
        }
    }
    __device__ __forceinline__ int Tj(int j, int s) const { return jc(j, s).w <= G ? T : 0; }
    __device__ __forceinline__ double fval(int j, int s, int n) const {
        const sw_jobc c = jc(j, s);
        return sw_f(&c, n, nb, beta, ell, slope);
    }
    __device__ __forceinline__ double gval(int j, int s, int n) const {
        const sw_jobc c = jc(j, s);
        return sw_g(&c, n);
    }

    __device__ __forceinline__ uint32_t kbits(int j, int s, int n) const {
        if constexpr (ONE) {
            (void)j;
            uint32_t v = 0;
#pragma unroll
            for (int i = 0; i < KT; ++i) v = (i == n) ? sw_fbits_of(kr[s][i]) : v;
            return v;
        } else {
            (void)s;
            return sw_fbits_of(gkeys[(size_t)j * KT + n]);
        }
    }

    /* twin: lforce */
    __device__ __forceinline__ int lforce(int j, int s, double M) const {
        double gi, gb;
        return lforce_g(j, s, M, gi, gb);
    }
    /* The same count with the row values either side of it: gi = g(cnt)
     * (when cnt < Tj) and gb = g(cnt − 1) (when cnt > 0).  g is
     * nonincreasing, flat from where e(n) reaches its cap and otherwise
     * g(n) = R − d·rate·n = R − Δ·n up to rounding, so the count is guessed
     * from (R − M)/Δ and settled by an exact walk on sw_g — two or three
     * evaluations instead of a 5-step binary search plus two. */
    __device__ __forceinline__ int lforce_g(int j, int s, double M, double& gi, double& gb) const {
        const sw_jobc c = jc(j, s);
        const int tj = Tj(j, s);
        if (tj == 0) return 0;
        const double gl = sw_g(&c, tj - 1);
        if (gl > M) { /* every round is forced (the flat tail is above M) */
            gb = gl;
            return tj;
        }
        /* the answer is the smallest n < tj with g(n) ≤ M */
        const double x = (c.R - M) * inv_delta;
        int n = x <= 0.0 ? 0 : (x >= (double)(tj - 1) ? tj - 1 : (int)ceil(x));
        double gn = n == tj - 1 ? gl : sw_g(&c, n);
        if (gn > M) {
            do {
                gb = gn;
                ++n;
                gn = n == tj - 1 ? gl : sw_g(&c, n);
            } while (gn > M);
            gi = gn;
            return n;
        }
        gi = gn;
        while (n > 0) {
            const double gp = sw_g(&c, n - 1);
            if (gp > M) {
                gb = gp;
                break;
            }
            gi = gp;
            --n;
        }
        return n;
    }
    /* #{n ≤ Tj : g(n) > x} (GE: ≥ x) — the first n ∈ [0, Tj] where the
     * monotone predicate fails, found like lforce_g: guessed from the linear
     * part of g, settled by an exact walk (the binary search's answer in
     * two or three evaluations of g instead of five or six) */
    template <bool GE>
    __device__ __forceinline__ int g_cnt(int j, int s, double x) const {
        const sw_jobc c = jc(j, s);
        const int tj = Tj(j, s);
        const double gt = sw_g(&c, tj);
        if (GE ? (gt >= x) : (gt > x)) return tj + 1;
        const double xx = (c.R - x) * inv_delta;
        int n = xx <= 0.0 ? 0 : (xx >= (double)tj ? tj : (int)ceil(xx));
        double gn = n == tj ? gt : sw_g(&c, n);
        if (GE ? (gn >= x) : (gn > x)) {
            do {
                ++n;
                gn = n == tj ? gt : sw_g(&c, n);
            } while (GE ? (gn >= x) : (gn > x));
            return n;
        }
        while (n > 0) {
            const double gp = sw_g(&c, n - 1);
            if (GE ? (gp >= x) : (gp > x)) break;
            --n;
        }
        return n;
    }
    /* twin: cnt_gt / cnt_ge.  Keys are nonincreasing, so the items with
     * key > ρ (≥ ρ) form a prefix [0, c) and the count over [l, Tj) is
     * min(c, Tj) − l, clamped at 0.  On chip the register row is zero past
     * Tj, so c needs one compare per key. */
    template <bool GE>
    __device__ __forceinline__ int cnt(int j, int s, uint32_t rho, int l) const {
        const int tj = Tj(j, s);
        int c = 0;
        if constexpr (ONE) {
#pragma unroll
            for (int n = 0; n < KT; ++n) {
                const uint32_t b = sw_fbits_of(kr[s][n]);
                c += (GE ? (b >= rho) : (b > rho)) ? 1 : 0;
            }
            c = (c < tj ? c : tj) - l;
            c = c > 0 ? c : 0;
        } else {
            const float* row = gkeys + (size_t)j * KT;
            int lo = l, hi = tj;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                const uint32_t b = sw_fbits_of(row[mid]);
                if (GE ? (b >= rho) : (b > rho)) lo = mid + 1; else hi = mid;
            }
            c = lo - l;
        }
        return c;
    }

    /* cnt<false>(ρ = mid) of an open job, plus its key bits around mid:
     * mx = max(mx, largest key ≤ mid), mn = min(mn, smallest key > mid)
     * (twin: the snapped bisection of select_level).  The row is
     * nonincreasing, so the raw count c0 splits it there. */
    __device__ __forceinline__ int cnt_snap(int j, int s, uint32_t mid, int l, int32_t& mx,
                                            int32_t& mn) const {
        const int tj = Tj(j, s);
        int c = 0;
        if constexpr (ONE) {
            (void)j;
            /* the keys > mid are the prefix [0, c0): the last of them is
             * row[c0 − 1] and the key after it row[c0] (0 past the row), so
             * two selects on the compare, no min / max per key */
            uint32_t lo_k = 0x7FFFFFFFu, hi_k = sw_fbits_of(kr[s][0]);
#pragma unroll
            for (int n = 0; n < KT; ++n) {
                const uint32_t b = sw_fbits_of(kr[s][n]);
                const uint32_t nx = n + 1 < KT ? sw_fbits_of(kr[s][n + 1 < KT ? n + 1 : n]) : 0u;
                const bool gt = b > mid;
                c += gt ? 1 : 0;
                lo_k = gt ? b : lo_k;
                hi_k = gt ? nx : hi_k;
            }
            mn = min(mn, (int32_t)lo_k);
            mx = max(mx, (int32_t)hi_k);
        } else {
            (void)s;
            const float* row = gkeys + (size_t)j * KT;
            int lo = 0, hi = tj;
            while (lo < hi) {
                const int m = (lo + hi) >> 1;
                if (sw_fbits_of(row[m]) > mid) lo = m + 1; else hi = m;
            }
            c = lo;
            if (c < tj) mx = max(mx, (int32_t)sw_fbits_of(row[c]));
            if (c > 0) mn = min(mn, (int32_t)sw_fbits_of(row[c - 1]));
        }
        c = (c < tj ? c : tj) - l;
        return c > 0 ? c : 0;
    }

    /* twin: build() — constants and key rows */
    __device__ __forceinline__ void setup() {
        double amax = 0.0;
        for_jobs([&](int j, int s) { amax = sw_max(amax, jc(j, s).a); });
        A = blk.dmax(amax);
        if constexpr (ONE) {
            /* rolled evaluation into an LDS staging window (SW_SETUP_CH keys
             * × SW_JPT jobs per thread per chunk), then compile-time-indexed
             * copies */
            constexpr int CH = SW_SETUP_CH;
            float* stage = reinterpret_cast<float*>(sbuf);
            double prev[SW_JPT], vm[SW_JPT], ksc[SW_JPT];
            /* f(n) = a·φ(u(n)) evaluated incrementally: u(n) is nondecreasing
             * in n, so the PWL segment sw_phi would select only moves up;
             * each job keeps its segment's (β_b, ℓ_b, slope_b) and the next
             * breakpoint in registers and re-reads them from LDS only when u
             * crosses a breakpoint.  Same operations on the same operands as
             * sw_f, so the same bits. */
            int sb[SW_JPT];
            double sbeta[SW_JPT], sell[SW_JPT], sslope[SW_JPT], snext[SW_JPT];
            auto seg_load = [&](int s, int b) {
                sb[s] = b;
                sbeta[s] = beta[b];
                sell[s] = ell[b];
                sslope[s] = slope[b];
                snext[s] = b + 1 <= nb - 2 ? beta[b + 1] : __builtin_inf();
            };
            auto f_inc = [&](int s, const sw_jobc& cj, int n) {
                const double u = (cj.Fd + sw_e(&cj, n)) * cj.invE;
                while (snext[s] <= u) seg_load(s, sb[s] + 1);
                return cj.a * (sell[s] + sslope[s] * (u - sbeta[s]));
            };
#pragma unroll
            for (int s = 0; s < SW_JPT; ++s) {
                prev[s] = 0.0;
                vm[s] = 0.0;
                const sw_jobc c0 = jc(jlo() + s, s);
                ksc[s] = sw_key_scale(c0.w, A);
                seg_load(s, 0);
                if (s < q && jlo() + s < N) prev[s] = f_inc(s, c0, 0);
            }
#pragma unroll
            for (int ch = 0; ch < KT / CH; ++ch) {
#pragma unroll
                for (int s = 0; s < SW_JPT; ++s) {
                    const bool act = s < q && jlo() + s < N;
                    for (int i = 0; i < CH; ++i) {
                        const int n = ch * CH + i;
                        float kv = 0.0f;
                        const sw_jobc cs = jc(jlo() + s, s);
                        if (act && n < T && cs.w <= G) {
                            const double cur = f_inc(s, cs, n + 1);
                            const double v = sw_pos(cur - prev[s]);
                            vm[s] = (n == 0) ? v : sw_min(vm[s], v);
                            kv = sw_key(vm[s], ksc[s]);
                            prev[s] = cur;
                        }
                        stage[(s * CH + i) * SW_BLOCK + threadIdx.x] = kv;
                    }
                }
#pragma unroll
                for (int s = 0; s < SW_JPT; ++s)
#pragma unroll
                    for (int i = 0; i < CH; ++i)
                        kr[s][ch * CH + i] = stage[(s * CH + i) * SW_BLOCK + threadIdx.x];
            }
        } else {
            for (int j = jlo(); j < jhi(); ++j) {
                const sw_jobc& c = gjc[j];
                double prev = sw_f(&c, 0, nb, beta, ell, slope), vm = 0.0;
                float* row = gkeys + (size_t)j * KT;
                for (int n = 0; n < T; ++n) {
                    const double cur = sw_f(&c, n + 1, nb, beta, ell, slope);
                    const double v = sw_pos(cur - prev);
                    vm = (n == 0) ? v : sw_min(vm, v);
                    row[n] = sw_key(vm, sw_key_scale(c.w, A));
                    prev = cur;
                }
            }
        }
        __syncthreads();
    }

    /* twin: select_level */
    /* [plo, phi] brackets ρ*(M) from evaluated neighbour levels (twin:
     * select_level); ev.rho returns ρ* (0 when every item fits) */
    __device__ __forceinline__ SelEval select_level(double M, bool is_inf, uint32_t plo,
                                                    uint32_t phi) {
        int64_t wf = 0, wall = 0;
        for_jobs([&](int j, int s) {
            const int l = is_inf ? 0 : lforce(j, s, M);
            lcur[j] = (uint8_t)l;
            wf += (int64_t)jc(j, s).w * l;
            wall += (int64_t)jc(j, s).w * (Tj(j, s) - l);
        });
        int64_t Wf, Wall;
        blk.sum2(wf, wall, Wf, Wall);
        passes++;
        LS_STAMP(0);
        SelEval ev;
        ev.rho = 0;
        if (Wf > C) {
            ev.U = 0; ev.Mact = 0; ev.J = -1e308; ev.ubound = 0;
            return ev;
        }
        const int64_t bud = C - Wf;
        double rho_d = 0.0;
        int64_t wgt_star;
        if (Wall <= bud) {
            for_jobs([&](int j, int s) {
                ncur[j] = (uint8_t)Tj(j, s);
                tkcur[j] = (uint8_t)(Tj(j, s) - lcur[j]);
            });
            wgt_star = Wall;
        } else {
            uint32_t lo = plo, hi = phi;
            if constexpr (ONE) {
                /* Per-job windows: ca = #keys ≥ lo (= count above lo − 1),
                 * cb = #keys > hi.  Every probe mid ∈ [lo, hi) counts
                 * between them, so a job whose window is closed (ca == cb)
                 * skips its 32 compares; as the bracket narrows, whole
                 * waves skip.  Same probes, same ρ*. */
                int ca[SW_JPT], cb[SW_JPT], cm[SW_JPT];
#pragma unroll
                for (int s = 0; s < SW_JPT; ++s) { ca[s] = 0; cb[s] = 0; cm[s] = 0; }
                if (lo < hi)
                    for_jobs([&](int j, int s) {
                        ca[s] = cnt<true>(j, s, lo, lcur[j]);
                        cb[s] = cnt<false>(j, s, hi, lcur[j]);
                    });
                /* Snapped to key values (twin: select_level): the open
                 * jobs also report the keys either side of mid, W is
                 * constant between them, and the bracket jumps there.
                 * ca / cb stay exact: no open job has a key strictly
                 * between the snapped end and mid. */
                int64_t Wb = -1, Wh = -1; /* twin: interpolated probes */
                while (lo < hi) {
                    uint32_t mid = lo + ((hi - lo) >> 1);
                    if (Wb >= 0 && Wh >= 0) {
                        mid = lo + (uint32_t)(((uint64_t)(hi - lo) * (uint64_t)(Wb - bud)) /
                                              (uint64_t)(Wb - Wh));
                        if (mid >= hi) mid = hi - 1;
                    }
                    int32_t wg = 0, mx = 0, mn = 0x7FFFFFFF;
                    for_jobs([&](int j, int s) {
                        int c = cb[s];
                        if (ca[s] != cb[s]) c = cnt_snap(j, s, mid, lcur[j], mx, mn);
                        cm[s] = c;
                        wg += jc(j, s).w * c;
                    });
                    int32_t MX, MN;
                    wg = blk.sum32_max_min(wg, mx, mn, MX, MN);
                    passes++;
#ifdef SW_STAMPS
                    lsa[7] += 1; /* price probes */
#endif
                    const bool down = wg <= bud;
#pragma unroll
                    for (int s = 0; s < SW_JPT; ++s) {
                        cb[s] = down ? cm[s] : cb[s];
                        ca[s] = down ? ca[s] : cm[s];
                    }
                    if (down) { hi = (uint32_t)MX > lo ? (uint32_t)MX : lo; Wh = wg; }
                    else { lo = (uint32_t)MN < hi ? (uint32_t)MN : hi; Wb = wg; }
                }
            } else {
                int64_t Wb = -1, Wh = -1;
                while (lo < hi) {
                    uint32_t mid = lo + ((hi - lo) >> 1);
                    if (Wb >= 0 && Wh >= 0) {
                        mid = lo + (uint32_t)(((uint64_t)(hi - lo) * (uint64_t)(Wb - bud)) /
                                              (uint64_t)(Wb - Wh));
                        if (mid >= hi) mid = hi - 1;
                    }
                    int32_t wg = 0, mx = 0, mn = 0x7FFFFFFF;
                    for_jobs([&](int j, int s) {
                        const int l = lcur[j];
                        if (cnt<true>(j, s, lo, l) != cnt<false>(j, s, hi, l))
                            wg += jc(j, s).w * cnt_snap(j, s, mid, l, mx, mn);
                        else
                            wg += jc(j, s).w * cnt<false>(j, s, mid, l);
                    });
                    int32_t MX, MN;
                    wg = blk.sum32_max_min(wg, mx, mn, MX, MN);
                    passes++;
                    if (wg <= bud) { hi = (uint32_t)MX > lo ? (uint32_t)MX : lo; Wh = wg; }
                    else { lo = (uint32_t)MN < hi ? (uint32_t)MN : hi; Wb = wg; }
                }
            }
            LS_STAMP(1);
            const uint32_t rho = lo;
            ev.rho = rho;
            rho_d = (double)sw_float_of(rho);
            int64_t wt_l = 0;
            int32_t tie_l = 0;
            for_jobs([&](int j, int s) {
                const int tk = cnt<false>(j, s, rho, lcur[j]);
                const int tie = cnt<true>(j, s, rho, lcur[j]) - tk;
                tkcur[j] = (uint8_t)tk;
                tiecur[j] = (uint8_t)tie;
                wt_l += (int64_t)jc(j, s).w * tk;
                tie_l += jc(j, s).w * tie;
            });
            const int64_t wt = blk.sum(wt_l);
            wgt_star = wt;
            const int64_t rem = bud - wt;
            int32_t tot;
            int64_t excl = blk.exscan(tie_l, tot);
            int64_t used_l = 0;
            for_jobs([&](int j, int s) {
                const int tk = tkcur[j];
                const int tie = tiecur[j];
                const int64_t wj = jc(j, s).w;
                int tt;
                if (excl + wj * tie <= rem) tt = tie;
                else if (excl <= rem) tt = (int)((rem - excl) / wj);
                else tt = 0;
                ncur[j] = (uint8_t)(lcur[j] + tk + tt);
                used_l += wj * tt;
                excl += wj * tie;
            });
            const int64_t used = blk.sum(used_l);
            passes++;
            LS_STAMP(2);
            int64_t rem2 = rem - used;
            while (rem2 > 0) {
                uint64_t best = 0;
                for_jobs([&](int j, int s) {
                    const int nj = ncur[j];
                    if (nj < Tj(j, s) && (int64_t)jc(j, s).w <= rem2) {
                        const uint64_t key = ((uint64_t)kbits(j, s, nj) << 32) |
                                             (uint64_t)(0xFFFFFFFFu - (uint32_t)j);
                        best = key > best ? key : best;
                    }
                });
                best = blk.umax(best);
                passes++;
                if (best == 0) break;
                const int jb = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu));
                if (jb >= jlo() && jb < jhi()) ncur[jb] = (uint8_t)(ncur[jb] + 1);
                rem2 -= w_in[jb];
            }
            LS_STAMP(3);
        }
        double fs = 0.0, gm = 0.0, ub = 0.0;
        for_jobs([&](int j, int s) {
            /* the bound's count l + taken equals n for every job outside the
             * tie group and the width tail: one f evaluation serves both */
            const int nj = ncur[j], lt = lcur[j] + tkcur[j];
            const double fn = fval(j, s, nj);
            fs = fs + fn;
            gm = sw_max(gm, gval(j, s, nj));
            ub = ub + (lt == nj ? fn : fval(j, s, lt));
        });
        blk.detsum_max(fs, gm, ev.U, ev.Mact);
        ev.J = ev.U - k * ev.Mact;
        ev.ubound = blk.detsum(ub) + (rho_d * A) * (double)(bud - wgt_star);
        passes++;
        LS_STAMP(4);
        return ev;
    }

    __device__ __forceinline__ void keep_best(const SelEval& e, SelEval& best) {
        if (e.J > best.J || (e.J == best.J && e.Mact < best.Mact)) {
            best = e;
            for_jobs([&](int j, int s) { (void)s; nbest[j] = ncur[j]; });
        }
    }

    /* twin: feasible_level */
    __device__ __forceinline__ bool feasible_level(double M) {
        int64_t wf = 0;
        for_jobs([&](int j, int s) { wf += (int64_t)jc(j, s).w * lforce(j, s, M); });
        wf = blk.sum(wf);
        passes++;
        return wf <= C;
    }

    /* twin: levels_between — #{(j, n ≤ Tj) : a < g_j(n) < b} */
    __device__ __forceinline__ int64_t levels_between(double a, double b) {
        int64_t c = 0;
        for_jobs([&](int j, int s) {
            const int d = g_cnt<false>(j, s, a) - g_cnt<true>(j, s, b);
            c += d > 0 ? d : 0;
        });
        c = blk.sum(c);
        passes++;
        LS_STAMP(6);
        return c;
    }

    /* twin: level_search — best counts land in nbest; returns the bound.
     * Written as a loop over evaluation requests so select_level has a
     * single call site (phase 1: M = M_lo; 0: M = +inf; 2: a branch-and-
     * bound probe at the midpoint of the interval of largest bound). */
    __device__ __forceinline__ double level_search() {
#ifdef SW_STAMPS
        ls_t = __builtin_amdgcn_s_memtime();
        for (int k = 0; k < 9; ++k) lsa[k] = 0;
#endif
        SelEval best, elo;
        best.U = best.Mact = best.ubound = 0.0;
        best.J = -1e308;
        best.rho = 0;
        elo = best;
        double M_lo = 0.0, ret = 0.0;
        uint32_t plo = 0, phi = SW_KEY_INF_BITS;
        const bool levels = N > 0 && k > 0.0;
        if (levels) {
            /* twin: the M_lo search on [lb, top] that snaps to row values */
            double lb = 0.0, top = 0.0;
            for_jobs([&](int j, int s) {
                lb = sw_max(lb, gval(j, s, Tj(j, s)));
                top = sw_max(top, gval(j, s, 0));
            });
            lb = blk.dmax(lb);
            top = blk.dmax(top);
            uint64_t lo = sw_bits(lb), hi = sw_bits(top);
            int64_t Fb = -1, Fh = -1; /* twin: interpolated probes */
            while (lo < hi) {
                double x = (sw_from_bits(lo) + sw_from_bits(hi)) * 0.5;
                if (Fb >= 0 && Fh >= 0)
                    x = sw_from_bits(lo) + (sw_from_bits(hi) - sw_from_bits(lo)) *
                                               ((double)(Fb - C) / (double)(Fb - Fh));
                if (sw_bits(x) >= hi) x = sw_from_bits(hi - 1);
                if (sw_bits(x) < lo) x = sw_from_bits(lo);
                int64_t f = 0;
                uint64_t bmx = 0, bmn = ~0ull;
                for_jobs([&](int j, int s) {
                    double gi = 0.0, gb = 0.0;
                    const int cn = lforce_g(j, s, x, gi, gb);
                    f += (int64_t)jc(j, s).w * cn;
                    if (cn < Tj(j, s)) {
                        const uint64_t bb = sw_bits(gi);
                        bmx = bb > bmx ? bb : bmx;
                    }
                    if (cn > 0) {
                        const uint64_t bb = sw_bits(gb);
                        bmn = bb < bmn ? bb : bmn;
                    }
                });
                int64_t F;
                uint64_t BMX, BMN;
                blk.sum_max_min(f, bmx, bmn, F, BMX, BMN);
                passes++;
#ifdef SW_STAMPS
                lsa[8] += 1; /* M_lo passes */
#endif
                if (F <= C) { hi = BMX >= lo ? BMX : lo; Fh = F; }
                else { lo = BMN <= hi ? BMN : hi; Fb = F; }
            }
            M_lo = sw_uni(sw_from_bits(lo));
            LS_STAMP(5);
        }
        int phase = levels ? 1 : 0;
        /* branch and bound over the levels in (M_lo, M_free] (twin:
         * level_search; sw_bnb.h): the interval list lives in bnb, written
         * by thread 0 between barriers; every thread picks from it alike */
        int32_t nL = 0, probes = 0;
        double cert = 0.0, m = 0.0;
        double Ia = 0.0, Ib = 0.0, Ivb = 0.0;
        uint32_t Ira = 0, Irb = 0;
        while (true) {
            double M = 0.0;
            if (phase == 1) M = M_lo;
            else if (phase == 2) M = m;
            const SelEval ev = sw_uni(select_level(M, phase == 0, plo, phi));
            if (phase == 1) {
                best = ev;
                elo = ev;
                for_jobs([&](int j, int s) { (void)s; nbest[j] = ncur[j]; });
                /* twin: can a higher level win?  Only below
                 * M_lo + (U_max − U(M_lo))/k, U_max = Σ_j f_j(T_j) */
                double um = 0.0;
                for_jobs([&](int j, int s) { um = um + fval(j, s, Tj(j, s)); });
                const double U_max = blk.detsum(um);
                passes++;
                const double wmax = sw_uni((U_max - ev.U) / k);
                ret = sw_uni(ev.ubound - k * M_lo);
                if (!(wmax > 0.0)) break;
                if (levels_between(M_lo, M_lo + wmax) == 0) break;
                plo = 0;
                phi = ev.rho; /* ρ*(+∞) ≤ ρ*(M_lo) */
                phase = 0;
                continue;
            }
            if (phase == 0) {
                if (!levels) { /* no makespan term: the utility optimum */
                    best = ev;
                    for_jobs([&](int j, int s) { (void)s; nbest[j] = ncur[j]; });
                    ret = sw_uni(ev.ubound - k * ev.Mact);
                    break;
                }
                keep_best(ev, best);
                cert = sw_uni(sw_max(elo.ubound - k * M_lo, ev.ubound - k * ev.Mact));
                if (M_lo < ev.Mact) {
                    if (threadIdx.x == 0) bnb[0] = sw_bnb_make(M_lo, ev.Mact, ev.ubound, elo.rho, ev.rho);
                    nL = 1;
                }
            } else { /* a probe at the midpoint m of the interval I */
                keep_best(ev, best);
                ++probes;
                const bool pl = sw_bnb_key(ev.ubound, k, Ia) > best.J;
                const bool pr = sw_bnb_key(Ivb, k, m) > best.J;
                if (threadIdx.x == 0) {
                    int32_t n2 = nL;
                    if (pl) bnb[n2++] = sw_bnb_make(Ia, m, ev.ubound, Ira, ev.rho);
                    if (pr) bnb[n2++] = sw_bnb_make(m, Ib, Ivb, ev.rho, Irb);
                }
                nL += (pl ? 1 : 0) + (pr ? 1 : 0);
            }
            /* the next interval worth a probe */
            bool more = false;
            while (nL > 0) {
                __syncthreads(); /* thread 0's list writes are visible */
                double kb;
                const int32_t i = sw_u32(sw_bnb_pick(bnb, nL, k, &kb));
                kb = sw_uni(kb);
                if (kb <= best.J) break; /* nothing left can beat the best plan */
                if (probes == SW_BNB_PROBES) {
                    cert = sw_uni(sw_max(cert, kb));
                    break;
                }
                Ia = sw_uni(bnb[i].a);
                Ib = sw_uni(bnb[i].b);
                Ivb = sw_uni(bnb[i].vb);
                Ira = sw_uni(bnb[i].ra);
                Irb = sw_uni(bnb[i].rb);
                __syncthreads(); /* every thread has read the list */
                if (threadIdx.x == 0) bnb[i] = bnb[nL - 1];
                --nL;
                if (levels_between(Ia, Ib) == 0) { /* only b itself, if b is a level */
                    cert = sw_uni(sw_max(cert, Ivb - k * Ib));
                    continue;
                }
                m = sw_uni(sw_bnb_mid(Ia, Ib));
                plo = Irb;
                phi = Ira;
                more = true;
                break;
            }
            if (!more) {
                ret = sw_uni(sw_max(cert, best.J));
                break;
            }
            phase = 2;
        }
        lsU = best.U;
        lsM = best.Mact;
#ifdef SW_STAMPS
        if (threadIdx.x == 0 && lsp)
            for (int k = 0; k < 9; ++k) lsp[k] += lsa[k];
#endif
        __syncthreads();
        return ret;
    }

    /* ---- packing ---------------------------------------------------------- */

    /* position p (of A, PPL per lane of wave 0) → transposed slot */
    __device__ __forceinline__ int tslot(int p, int PPL) const { return (p % PPL) * 64 + p / PPL; }

    /* Sort (hi, lo) descending.  ONE: register bitonic over E·SW_BLOCK =
     * 1024 elements, E per thread (element e = E·tid + s).  Strides < E
     * compare inside the thread, strides E … 32·E pair threads of one wave
     * (shuffles), larger strides go through a double-buffered LDS exchange
     * (one barrier per stage).  After the sort thread t holds positions
     * E·t … E·t + E − 1. */
    __device__ __forceinline__ void sort_regs(uint64_t (&hi)[SW_JPT], uint64_t (&lo)[SW_JPT]) {
        constexpr int E = SW_JPT;
        constexpr int NE = E * SW_BLOCK;
        const int tid = threadIdx.x;
        int buf = 0;
        for (int kk = 2; kk <= NE; kk <<= 1) {
            for (int jj = kk >> 1; jj > 0; jj >>= 1) {
                if (jj < E) {
#pragma unroll
                    for (int s = 0; s < E; ++s) {
                        if ((s & jj) == 0) {
                            const int t2 = s | jj;
                            const bool up = ((E * tid + s) & kk) == 0;
                            const bool gt = (hi[s] > hi[t2]) || (hi[s] == hi[t2] && lo[s] > lo[t2]);
                            if (up ? !gt : gt) {
                                const uint64_t th = hi[s], tl = lo[s];
                                hi[s] = hi[t2]; lo[s] = lo[t2]; hi[t2] = th; lo[t2] = tl;
                            }
                        }
                    }
                    continue;
                }
                uint64_t ph[E], pl[E];
                const int tj = jj / E;
                if (tj >= 64) {
                    uint64_t* xh = sbuf + (size_t)buf * 2 * NE;
                    uint64_t* xl = xh + NE;
#pragma unroll
                    for (int s = 0; s < E; ++s) { xh[E * tid + s] = hi[s]; xl[E * tid + s] = lo[s]; }
                    __syncthreads();
#pragma unroll
                    for (int s = 0; s < E; ++s) {
                        ph[s] = xh[(E * tid + s) ^ jj];
                        pl[s] = xl[(E * tid + s) ^ jj];
                    }
                    buf ^= 1;
                } else {
#pragma unroll
                    for (int s = 0; s < E; ++s) {
                        ph[s] = __shfl_xor(hi[s], tj, 64);
                        pl[s] = __shfl_xor(lo[s], tj, 64);
                    }
                }
#pragma unroll
                for (int s = 0; s < E; ++s) {
                    const int e = E * tid + s;
                    const bool up = (e & kk) == 0;
                    const bool lower = (e & jj) == 0;
                    const bool mine_gt = (hi[s] > ph[s]) || (hi[s] == ph[s] && lo[s] > pl[s]);
                    const bool keep_max = (lower == up);
                    if (keep_max ? !mine_gt : mine_gt) { hi[s] = ph[s]; lo[s] = pl[s]; }
                }
            }
        }
    }

    /* sort_regs for one 64-bit key per element (the ratio orders of pack
     * modes 2 / 4 / 5: sw_ratio_key << 11 | (2047 − job)): the same network,
     * half the data through the shuffles and the LDS exchange. */
    __device__ __forceinline__ void sort_regs64(uint64_t (&k)[SW_JPT]) {
        constexpr int E = SW_JPT;
        constexpr int NE = E * SW_BLOCK;
        const int tid = threadIdx.x;
        int buf = 0;
        for (int kk = 2; kk <= NE; kk <<= 1) {
            for (int jj = kk >> 1; jj > 0; jj >>= 1) {
                if (jj < E) {
#pragma unroll
                    for (int s = 0; s < E; ++s) {
                        if ((s & jj) == 0) {
                            const int t2 = s | jj;
                            const bool up = ((E * tid + s) & kk) == 0;
                            const bool gt = k[s] > k[t2];
                            if (up ? !gt : gt) {
                                const uint64_t tk = k[s];
                                k[s] = k[t2];
                                k[t2] = tk;
                            }
                        }
                    }
                    continue;
                }
                uint64_t pk[E];
                const int tj = jj / E;
                if (tj >= 64) {
                    uint64_t* xk = sbuf + (size_t)buf * NE;
#pragma unroll
                    for (int s = 0; s < E; ++s) xk[E * tid + s] = k[s];
                    __syncthreads();
#pragma unroll
                    for (int s = 0; s < E; ++s) pk[s] = xk[(E * tid + s) ^ jj];
                    buf ^= 1;
                } else {
#pragma unroll
                    for (int s = 0; s < E; ++s) pk[s] = __shfl_xor(k[s], tj, 64);
                }
#pragma unroll
                for (int s = 0; s < E; ++s) {
                    const int e = E * tid + s;
                    const bool up = (e & kk) == 0;
                    const bool lower = (e & jj) == 0;
                    const bool mine_gt = k[s] > pk[s];
                    const bool keep_max = (lower == up);
                    if (keep_max ? !mine_gt : mine_gt) k[s] = pk[s];
                }
            }
        }
    }

    /* Descending bitonic sort of SW_BLOCK keys, one per thread (the compacted
     * active jobs of a pack, pack()): strides < 64 pair lanes of one wave
     * (shuffles), larger ones go through a double-buffered LDS exchange at
     * x (4·SW_BLOCK words).  TWO: (hi, lo) pairs; else hi alone. */
    template <bool TWO>
    __device__ __forceinline__ void sort_one(uint64_t& hi, uint64_t& lo, uint64_t* x) {
        const int e = (int)threadIdx.x;
        int buf = 0;
        for (int kk = 2; kk <= SW_BLOCK; kk <<= 1) {
            for (int jj = kk >> 1; jj > 0; jj >>= 1) {
                uint64_t ph, pl = 0;
                if (jj >= 64) {
                    uint64_t* xh = x + (size_t)buf * (TWO ? 2 : 1) * SW_BLOCK;
                    uint64_t* xl = xh + SW_BLOCK;
                    xh[e] = hi;
                    if (TWO) xl[e] = lo;
                    __syncthreads();
                    ph = xh[e ^ jj];
                    if (TWO) pl = xl[e ^ jj];
                    buf ^= 1;
                } else {
                    ph = __shfl_xor(hi, jj, 64);
                    if (TWO) pl = __shfl_xor(lo, jj, 64);
                }
                const bool up = (e & kk) == 0;
                const bool lower = (e & jj) == 0;
                const bool mine_gt = TWO ? (hi > ph) || (hi == ph && lo > pl) : hi > ph;
                if ((lower == up) ? !mine_gt : mine_gt) {
                    hi = ph;
                    if (TWO) lo = pl;
                }
            }
        }
    }

    /* Sort in the HBM workspace (!ONE): bitonic over NP entries. */
    __device__ __forceinline__ void sort_global(int NP) {
        uint64_t* shi = sbuf;
        uint64_t* slo = sbuf + NP;
        for (int kk = 2; kk <= NP; kk <<= 1) {
            for (int jj = kk >> 1; jj > 0; jj >>= 1) {
                for (int i = threadIdx.x; i < NP; i += SW_BLOCK) {
                    const int ixj = i ^ jj;
                    if (ixj > i) {
                        const uint64_t ah = shi[i], al = slo[i], bh = shi[ixj], bl = slo[ixj];
                        const bool a_gt = (ah > bh) || (ah == bh && al > bl);
                        const bool up = (i & kk) == 0;
                        if (up ? !a_gt : a_gt) {
                            shi[i] = bh; slo[i] = bl; shi[ixj] = ah; slo[ixj] = al;
                        }
                    }
                }
                __syncthreads();
            }
        }
    }

    /* Order key of job j for pack<MODE> (twin: the k1/k2 of each caller). */
    /* rounds job j brings to pack<MODE>: MODE 5 keeps only the class pwc */
    __device__ __forceinline__ int nin_of(int MODE, const uint8_t* nin, int j) const {
        return (MODE == 5 && w_in[j] != pwc) ? 0 : (int)nin[j];
    }
    /* does pack<MODE> own job j's row (MODE 5: only its class) */
    __device__ __forceinline__ bool owns(int MODE, const uint8_t* nin, int j) const {
        return MODE != 5 || (w_in[j] == pwc && nin[j] > 0);
    }

    /* Order key of job j for pack<MODE> (twin: the k1/k2 of each caller). */
    __device__ __forceinline__ void key_of(int MODE, const uint8_t* nin, double Mb, int j, int s,
                                           uint64_t& khi, uint64_t& klo) const {
        const int nj = nin_of(MODE, nin, j);
        khi = 0;
        klo = 0;
        if (nj > 0) {
            uint64_t k1;
            uint32_t k2;
            if (MODE == 4) {
                k1 = sw_ratio_key(p_in[j] / (double)(nj * w_in[j]));
                k2 = 0;
            } else if (MODE != 2 && MODE != 5) {
                const double lvl = gval(j, s, nj - 1);
                const bool crit = k > 0.0 && lvl > Mb;
                k1 = crit ? (SW_CRIT_BIT | sw_bits(lvl)) : (MODE == 3 ? (uint64_t)jc(j, s).w : 0);
                k2 = kbits(j, s, nj - 1);
            } else {
                k1 = sw_ratio_key(p_in[j] / (double)nj);
                k2 = 0;
            }
            khi = k1;
            klo = ((uint64_t)k2 << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)j);
        }
    }

    /*
     * twin: pack — place nin[j] rounds per job into T rounds of capacity G.
     * MODE 1 / 3: P1 packing orders A / B; MODE 2: P2 weight order p_j/n_j;
     * MODE 4: P2 density order p_j/(n_j·w_j); MODE 5: class-wise P2 — the jobs
     * of width pwc with unit widths inside the per-round capacities caps[t],
     * every other job's row and count untouched.
     * Writes y[job] (round bitmask) and placed_out[job].
     */
    __device__ __forceinline__ void pack(int MODE, const uint8_t* nin, uint64_t* y,
                                         uint8_t* placed_out) {
        __syncthreads();
#ifdef SW_STAMPS
        /* pack sub-phases, thread 0's view: swp[40] keys and offsets, [41]
         * compaction after the sort, [42] the round loop with its staging,
         * [43] the row write-back (swp = stamps + 8: slots 48…51) */
        uint64_t pk0_ = __builtin_amdgcn_s_memtime();
#define PK_STAMP(k)                                                      \
    do {                                                                 \
        const uint64_t n_ = __builtin_amdgcn_s_memtime();                \
        if (threadIdx.x == 0 && swp) swp[40 + (k)] += n_ - pk0_;         \
        pk0_ = n_;                                                       \
    } while (0)
#else
#define PK_STAMP(k) \
    do {            \
    } while (0)
#endif
        double Mb = 0.0;
        const int32_t* capsp = MODE == 5 ? caps : nullptr;
        if (MODE == 1 || MODE == 3) {
            for_jobs([&](int j, int s) { Mb = sw_max(Mb, gval(j, s, nin[j])); });
            Mb = blk.dmax(Mb);
        }
        int64_t act_l = 0;
        if constexpr (ONE) {
            constexpr int E = SW_JPT;
            uint64_t khi[E], klo[E];
#pragma unroll
            for (int s = 0; s < E; ++s) { khi[s] = 0; klo[s] = 0; }
            for_jobs([&](int j, int s) {
                key_of(MODE, nin, Mb, j, s, khi[s], klo[s]);
                act_l += nin_of(MODE, nin, j) > 0;
                if (owns(MODE, nin, j)) y[j] = 0;
            });
            /* the active jobs' slots in job order (klo ≠ 0 exactly when the
             * job brings rounds); the total is A */
            int32_t A32;
            const int32_t abase = blk.exscan((int32_t)act_l, A32);
            const int A_ = A32;
            PK_STAMP(0);
#ifdef SW_STAMPS
            const uint64_t srt0_ = __builtin_amdgcn_s_memtime();
#endif
            /* the ratio orders (modes 2, 4, 5: k2 = 0) sort one 64-bit word
             * per job, key << 11 | (2047 − job) (N ≤ SW_LDS_JOBS), exactly
             * the order (k1 desc, job asc); the P1 orders 1 / 3 sort (k1, k2,
             * job) as two words */
            const bool ratio = MODE == 2 || MODE == 4 || MODE == 5;
            if (ratio) {
#pragma unroll
                for (int s = 0; s < E; ++s)
                    khi[s] = khi[s] != 0 || klo[s] != 0
                                 ? (khi[s] << 11) | (uint64_t)(2047u - (0xFFFFFFFFu - (uint32_t)klo[s]))
                                 : 0ull;
            }
            if (SMALL || A_ <= SW_BLOCK) {
                /* at most one position per thread (a C3 instance places ~1/3
                 * of its jobs): compact the active keys through LDS, sort
                 * SW_BLOCK of them one per thread (half the network of the
                 * 1024-slot sort), and thread t owns position t, so every pass
                 * of the round loop walks one position instead of E */
                /* the pack kernel (SMALL) sorts ratio orders only (modes 4
                 * and 5): one word per position, and its LDS holds
                 * 3·SW_BLOCK words here (four instances per CU) */
                uint64_t* xh = sbuf;
                uint64_t* xl = sbuf + SW_BLOCK;
                int b = abase;
#pragma unroll
                for (int s = 0; s < E; ++s)
                    if (klo[s] != 0) {
                        xh[b] = khi[s];
                        if constexpr (!SMALL) xl[b] = klo[s];
                        ++b;
                    }
                __syncthreads();
                const bool mine = (int)threadIdx.x < A_;
                uint64_t h1 = mine ? xh[threadIdx.x] : 0ull;
                uint64_t l1 = 0ull;
                if constexpr (SMALL) {
                    sort_one<false>(h1, l1, sbuf + SW_BLOCK);
                } else {
                    l1 = mine ? xl[threadIdx.x] : 0ull;
                    if (ratio) sort_one<false>(h1, l1, sbuf + 2 * SW_BLOCK);
                    else sort_one<true>(h1, l1, sbuf + 2 * SW_BLOCK);
                }
#ifdef SW_STAMPS
                if (threadIdx.x == 0 && swp) swp[7] += __builtin_amdgcn_s_memtime() - srt0_;
                pk0_ = __builtin_amdgcn_s_memtime();
#endif
                const int jp1 = !mine ? 0
                                : ratio ? (int)(2047u - (uint32_t)(h1 & 2047u))
                                        : (int)(0xFFFFFFFFu - (uint32_t)(l1 & 0xFFFFFFFFu));
                const uint32_t wq = MODE == 5 ? 1u : (uint32_t)w_in[jp1];
                uint32_t st1[1] = {mine ? ((uint32_t)nin[jp1] | (wq << 8)) : 0u};
                uint64_t mk1[1] = {0ull};
                PK_STAMP(1);
                /* the round loop in wave 0 (sw_pack_rounds_one; the sort is
                 * done with sbuf, whose first 6 KB stage the states): the
                 * pack kernel sizes it by A, the plan kernel takes the 6-
                 * or 8-position form (its register file has no room for
                 * four copies) */
#ifdef SW_STAMPS
                sw_pack_rounds_one<SMALL>(PL, A_, T, G, st1[0], mk1[0], sbuf, capsp, swp);
#else
                sw_pack_rounds_one<SMALL>(PL, A_, T, G, st1[0], mk1[0], sbuf, capsp);
#endif
                PK_STAMP(2);
                for_jobs([&](int j, int s) {
                    (void)s;
                    if (owns(MODE, nin, j)) placed_out[j] = 0;
                });
                __syncthreads();
                if (mine) {
                    y[jp1] = mk1[0];
                    placed_out[jp1] = (uint8_t)(nin[jp1] - st_r(st1[0]));
                }
                __syncthreads();
                PK_STAMP(3);
            } else {
                if constexpr (!SMALL) {
                if (ratio) sort_regs64(khi);
                else sort_regs(khi, klo);
#ifdef SW_STAMPS
                if (threadIdx.x == 0 && swp) swp[7] += __builtin_amdgcn_s_memtime() - srt0_;
#endif
                uint32_t st[E];
                uint64_t mk[E];
                int jp[E];
#pragma unroll
                for (int s = 0; s < E; ++s) {
                    const int p = E * (int)threadIdx.x + s;
                    mk[s] = 0;
                    jp[s] = ratio ? (int)(2047u - (uint32_t)(khi[s] & 2047u))
                                  : (int)(0xFFFFFFFFu - (uint32_t)(klo[s] & 0xFFFFFFFFu));
                    const uint32_t wq = MODE == 5 ? 1u : (uint32_t)w_in[jp[s]];
                    st[s] = (p < A_) ? ((uint32_t)nin[jp[s]] | (wq << 8)) : 0u;
                }
#ifdef SW_STAMPS
                sw_pack_rounds<SW_JPT>(blk, PL, A_, T, G, st, mk, capsp, swp);
#else
                sw_pack_rounds<SW_JPT>(blk, PL, A_, T, G, st, mk, capsp);
#endif
                for_jobs([&](int j, int s) {
                    (void)s;
                    if (owns(MODE, nin, j)) placed_out[j] = 0;
                });
                __syncthreads();
#pragma unroll
                for (int s = 0; s < E; ++s) {
                    const int p = E * (int)threadIdx.x + s;
                    if (p < A_) {
                        y[jp[s]] = mk[s];
                        placed_out[jp[s]] = (uint8_t)(nin[jp[s]] - st_r(st[s]));
                    }
                }
                __syncthreads();
                            }
            }
        } else {
            int NPg = 1;
            while (NPg < N) NPg <<= 1;
            uint64_t* shi = sbuf;
            uint64_t* slo = sbuf + NPg;
            for (int i = threadIdx.x; i < NPg; i += SW_BLOCK) { shi[i] = 0; slo[i] = 0; }
            __syncthreads();
            for (int j = jlo(); j < jhi(); ++j) {
                uint64_t khi, klo;
                key_of(MODE, nin, Mb, j, 0, khi, klo);
                shi[j] = khi;
                slo[j] = klo;
                act_l += nin_of(MODE, nin, j) > 0;
                if (owns(MODE, nin, j)) y[j] = 0;
            }
            const int A_ = (int)blk.sum(act_l);
            sort_global(NPg);
            const int PPL = (A_ + 63) / 64;
            for (int p = threadIdx.x; p < A_; p += SW_BLOCK) {
                const int j = (int)(0xFFFFFFFFu - (uint32_t)(slo[p] & 0xFFFFFFFFu));
                const int s = tslot(p, PPL);
                pord[s] = j;
                pst[s] = (uint32_t)nin[j] | ((MODE == 5 ? 1u : (uint32_t)w_in[j]) << 8);
                pmask[s] = 0;
            }
            __syncthreads();
            if (wave_id() == 0) rounds(A_, PPL, capsp);
            __syncthreads();
            for (int j = jlo(); j < jhi(); ++j)
                if (owns(MODE, nin, j)) placed_out[j] = 0;
            __syncthreads();
            for (int p = threadIdx.x; p < A_; p += SW_BLOCK) {
                const int s = tslot(p, PPL);
                const int j = pord[s];
                y[j] = pmask[s];
                placed_out[j] = (uint8_t)(nin[j] - st_r(pst[s]));
            }
            __syncthreads();
        }
#undef PK_STAMP
    }

    /*
     * twin: repair_pack — yd / pd are the density-order pack of nin that left
     * rounds unplaced.  The width classes' profile and the free GPUs per
     * round are gathered from it (LDS atomics), one thread repairs the
     * profile (sw_repair.h), and every changed class is repacked alone
     * (pack mode 5, unit widths, order p_j/n_j) inside its new capacities
     * into yout / pout; unchanged classes keep their density rows.  True
     * when every round of nin is placed.
     */
    __device__ __forceinline__ bool repair_pack(const uint8_t* nin, const uint64_t* yd,
                                                const uint8_t* pd, uint64_t* yout, uint8_t* pout) {
        sw_repair_t* R = rep;
        uint32_t* wset = reinterpret_cast<uint32_t*>(misc); /* widths present: 256 bits */
        int32_t* flag = reinterpret_cast<int32_t*>(misc) + 8;
        __syncthreads(); /* earlier users of caps / misc are done */
        for (int i = threadIdx.x; i < (int)(sizeof(sw_repair_t) / 4); i += SW_BLOCK)
            reinterpret_cast<int32_t*>(R)[i] = 0;
        if (threadIdx.x < 8) wset[threadIdx.x] = 0;
        __syncthreads();
        for_jobs([&](int j, int s) {
            (void)s;
            if (nin[j] > 0) atomicOr(&wset[(w_in[j] >> 5) & 7], 1u << (w_in[j] & 31));
        });
        if (threadIdx.x < T) R->L[threadIdx.x] = G;
        __syncthreads();
        if (threadIdx.x == 0) {
            int32_t n = 0;
            for (int wd = 0; wd < 8; ++wd) {
                uint32_t m = wset[wd];
                while (m) {
                    const int b = __builtin_ctz(m);
                    m &= m - 1u;
                    if (n < SW_RCLS_MAX) R->wc[n] = wd * 32 + b;
                    ++n;
                }
            }
            R->ncls = n;
        }
        __syncthreads();
        if (R->ncls > SW_RCLS_MAX) return false; /* uniform */
        for_jobs([&](int j, int s) {
            (void)s;
            const uint64_t m = yd[j];
            const int32_t w = w_in[j];
            for (int t = 0; t < T; ++t)
                if ((m >> t) & 1ull) atomicSub(&R->L[t], w);
            if (nin[j] > 0) {
                const int32_t c = sw_repair_class(R, w);
                atomicAdd(&R->M[c], 1);
                atomicAdd(&R->D[c], (int32_t)nin[j] - (int32_t)pd[j]);
                for (int t = 0; t < T; ++t)
                    if ((m >> t) & 1ull) atomicAdd(&R->caps[c][t], 1);
            }
        });
        __syncthreads();
        if (threadIdx.x == 0) flag[0] = sw_profile_repair(R, T);
        __syncthreads();
        if (flag[0] != 0) return false; /* uniform */
        for_jobs([&](int j, int s) {
            (void)s;
            yout[j] = yd[j];
            pout[j] = pd[j];
        });
        for (int ci = 0; ci < R->ncls; ++ci) {
            if (!R->changed[ci]) continue;
            __syncthreads(); /* the previous class's pack has read caps */
            if (threadIdx.x < 64) caps[threadIdx.x] = threadIdx.x < T ? R->caps[ci][threadIdx.x] : 0;
            pwc = R->wc[ci];
            pack(5, nin, yout, pout);
        }
        int64_t bad = 0;
        for_jobs([&](int j, int s) {
            (void)s;
            bad += pout[j] != nin[j];
        });
        return blk.sum(bad) == 0;
    }

    /*
     * twin: pattern_pack — neither the density order nor its repair placed
     * nin: the width classes' count histograms are gathered (LDS atomics),
     * one thread searches an exact class profile over round patterns
     * (sw_profile_search, scratch in scr), and every class is packed inside
     * it (pack mode 5) into y / pout, which hold the density pack of nin.
     * True when every round of nin is placed.
     */
    __device__ __forceinline__ bool pattern_pack(const uint8_t* nin, uint64_t* y, uint8_t* pout,
                                                 int32_t* scr) {
        sw_repair_t* R = rep;
        uint32_t* wset = reinterpret_cast<uint32_t*>(misc); /* widths present: 256 bits */
        int32_t* flag = reinterpret_cast<int32_t*>(misc) + 8;
        __syncthreads(); /* earlier users of caps / misc are done */
        for (int i = threadIdx.x; i < (int)(sizeof(sw_repair_t) / 4); i += SW_BLOCK)
            reinterpret_cast<int32_t*>(R)[i] = 0;
        if (threadIdx.x < 8) wset[threadIdx.x] = 0;
        __syncthreads();
        for_jobs([&](int j, int s) {
            (void)s;
            if (nin[j] > 0) atomicOr(&wset[(w_in[j] >> 5) & 7], 1u << (w_in[j] & 31));
        });
        __syncthreads();
        if (threadIdx.x == 0) {
            int32_t n = 0;
            for (int wd = 0; wd < 8; ++wd) {
                uint32_t msk = wset[wd];
                while (msk) {
                    const int b = __builtin_ctz(msk);
                    msk &= msk - 1u;
                    if (n < SW_RCLS_MAX) R->wc[n] = wd * 32 + b;
                    ++n;
                }
            }
            R->ncls = n;
        }
        __syncthreads();
        const int K = R->ncls;
        if (K > SW_RCLS_MAX || K == 0) return false; /* uniform */
        const int HT = T + 1;
        for (int i = threadIdx.x; i < K * HT; i += SW_BLOCK) scr[i] = 0;
        __syncthreads();
        for_jobs([&](int j, int s) {
            (void)s;
            if (nin[j] > 0) {
                const int32_t c = sw_repair_class(R, w_in[j]);
                atomicAdd(&R->M[c], 1);
                atomicAdd(&scr[c * HT + nin[j]], 1);
            }
        });
        __syncthreads();
        if (threadIdx.x == 0) flag[0] = sw_profile_search(R, T, G, scr, scr + K * HT, nullptr);
        __syncthreads();
        if (flag[0] == 0) return false; /* uniform */
        for (int ci = 0; ci < K; ++ci) {
            __syncthreads(); /* the previous class's pack has read caps */
            if (threadIdx.x < 64) caps[threadIdx.x] = threadIdx.x < T ? R->caps[ci][threadIdx.x] : 0;
            pwc = R->wc[ci];
            pack(5, nin, y, pout);
        }
        int64_t bad = 0;
        for_jobs([&](int j, int s) {
            (void)s;
            bad += pout[j] != nin[j];
        });
        return blk.sum(bad) == 0;
    }

    /* The round loop of pack, run by wave 0 alone (twin: the t loop of
     * pack).  Lane L owns positions [L·PPL, L·PPL + PPL) (prefix order =
     * lane-major); their state lives at tslot(p). */
    __device__ __forceinline__ void rounds(int A_, int PPL, const int32_t* capsp) {
        rounds_mem(A_, PPL, capsp);
    }

    /* !ONE: the same loop over position state in the HBM workspace. */
    __device__ __forceinline__ void rounds_mem(int A_, int PPL, const int32_t* capsp) {
        const int lane = lane_id();
        /* lane owns positions p = lane·PPL + i, i < cnt; slot(p) = i·64 + lane */
        const int p0 = lane * PPL;
        const int cnt_l = (p0 + PPL < A_ ? p0 + PPL : A_) - p0;
        const int my = cnt_l > 0 ? cnt_l : 0;
        for (int t = 0; t < T; ++t) {
            const int R = T - t;
            int64_t cap = capsp ? capsp[t] : G;
            H[lane] = 0;
            SH[lane] = 0;
            if (lane == 0) { H[64] = 0; SH[64] = 0; }
            wave_sync();
            for (int i = 0; i < my; ++i) {
                const uint32_t s = pst[i * 64 + lane];
                const int rr = (int)st_r(s) < R ? (int)st_r(s) : R;
                atomicAdd(&H[rr], (int32_t)st_w(s));
            }
            wave_sync();
            /* need_m = Σ_{v>m} (v−m)·H[v] − room_m; lane m holds m */
            const int64_t hv = (lane + 1 <= R) ? (int64_t)H[lane + 1] : 0;
            const int64_t S0 = wave_sufscan(hv);
            const int64_t S1 = wave_sufscan(hv * (int64_t)(lane + 1));
            const int64_t room = (int64_t)sw_pack_room(capsp, t, R, G);
            const int64_t need = (lane < R) ? (S1 - (int64_t)lane * S0) - room : (int64_t)-1;
            /* tiers, highest m first */
            int mstart = R - 1;
            while (mstart >= 0) {
                const int64_t shv = (lane + 1 <= R) ? (int64_t)SH[lane + 1] : 0;
                const int64_t red = wave_sufscan(shv);
                const int64_t qv = need - red;
                const uint64_t mask = __ballot(lane <= mstart && qv > 0);
                if (mask == 0) break;
                const int m = 63 - __builtin_clzll(mask);
                const int64_t q = __shfl(qv, m, 64);
                int32_t lt = 0;
                for (int i = 0; i < my; ++i) {
                    const uint32_t s = pst[i * 64 + lane];
                    const int rr = (int)st_r(s) < R ? (int)st_r(s) : R;
                    if (!st_sel(s) && rr > m) lt += (int32_t)st_w(s);
                }
                int64_t ex = (int64_t)(wave_incscan(lt) - lt);
                int32_t took = 0;
                for (int i = 0; i < my; ++i) {
                    const int sl = i * 64 + lane;
                    const uint32_t s = pst[sl];
                    const int rr = (int)st_r(s) < R ? (int)st_r(s) : R;
                    if (!st_sel(s) && rr > m) {
                        const int64_t w = st_w(s);
                        if (ex < q && ex + w <= cap) {
                            pst[sl] = s | (1u << 16);
                            atomicAdd(&SH[rr], (int32_t)w);
                            took += (int32_t)w;
                        }
                        ex += w;
                    }
                }
                cap -= wave_sum(took);
                wave_sync();
                mstart = m - 1;
            }
            /* fill in order */
            {
                int32_t lt = 0;
                for (int i = 0; i < my; ++i) {
                    const uint32_t s = pst[i * 64 + lane];
                    if (!st_sel(s) && st_r(s) > 0) lt += (int32_t)st_w(s);
                }
                int64_t ex = (int64_t)(wave_incscan(lt) - lt);
                int32_t took = 0;
                for (int i = 0; i < my; ++i) {
                    const int sl = i * 64 + lane;
                    const uint32_t s = pst[sl];
                    if (!st_sel(s) && st_r(s) > 0) {
                        const int64_t w = st_w(s);
                        if (ex + w <= cap) { pst[sl] = s | (1u << 16); took += (int32_t)w; }
                        ex += w;
                    }
                }
                cap -= wave_sum(took);
                wave_sync();
            }
            /* width tail: first position in order that still fits */
            while (cap > 0) {
                int first = 0x7FFFFFFF;
                for (int i = 0; i < my; ++i) {
                    const uint32_t s = pst[i * 64 + lane];
                    if (!st_sel(s) && st_r(s) > 0 && (int64_t)st_w(s) <= cap) { first = p0 + i; break; }
                }
                first = wave_min(first);
                if (first == 0x7FFFFFFF) break;
                const int owner = first / PPL;
                const int sl = (first - owner * PPL) * 64 + owner;
                const uint32_t s = pst[sl];
                wave_sync();
                if (lane == owner) pst[sl] = s | (1u << 16);
                cap -= st_w(s);
                wave_sync();
            }
            /* apply: selected positions run in round t */
            for (int i = 0; i < my; ++i) {
                const int sl = i * 64 + lane;
                const uint32_t s = pst[sl];
                if (st_sel(s)) {
                    pmask[sl] |= (1ull << t);
                    pst[sl] = (s & 0xFF00u) | (st_r(s) - 1u);
                }
            }
            wave_sync();
        }
    }
};

/* Dynamic LDS of the plan kernel: the carve-up in solve_instance, region by
 * region (16-byte aligned).  The launch sizes the allocation with it and the
 * kernel compares its own carve offset against it (constant-folded). */
__host__ __device__ constexpr size_t sw_plan_lds_bytes(bool one) {
    auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    size_t s = r16(sizeof(sw_xchg)) + r16(sizeof(double) * 3 * SW_BMAX) +
               r16(sizeof(sw_pack_lds)) + r16(sizeof(int64_t) * 8) + r16(sizeof(sw_repair_t));
    if (one) {
        const size_t NJ = SW_LDS_JOBS;
        s += 8 * r16(NJ) + 3 * r16(8 * NJ) + r16(8 * 4 * SW_JPT * SW_BLOCK) + SW_JOB_LDS_BYTES;
    } else {
        /* the re-optimisation's knapsack rows and take bits (sw_reround_dev.h;
         * on chip they reuse the sort buffer and two mask rows) */
        s += 2 * r16(8 * (SW_RR_CAPMAX + 1)) + r16(8 * SW_RR_WORDS);
    }
    return s;
}

/* LDS of the level-search kernel: the setup's key staging window (whose
 * space the per-job level-search bytes reuse afterwards) and the per-job
 * constants. */
__host__ __device__ constexpr size_t sw_level_lds_bytes() {
    auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    return r16(sizeof(sw_xchg)) + r16(sizeof(double) * 3 * SW_BMAX) +
           r16(sizeof(float) * SW_JPT * SW_SETUP_CH * SW_BLOCK) + SW_JOB_LDS_BYTES;
}

/* LDS of the pack kernel: pack and repair state, counts, masks, sort exchange. */
__host__ __device__ constexpr size_t sw_pack_lds_bytes() {
    auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    const size_t NJ = SW_LDS_JOBS;
    return r16(sizeof(sw_xchg)) + r16(sizeof(sw_pack_lds)) + r16(sizeof(int64_t) * 8) +
           r16(sizeof(sw_repair_t)) + 3 * r16(NJ) + 2 * r16(8 * NJ) + r16(8 * 3 * SW_BLOCK);
}

/*
 * The level-search kernel (on-chip instances): setup and the P1 level search
 * of solve_instance's first iteration, nothing else; the counts and the best
 * level's utility, makespan, bound and passes go to HBM for sw_pack_kernel.
 * Without the packer's state its LDS is ~85 KB.
 */
template <int KT>
__device__ __forceinline__ void level_instance(const sw_batch_dev& B, unsigned char* smem, int inst_) {
    const sw_inst_dev* I = &B.inst[inst_];
    Ctx<KT, true> c;
    c.inst = I;
    c.N = I->N;
    c.T = I->T;
    c.G = I->G;
    c.nb = I->nb;
    c.C = (int64_t)I->G * I->T;
    c.k = I->k;
    c.inv_delta = 1.0 / I->delta;
    c.passes = 0;
    c.q = (c.N + SW_BLOCK - 1) / SW_BLOCK;
    const int N = c.N;
    const int64_t jo = I->job_off;
    c.w_in = B.w + jo;
    c.p_in = B.p + jo;
#ifdef SW_STAMPS
    c.swp = nullptr;
    c.lsp = nullptr;
#endif
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        unsigned char* p = smem + off;
        off += (bytes + 15) & ~(size_t)15;
        return p;
    };
    c.blk.X = (sw_xchg*)carve(sizeof(sw_xchg));
    c.blk.par = 0;
    double* bt = (double*)carve(sizeof(double) * 3 * SW_BMAX);
    c.beta = bt;
    c.ell = bt + SW_BMAX;
    c.slope = bt + 2 * SW_BMAX;
    if (threadIdx.x < SW_BMAX) {
        const int b = (int)threadIdx.x;
        bt[b] = I->beta[b];
        bt[SW_BMAX + b] = I->ell[b];
        bt[2 * SW_BMAX + b] = b < I->nb - 1 ? (I->ell[b + 1] - I->ell[b]) / (I->beta[b + 1] - I->beta[b])
                                            : 0.0;
    }
    /* the setup's staging window; the level search's per-job bytes use the
     * same space once the key rows are in registers */
    unsigned char* stage = carve(sizeof(float) * SW_JPT * SW_SETUP_CH * SW_BLOCK);
    static_assert(sizeof(float) * SW_JPT * SW_SETUP_CH * SW_BLOCK >= 5 * SW_LDS_JOBS,
                  "the staging window holds the level search's five per-job byte arrays");
    c.sbuf = reinterpret_cast<uint64_t*>(stage);
    const int NJ = SW_LDS_JOBS;
    c.ncur = stage;
    c.lcur = stage + NJ;
    c.tkcur = stage + 2 * NJ;
    c.nbest = stage + 3 * NJ;
    c.tiecur = stage + 4 * NJ;
    static_assert(sizeof(float) * SW_JPT * SW_SETUP_CH * SW_BLOCK >=
                      5 * SW_LDS_JOBS + sizeof(sw_bnb_ivl) * SW_BNB_CAP,
                  "the staging window also holds the level search's interval list");
    c.bnb = reinterpret_cast<sw_bnb_ivl*>(stage + 5 * NJ);
    c.placed = c.placed2 = c.nfin = nullptr;
    c.ycur = c.ybest = c.y2 = nullptr;
    c.pst = nullptr;
    c.pord = nullptr;
    c.pmask = nullptr;
    c.PL = nullptr;
    c.H = c.SH = c.caps = nullptr;
    c.pwc = 0;
    c.misc = nullptr;
    c.rep = nullptr;
    c.gkeys = nullptr;
    c.gjc = nullptr;
    c.JL.carve(carve);
    for (int j = threadIdx.x; j < NJ; j += SW_BLOCK)
        c.JL.put(j, j < N ? sw_make_jobc(N, c.T, I->delta, B.w[jo + j], B.d[jo + j], B.F[jo + j],
                                         B.E[jo + j], B.R[jo + j], B.p[jo + j])
                          : sw_make_jobc(1, 1, 1.0, 1, 1.0, 0, 1, 0.0, 0.0));
    if (off != sw_level_lds_bytes()) __builtin_trap();
    __syncthreads();
    c.setup(); /* its closing barrier: the staging window is free */
    const double bound = c.level_search();
    c.for_jobs([&](int j, int s) {
        (void)s;
        B.nb[jo + j] = c.nbest[j];
    });
    if (threadIdx.x == 0) {
        sw_lvl_dev v;
        v.U = c.lsU;
        v.M = c.lsM;
        v.bound = bound;
        v.passes = c.passes;
        B.lvl[inst_] = v;
    }
}

/* The 16-byte plan stores of the emit (shockwave.py:390-398 reads x[j][t]):
 * the instance's N·T-byte range written with aligned 16-byte stores, each
 * thread expanding 16 consecutive bytes from the round masks ym. */
__device__ __forceinline__ void emit_plan_bytes(uint8_t* plan, const uint64_t* ym, int N, int T) {
    const int32_t nbytes = N * T;
    const int32_t mis = (int32_t)(reinterpret_cast<uintptr_t>(plan) & 15u);
    const int32_t head = min(nbytes, (16 - mis) & 15);
    const int32_t nch = (nbytes - head) >> 4;
    auto byte_at = [&](int32_t b) {
        const int32_t j = b / T;
        return (uint8_t)((ym[j] >> (b - j * T)) & 1ull);
    };
    for (int32_t b = threadIdx.x; b < head; b += SW_BLOCK) plan[b] = byte_at(b);
    for (int32_t b = head + nch * 16 + threadIdx.x; b < nbytes; b += SW_BLOCK) plan[b] = byte_at(b);
    uint4* dst = reinterpret_cast<uint4*>(plan + head);
    for (int32_t ci = threadIdx.x; ci < nch; ci += SW_BLOCK) {
        const int32_t b0 = head + ci * 16;
        int32_t j = b0 / T, t = b0 - j * T;
        uint64_t m = ym[j];
        uint32_t wv[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            wv[k >> 2] |= (uint32_t)((m >> t) & 1ull) << ((k & 3) * 8);
            if (++t == T) {
                t = 0;
                ++j;
                if (k < 15 && j < N) m = ym[j];
            }
        }
        dst[ci] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    }
}

/*
 * The pack kernel (on-chip instances): solve_instance's path after the level
 * search when the density order places the counts (with its width-profile
 * repair if it strands rounds) — then that placement is P1's and P2's, and
 * the emit's utility and makespan are the level search's (same counts, same
 * sums).  Otherwise the instance is marked SW_STATUS_SLOW_MARK and
 * sw_plan_kernel solves it whole, as it does an instance with more than
 * SW_BLOCK jobs to place (one position per thread here).  No per-job
 * constants, no key rows: ~47 KB of LDS and ≤ 80 VGPRs, so three instances
 * share a CU.
 */
/* Returns the instance's final placement (the masks, in LDS) for the tail
 * below, or nullptr when the instance was left to sw_plan_kernel. */
__device__ __forceinline__ const uint64_t* pack_instance(const sw_batch_dev& B, unsigned char* smem, int inst_) {
    const sw_inst_dev* I = &B.inst[inst_];
    Ctx<32, true, true> c;
    c.inst = I;
    c.N = I->N;
    c.T = I->T;
    c.G = I->G;
    c.nb = I->nb;
    c.C = (int64_t)I->G * I->T;
    c.k = I->k;
    c.inv_delta = 1.0 / I->delta;
    const sw_lvl_dev lv = B.lvl[inst_];
    c.passes = lv.passes;
    c.q = (c.N + SW_BLOCK - 1) / SW_BLOCK;
    const int64_t jo = I->job_off;
    c.w_in = B.w + jo;
    c.p_in = B.p + jo;
#ifdef SW_STAMPS
    c.swp = nullptr;
    c.lsp = nullptr;
#endif
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        unsigned char* p = smem + off;
        off += (bytes + 15) & ~(size_t)15;
        return p;
    };
    c.blk.X = (sw_xchg*)carve(sizeof(sw_xchg));
    c.blk.par = 0;
    c.beta = c.ell = c.slope = nullptr;
    c.PL = (sw_pack_lds*)carve(sizeof(sw_pack_lds));
    c.H = c.PL->H[0];
    c.SH = c.PL->SH[0];
    c.caps = c.PL->H[1];
    c.pwc = 0;
    c.misc = (int64_t*)carve(sizeof(int64_t) * 8);
    c.rep = (sw_repair_t*)carve(sizeof(sw_repair_t));
    const int NJ = SW_LDS_JOBS;
    c.nbest = carve(NJ);
    c.placed = carve(NJ);
    c.placed2 = carve(NJ);
    c.ncur = c.lcur = c.tkcur = c.nfin = c.tiecur = nullptr;
    c.bnb = nullptr;
    c.ycur = (uint64_t*)carve(sizeof(uint64_t) * NJ);
    c.y2 = (uint64_t*)carve(sizeof(uint64_t) * NJ);
    c.ybest = nullptr;
    c.sbuf = (uint64_t*)carve(sizeof(uint64_t) * 3 * SW_BLOCK); /* compaction + sort_one exchange */
    c.pst = nullptr;
    c.pord = nullptr;
    c.pmask = nullptr;
    c.gkeys = nullptr;
    c.gjc = nullptr;
    if (off != sw_pack_lds_bytes()) __builtin_trap();
    int64_t act_l = 0;
    c.for_jobs([&](int j, int s) {
        (void)s;
        c.nbest[j] = B.nb[jo + j];
        act_l += c.nbest[j] > 0;
    });
    sw_out_dev* out = &B.out[inst_];
    if (c.blk.sum(act_l) > SW_BLOCK) { /* more positions than threads: sw_plan_kernel */
        if (threadIdx.x == 0) out->status = SW_STATUS_SLOW_MARK;
        return nullptr;
    }
    /* twin_plan_solve's first pack: the density order (mode 4) */
    c.pack(4, c.nbest, c.ycur, c.placed);
    int64_t def_l = 0;
    c.for_jobs([&](int j, int s) {
        (void)s;
        def_l += (int64_t)c.w_in[j] * (c.nbest[j] - c.placed[j]);
    });
    int64_t dfc = c.blk.sum(def_l);
    c.passes++;
    int32_t status = 0;
    if (dfc != 0 && c.repair_pack(c.nbest, c.ycur, c.placed, c.y2, c.placed2)) {
        c.for_jobs([&](int j, int s) {
            (void)s;
            c.ycur[j] = c.y2[j];
        });
        c.passes++;
        dfc = 0;
        status |= SW_STATUS_P2_REPAIRED;
    }
    if (dfc != 0) { /* the other P1 orders, re-solves, fill: sw_plan_kernel */
        if (threadIdx.x == 0) out->status = SW_STATUS_SLOW_MARK;
        return nullptr;
    }
    /* emit (solve_instance's, with the level search's U and M) */
    int64_t any_l = 0;
    double p2 = 0.0;
    c.for_jobs([&](int j, int s) {
        (void)s;
        const uint64_t m = c.ycur[j];
        const int cnt = __popcll(m);
        any_l += (cnt > 0);
        double term = 0.0;
        if (cnt > 0) {
            const int64_t Ssum = (int64_t)__popcll(m & 0xAAAAAAAAAAAAAAAAull) +
                                 2 * (int64_t)__popcll(m & 0xCCCCCCCCCCCCCCCCull) +
                                 4 * (int64_t)__popcll(m & 0xF0F0F0F0F0F0F0F0ull) +
                                 8 * (int64_t)__popcll(m & 0xFF00FF00FF00FF00ull) +
                                 16 * (int64_t)__popcll(m & 0xFFFF0000FFFF0000ull) +
                                 32 * (int64_t)__popcll(m & 0xFFFFFFFF00000000ull);
            term = ((double)Ssum / (double)cnt) * c.p_in[j];
        }
        p2 = p2 + term;
        B.planned[jo + j] = cnt;
    });
    const double P2 = c.blk.detsum(p2);
    const int64_t any_n = c.blk.sum(any_l); /* its barrier: every mask row is final */
    if (any_n == 0) status |= SW_STATUS_NO_PLANNED;
    /* the result record first: the reduction's values die before the plan
     * bytes' loop instead of being spilled across it */
    if (threadIdx.x == 0) {
        sw_out_dev o;
        o.objective = lv.U - c.k * lv.M;
        o.utility = lv.U;
        o.makespan = lv.M;
        o.p2_objective = P2;
        o.bound = lv.bound;
        o.iters = (int32_t)c.passes;
        o.status = status | (sw_p1_uncertified(o.objective, lv.bound) ? SW_STATUS_P1_UNCERTIFIED : 0);
        *out = o;
    }
    return c.ycur; /* the plan bytes and masks: after the exchange step (pack_tail) */
}

/*
 * The pack kernel's tail: the instance's P2 exchange step (sw_p2x_block,
 * DESIGN.md §3.6) on the placement ym the pack left in LDS, then the plan
 * bytes — stored once, from the final masks — and the masks themselves only
 * when a caller asked for them (B.want_masks).  The masks go to registers
 * first (thread l holds jobs [l·q, l·q + q), q ≤ 2 on chip), so the step may
 * reuse every byte of LDS; its 24-byte-per-job arrays go to LDS behind the
 * step's own state when the launch's allocation (B.lds_bytes) holds them, and
 * to the HBM workspace otherwise.  The same step on the same arrays as
 * sw_p2x_instance (sw_p2x_inst.h), so the same masks and P2 bits; it only
 * moves where the arrays live and drops the mask round trip through HBM
 * (written back from L2 for every instance of the batch).
 */
__device__ __forceinline__ void pack_tail(const sw_batch_dev& B, const uint64_t* ym, unsigned char* smem,
                                          int inst) {
    const sw_inst_dev* I = &B.inst[inst];
    sw_out_dev* out = &B.out[inst];
    const int N = I->N, T = I->T, G = I->G;
    const int64_t jo = I->job_off;
    const int q = (N + SW_BLOCK - 1) / SW_BLOCK; /* ≤ 2: N ≤ SW_LDS_JOBS */
    const int j0 = sw_tid_opaque() * q, j1 = min(j0 + q, N);
    __syncthreads(); /* the emit's status and ym are final; the pack's reductions are read */
    int act = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) act += (j0 + k < j1 && ym[j0 + k] != 0ull) ? 1 : 0;
    const bool run = B.fuse_p2x && !(out->status & SW_STATUS_P2_FALLBACK);
    sw_p2x_lds* L = reinterpret_cast<sw_p2x_lds*>(smem);
    const size_t Lsz = (sizeof(sw_p2x_lds) + 15) & ~(size_t)15;
    unsigned char* var = smem + Lsz;
    sw_blk blk;
    blk.X = &L->X;
    blk.par = 0;
    int A = 0;
    const int a0 = blk.exscan(act, A);
    A = __builtin_amdgcn_readfirstlane(A); /* uniform: the arrays' addresses stay scalar through the step */
    const uint64_t* yemit = ym; /* no step: ym is untouched (only blk.X was written) */
    if (run && A > 0 && A <= SW_P2X_AMAX) {
        /* the arrays in LDS behind the step's state when the allocation holds
         * them and they start past ym (read below while they are written) */
        const size_t vb = (sw_p2x_var_bytes(A, T) + 15) & ~(size_t)15;
        const bool onchip = Lsz + vb + (size_t)SW_P2X_ARR_BYTES * A <= (size_t)B.lds_bytes &&
                            var + vb >= reinterpret_cast<const unsigned char*>(ym + N);
        unsigned char* base = onchip ? var + vb : B.p2ws + (size_t)SW_P2X_ARR_BYTES * jo;
        const size_t n = onchip ? (size_t)A : (size_t)N;
        sw_p2x_arrays X;
        X.cc = reinterpret_cast<double*>(base);
        X.cm = reinterpret_cast<uint64_t*>(X.cc + n);
        X.cw = reinterpret_cast<int32_t*>(X.cm + n);
        X.cj = X.cw + n;
        for (int k = 0, a = a0; k < 2; ++k) {
            if (j0 + k >= j1) break;
            const uint64_t m = ym[j0 + k];
            if (m == 0ull) continue;
            const int j = j0 + k;
            X.cw[a] = B.w[jo + j];
            X.cj[a] = j;
            X.cc[a] = B.p[jo + j] / (double)__popcll(m);
            X.cm[a] = m;
            ++a;
        }
        __syncthreads();
#ifdef SW_STAMPS
        uint64_t* sp = B.stamps ? B.stamps + (size_t)inst * SW_STAMP_SLOTS + 32 : nullptr;
#else
        uint64_t* sp = nullptr;
#endif
        const int nc = sw_p2x_block<SW_WAVES>(blk, L, var, X, A, T, G, sp);
        __syncthreads(); /* the cancels' mask updates */
        /* the final masks: this thread's active jobs (count > 0, unchanged by
         * the step: B.planned) in compaction order, the offsets counted again
         * rather than kept live through the step */
        int act2 = 0;
        for (int j = j0r(N); j < j1r(N); ++j) act2 += B.planned[jo + j] > 0;
        int A2;
        int a = blk.exscan(act2, A2);
        uint64_t mf[2];
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int j = j0r(N) + k;
            mf[k] = 0ull;
            if (j >= j1r(N)) continue;
            if (B.planned[jo + j] <= 0) {
                acc = acc + 0.0;
                continue;
            }
            mf[k] = X.cm[a++];
            const int cnt = __popcll(mf[k]);
            const int64_t Ssum = (int64_t)__popcll(mf[k] & 0xAAAAAAAAAAAAAAAAull) +
                                 2 * (int64_t)__popcll(mf[k] & 0xCCCCCCCCCCCCCCCCull) +
                                 4 * (int64_t)__popcll(mf[k] & 0xF0F0F0F0F0F0F0F0ull) +
                                 8 * (int64_t)__popcll(mf[k] & 0xFF00FF00FF00FF00ull) +
                                 16 * (int64_t)__popcll(mf[k] & 0xFFFF0000FFFF0000ull) +
                                 32 * (int64_t)__popcll(mf[k] & 0xFFFFFFFF00000000ull);
            acc = acc + ((double)Ssum / (double)cnt) * B.p[jo + j];
        }
        if (nc > 0) { /* the P2 objective of the final masks, summed like the emit's */
            const double P2 = blk.detsum(acc);
            if (threadIdx.x == 0) {
                out->p2_objective = P2;
                out->status |= SW_STATUS_P2_EXCHANGED;
            }
        }
        __syncthreads(); /* every read of the step's LDS (and blk.X) is done: the masks go to offset 0 */
        uint64_t* yf = reinterpret_cast<uint64_t*>(smem);
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (j0r(N) + k < j1r(N)) yf[j0r(N) + k] = mf[k];
        yemit = yf;
        __syncthreads();
    }
    if (B.want_masks)
        for (int j = j0r(N); j < j1r(N); ++j) B.masks[jo + j] = yemit[j];
    emit_plan_bytes(B.plan + I->plan_off, yemit, N, T);
}

/* The re-optimisation's view of an instance (sw_reround_dev.h): the best P1
 * plan ybest / nfin; on chip the per-job values in registers, otherwise in
 * workspace rows that are free between P1 and P2. */
template <int KT, bool ONE>
struct RREnv {
    Ctx<KT, ONE>& c;
    sw_blk& blk;
    int N, T, G;
    double k;
    uint8_t *S, *Sb;
    uint32_t* items;
    double *iv, *dpA, *dpB;
    uint64_t* bits;
    double rv[SW_JPT], r0[SW_JPT], r1[SW_JPT]; /* ONE */
    double *gv, *g0, *g1;                      /* !ONE */
    __device__ RREnv(Ctx<KT, ONE>& cc) : c(cc), blk(cc.blk) {}
    template <class F>
    __device__ __forceinline__ void for_jobs(F&& f) { c.for_jobs(f); }
    __device__ __forceinline__ sw_jobc jc(int j) const { return c.jc(j, 0); }
    __device__ __forceinline__ double f(const sw_jobc& q, int n) const {
        return sw_f(&q, n, c.nb, c.beta, c.ell, c.slope);
    }
    __device__ __forceinline__ bool tj(int j) const { return c.jc(j, 0).w <= G; }
    __device__ __forceinline__ uint64_t& y(int j) { return c.ybest[j]; }
    __device__ __forceinline__ int cnt(int j) const { return c.nfin[j]; }
    __device__ __forceinline__ void add_cnt(int j, int d) { c.nfin[j] = (uint8_t)(c.nfin[j] + d); }
    __device__ __forceinline__ double& V(int j, int s) {
        if constexpr (ONE) { (void)j; return rv[s]; } else { (void)s; return gv[j]; }
    }
    __device__ __forceinline__ double& H0(int j, int s) {
        if constexpr (ONE) { (void)j; return r0[s]; } else { (void)s; return g0[j]; }
    }
    __device__ __forceinline__ double& H1(int j, int s) {
        if constexpr (ONE) { (void)j; return r1[s]; } else { (void)s; return g1[j]; }
    }
};

template <int KT, bool ONE>
__device__ __forceinline__ void solve_instance(const sw_batch_dev& B, unsigned char* smem,
                                                         int inst_) {
    const sw_inst_dev* I = &B.inst[inst_];
#ifdef SW_STAMPS
    /* placement diagnostics: 100 MHz wall clock at entry / exit, HW_ID, XCC_ID */
    const uint64_t rt0_ = __builtin_amdgcn_s_memrealtime();
#endif
    Ctx<KT, ONE> c;
    c.inst = I;
    c.N = I->N;
    c.T = I->T;
    c.G = I->G;
    c.nb = I->nb;
    c.C = (int64_t)I->G * I->T;
    c.k = I->k;
    c.inv_delta = 1.0 / I->delta;
    c.passes = 0;
    c.q = (c.N + SW_BLOCK - 1) / SW_BLOCK;
    const int N = c.N;
    const int64_t jo = I->job_off;
    c.w_in = B.w + jo;
#ifdef SW_STAMPS
    c.swp = B.stamps ? B.stamps + (size_t)inst_ * SW_STAMP_SLOTS + 8 : nullptr;
    c.lsp = B.stamps ? B.stamps + (size_t)inst_ * SW_STAMP_SLOTS + 16 : nullptr;
#endif
    c.p_in = B.p + jo;

    size_t off = 0;
    auto carve = [&](size_t bytes) {
        unsigned char* p = smem + off;
        off += (bytes + 15) & ~(size_t)15;
        return p;
    };
    c.blk.X = (sw_xchg*)carve(sizeof(sw_xchg));
    c.blk.par = 0;
    double* bt = (double*)carve(sizeof(double) * 3 * SW_BMAX);
    c.beta = bt;
    c.ell = bt + SW_BMAX;
    c.slope = bt + 2 * SW_BMAX;
    c.PL = (sw_pack_lds*)carve(sizeof(sw_pack_lds));
    c.H = c.PL->H[0];
    c.SH = c.PL->SH[0];
    c.caps = c.PL->H[1]; /* spare row of the pack LDS */
    c.pwc = 0;
    c.misc = (int64_t*)carve(sizeof(int64_t) * 8);
    c.rep = (sw_repair_t*)carve(sizeof(sw_repair_t));
    double *rr_dpA = nullptr, *rr_dpB = nullptr; /* !ONE: LDS for the re-optimisation */
    uint64_t* rr_bits = nullptr;
    if (threadIdx.x < SW_BMAX) {
        const int b = (int)threadIdx.x;
        bt[b] = I->beta[b];
        bt[SW_BMAX + b] = I->ell[b];
        /* sw_pwl_slopes, one segment per thread (same IEEE division) */
        bt[2 * SW_BMAX + b] = b < I->nb - 1 ? (I->ell[b + 1] - I->ell[b]) / (I->beta[b + 1] - I->beta[b])
                                            : 0.0;
    }
    if constexpr (ONE) {
        const int NJ = SW_LDS_JOBS;
        c.ncur = carve(NJ);
        c.lcur = carve(NJ);
        c.tkcur = carve(NJ);
        c.nbest = carve(NJ);
        c.placed = carve(NJ);
        c.placed2 = carve(NJ);
        c.nfin = carve(NJ);
        c.tiecur = carve(NJ);
        c.pst = nullptr;
        c.pord = nullptr;
        c.pmask = nullptr;
        c.ycur = (uint64_t*)carve(sizeof(uint64_t) * NJ);
        c.ybest = (uint64_t*)carve(sizeof(uint64_t) * NJ);
        c.y2 = (uint64_t*)carve(sizeof(uint64_t) * NJ);
        c.sbuf = (uint64_t*)carve(sizeof(uint64_t) * 4 * SW_JPT * SW_BLOCK);
        c.bnb = reinterpret_cast<sw_bnb_ivl*>(c.sbuf); /* free between the setup and each pack */
        c.gkeys = nullptr;
        c.gjc = nullptr;
        c.JL.carve(carve);
        /* every slot < SW_LDS_JOBS holds a valid record (a dummy past N) */
        for (int j = threadIdx.x; j < NJ; j += SW_BLOCK)
            c.JL.put(j, j < N ? sw_make_jobc(N, c.T, I->delta, B.w[jo + j], B.d[jo + j], B.F[jo + j],
                                             B.E[jo + j], B.R[jo + j], B.p[jo + j])
                              : sw_make_jobc(1, 1, 1.0, 1, 1.0, 0, 1, 0.0, 0.0));
    } else {
        uint8_t* u8 = B.ws.u8 + SW_WS_U8 * jo;
        c.ncur = u8 + 0 * (size_t)N;
        c.lcur = u8 + 1 * (size_t)N;
        c.tkcur = u8 + 2 * (size_t)N;
        c.nbest = u8 + 3 * (size_t)N;
        c.placed = u8 + 4 * (size_t)N;
        c.placed2 = u8 + 5 * (size_t)N;
        c.nfin = u8 + 6 * (size_t)N;
        c.tiecur = u8 + 7 * (size_t)N;
        /* 6N + 192 u64 per instance: three job-indexed rows, then the
         * three position-slot arrays of N + 64 entries each (pst and pord
         * use the low half of theirs) */
        uint64_t* m64 = B.ws.u64 + SW_WS_U64 * jo + (int64_t)SW_WS_PAD_U64 * inst_;
        const size_t NS = (size_t)N + 64;
        c.ycur = m64;
        c.ybest = m64 + N;
        c.y2 = m64 + 2 * (size_t)N;
        c.pmask = m64 + 3 * (size_t)N;
        c.pst = (uint32_t*)(m64 + 3 * (size_t)N + NS);
        c.pord = (int32_t*)(m64 + 3 * (size_t)N + 2 * NS);
        c.sbuf = B.ws.sort + 4 * jo;
        c.gkeys = B.ws.keys + (size_t)KT * jo;
        c.gjc = B.ws.jc + jo;
        rr_dpA = (double*)carve(8 * (SW_RR_CAPMAX + 1));
        rr_dpB = (double*)carve(8 * (SW_RR_CAPMAX + 1));
        rr_bits = (uint64_t*)carve(8 * SW_RR_WORDS);
        /* the re-optimisation's LDS is free until the end of P1 */
        static_assert(8 * (SW_RR_CAPMAX + 1) >= sizeof(sw_bnb_ivl) * SW_BNB_CAP, "interval list");
        c.bnb = reinterpret_cast<sw_bnb_ivl*>(rr_dpA);
        for (int j = c.jlo(); j < c.jhi(); ++j)
            c.gjc[j] = sw_make_jobc(N, c.T, I->delta, B.w[jo + j], B.d[jo + j], B.F[jo + j],
                                    B.E[jo + j], B.R[jo + j], B.p[jo + j]);
    }
    /* the pattern search's scratch (pattern_pack): ONE: the sort buffer; !ONE:
     * the re-optimisation's LDS rows when they hold it, else the workspace rows
     * from y2 on (dead while a P1 pack is decided: 4N + 192 words) */
    int32_t* pscr;
    if constexpr (ONE) {
        static_assert(8 * 4 * SW_JPT * SW_BLOCK >=
                          4 * (SW_RCLS_MAX * (SW_TMAX + 1) + SW_PAT_SCRATCH(SW_LDS_JOBS)),
                      "pattern scratch");
        pscr = reinterpret_cast<int32_t*>(c.sbuf);
    } else {
        const int64_t need = SW_RCLS_MAX * (SW_TMAX + 1) + SW_PAT_SCRATCH((int64_t)N);
        pscr = need <= 2 * 2 * (SW_RR_CAPMAX + 1) ? reinterpret_cast<int32_t*>(rr_dpA)
                                                  : reinterpret_cast<int32_t*>(c.y2);
    }
    /* folds away when the carve-up matches the launch's allocation */
    if (off != sw_plan_lds_bytes(ONE)) __builtin_trap();
    __syncthreads();

#ifdef SW_STAMPS
    uint64_t stamp_prev_ = __builtin_amdgcn_s_memtime();
#endif
    c.setup();
    SW_STAMP(0);

    /* ---- P1: level search + packing with budget re-solve, then P2
     *      (twin_plan_solve).  One pack call site: requests are
     *      (mode 1: P1 order A, mode 3: P1 order B, mode 2: P2). ---- */
    int32_t status = 0;
    double bound = 0.0, Jbest = 0.0, Jp = 0.0;
    int64_t deficit = 0;
    int it = 0, mode = 0; /* mode 0 = run the level search next */
    bool ok2 = true;
    bool dens = false, dens_best = false; /* P1 placed by the density order */
    bool rep = false, rep_best = false;   /* ... after a width-profile repair */
    bool dskip_best = false; /* density failed on exactly the final counts */
    while (true) {
        if (mode == 0) {
            const double b0 = c.level_search();
            if (it == 0) bound = b0;
            SW_STAMP(1);
            mode = 4; /* P1 orders: density, then A (1), then B (3) */
            dens = false;
            rep = false;
        }
        if (mode == 2) break; /* P2 below */
        uint8_t* pl = (mode == 3) ? c.placed2 : c.placed;
        uint64_t* yd = (mode == 3) ? c.y2 : c.ycur;
        c.pack(mode, c.nbest, yd, pl);
#ifdef SW_STAMPS
        const uint64_t ev0_ = __builtin_amdgcn_s_memtime();
#endif
        int64_t def_l = 0;
        double fs = 0.0, gm = 0.0;
        c.for_jobs([&](int j, int s) {
            def_l += (int64_t)c.jc(j, s).w * (c.nbest[j] - pl[j]);
            fs = fs + c.fval(j, s, pl[j]);
            gm = sw_max(gm, c.gval(j, s, pl[j]));
        });
        int64_t dfc = c.blk.sum(def_l);
        double U, Mx;
        c.blk.detsum_max(fs, gm, U, Mx);
        double Jo = U - c.k * Mx;
        c.passes++;
#ifdef SW_STAMPS
        if (threadIdx.x == 0 && c.swp) c.swp[44] += __builtin_amdgcn_s_memtime() - ev0_; /* slot 52 */
#endif
        if (mode == 4) { /* density order: also the P2 placement when it packs */
            /* stranded rounds: repair the width profile (sw_repair.h) */
            if (dfc != 0 && c.repair_pack(c.nbest, c.ycur, c.placed, c.y2, c.placed2)) {
                fs = 0.0;
                gm = 0.0;
                c.for_jobs([&](int j, int s) {
                    c.ycur[j] = c.y2[j];
                    c.placed[j] = c.placed2[j];
                    fs = fs + c.fval(j, s, c.placed[j]);
                    gm = sw_max(gm, c.gval(j, s, c.placed[j]));
                });
                c.blk.detsum_max(fs, gm, U, Mx);
                Jo = U - c.k * Mx;
                c.passes++;
                dfc = 0;
                rep = true;
            }
            if (dfc != 0) { mode = 1; continue; }
            Jp = Jo;
            deficit = 0;
            dens = true;
        } else if (mode == 1 || Jo > Jp) {
            Jp = Jo;
            deficit = dfc;
            if (mode == 3) {
                c.for_jobs([&](int j, int s) {
                    (void)s;
                    c.placed[j] = c.placed2[j];
                    c.ycur[j] = c.y2[j];
                });
            }
        }
        if (mode == 1 && dfc != 0) { mode = 3; continue; }
        /* no order places the counts: an exact class profile over round
         * patterns (twin: pattern_pack) — the counts as they are, no re-solve */
        if (deficit != 0 && c.pattern_pack(c.nbest, c.ycur, c.placed, pscr)) {
            fs = 0.0;
            gm = 0.0;
            c.for_jobs([&](int j, int s) {
                fs = fs + c.fval(j, s, c.placed[j]);
                gm = sw_max(gm, c.gval(j, s, c.placed[j]));
            });
            c.blk.detsum_max(fs, gm, U, Mx);
            Jp = U - c.k * Mx;
            c.passes++;
            deficit = 0;
        }
        /* this repack iteration is complete */
        SW_STAMP(2);
        if (it == 0 || Jp > Jbest) {
            Jbest = Jp;
            dens_best = dens;
            rep_best = rep;
            dskip_best = !dens && deficit == 0;
            c.for_jobs([&](int j, int s) {
                (void)s;
                c.nfin[j] = c.placed[j];
                c.ybest[j] = c.ycur[j];
            });
        }
        ++it;
        if (deficit == 0 || it >= SW_REPACK_ITERS) {
            SW_STAMP(3);
            mode = 2;
        } else {
            status |= SW_STATUS_P1_REPACKED;
            c.C -= deficit;
            mode = 0;
        }
        __syncthreads();
    }
    /* ---- fill of stranded capacity (twin: fill_stranded): a re-solved P1
     *      can leave round capacity idle; add single rounds there, largest
     *      utility gain first (sw_fill_key), one block max per round ---- */
    if (status & SW_STATUS_P1_REPACKED) {
        int32_t* load = c.caps; /* spare pack row, free until class-wise P2 */
        if (threadIdx.x < 64) load[threadIdx.x] = 0;
        __syncthreads();
        c.for_jobs([&](int j, int s) {
            const uint64_t m = c.ybest[j];
            const int32_t w = c.jc(j, s).w;
            for (int t = 0; t < c.T; ++t)
                if ((m >> t) & 1ull) atomicAdd(&load[t], w);
        });
        __syncthreads();
        int added = 0;
        for (int step = 0; step < SW_FILL_MAX; ++step) {
            uint64_t best = 0;
            c.for_jobs([&](int j, int s) {
                const int n = c.nfin[j];
                if (n >= c.Tj(j, s)) return;
                const uint64_t m = c.ybest[j];
                const int32_t w = c.jc(j, s).w;
                int tf = -1;
                for (int t = 0; t < c.T; ++t)
                    if (!((m >> t) & 1ull) && w <= c.G - load[t]) { tf = t; break; }
                if (tf < 0) return;
                const uint64_t key = sw_fill_key(c.fval(j, s, n + 1) - c.fval(j, s, n), j, tf);
                best = key > best ? key : best;
            });
            best = c.blk.umax(best); /* its barrier: every thread has read load */
            c.passes++;
            if (best == 0) break;
            const int jb = (int)sw_fill_job(best);
            const int tb = sw_fill_round(best);
            if (jb >= c.jlo() && jb < c.jhi()) {
                c.ybest[jb] |= 1ull << tb;
                c.nfin[jb] = (uint8_t)(c.nfin[jb] + 1);
            }
            if (threadIdx.x == 0) load[tb] += c.w_in[jb];
            ++added;
            __syncthreads();
        }
        if (added > 0) {
            dens_best = false;
            rep_best = false;
            dskip_best = false;
        }
        /* ... and re-optimise it round by round (twin: twin_reround_arrays).
         * Its scratch is the P1 level-search / packing state, dead here; on
         * chip: items in the level-search bytes, values in registers, the
         * knapsack rows in ycur / y2, take bits and item values in the sort
         * buffer */
        RREnv<KT, ONE> e(c);
        e.N = c.N;
        e.T = c.T;
        e.G = c.G;
        e.k = c.k;
        e.S = c.placed;
        e.Sb = c.placed2;
        if constexpr (ONE) {
            e.items = reinterpret_cast<uint32_t*>(c.ncur);
            e.bits = c.sbuf;
            e.iv = reinterpret_cast<double*>(c.sbuf + SW_RR_WORDS);
            e.dpA = reinterpret_cast<double*>(c.ycur);
            e.dpB = reinterpret_cast<double*>(c.y2);
            e.gv = e.g0 = e.g1 = nullptr;
        } else {
            e.items = c.pst;
            e.iv = reinterpret_cast<double*>(c.pord);
            e.gv = reinterpret_cast<double*>(c.ycur);
            e.g0 = reinterpret_cast<double*>(c.y2);
            e.g1 = reinterpret_cast<double*>(c.pmask);
            e.dpA = rr_dpA;
            e.dpB = rr_dpB;
            e.bits = rr_bits;
        }
        if (sw_rr_run(e, c.passes) > 0) {
            dens_best = false;
            rep_best = false;
            dskip_best = false;
        }
        /* ... and try raises (twin: raise_counts; sw_arith.h SW_RAISE_ITERS):
         * one job one more round, the whole plan re-placed by the pattern
         * search.  The try's counts go to nbest, its placement to ycur /
         * placed (dead here); every decision is a block reduction */
        for (int rit = 0; rit < SW_RAISE_ITERS; ++rit) {
            double fs = 0.0, gm = 0.0;
            int64_t ld_l = 0;
            c.for_jobs([&](int j, int s) {
                fs = fs + c.fval(j, s, c.nfin[j]);
                gm = sw_max(gm, c.gval(j, s, c.nfin[j]));
                ld_l += (int64_t)c.jc(j, s).w * c.nfin[j];
            });
            double U, M;
            c.blk.detsum_max(fs, gm, U, M);
            const double J = U - c.k * M;
            const int64_t load = c.blk.sum(ld_l);
            int32_t i1l = 0x7FFFFFFF; /* the first job attaining M, and the others' max */
            c.for_jobs([&](int j, int s) {
                if (j < i1l && c.gval(j, s, c.nfin[j]) == M) i1l = j;
            });
            const int32_t i1 = c.blk.min32(i1l);
            double m2l = 0.0;
            c.for_jobs([&](int j, int s) {
                if (j != i1) m2l = sw_max(m2l, c.gval(j, s, c.nfin[j]));
            });
            const double M2 = c.blk.dmax(m2l);
            c.passes++;
            int32_t tried[SW_RAISE_TRIES];
            bool took = false;
            for (int tr = 0; tr < SW_RAISE_TRIES && !took; ++tr) {
                uint64_t kl = 0;
                c.for_jobs([&](int j, int s) {
                    const int n = c.nfin[j];
                    if (n >= c.Tj(j, s)) return;
                    for (int q = 0; q < tr; ++q)
                        if (tried[q] == j) return;
                    const double Mo = j == i1 ? M2 : M;
                    const uint64_t key = sw_fill_key(sw_raise_gain(c.fval(j, s, n), c.fval(j, s, n + 1),
                                                                   c.gval(j, s, n + 1), Mo, M, c.k),
                                                     j, 0);
                    kl = key > kl ? key : kl;
                });
                const uint64_t best = c.blk.umax(kl);
                if (best == 0) break; /* uniform */
                const int b = (int)sw_fill_job(best);
                tried[tr] = b;
                if (load + c.w_in[b] > (int64_t)c.G * c.T) continue;
                /* pattern_pack rewrites the rows of the jobs with rounds; the
                 * others' rows (scratch of the re-optimisation) are cleared, as
                 * the twin's pattern_pack clears its output */
                c.for_jobs([&](int j, int s) {
                    (void)s;
                    c.nbest[j] = (uint8_t)(c.nfin[j] + (j == b ? 1 : 0));
                    c.ycur[j] = 0;
                    c.placed[j] = 0;
                });
                if (!c.pattern_pack(c.nbest, c.ycur, c.placed, pscr)) continue; /* uniform */
                double fs2 = 0.0, gm2 = 0.0;
                c.for_jobs([&](int j, int s) {
                    fs2 = fs2 + c.fval(j, s, c.placed[j]);
                    gm2 = sw_max(gm2, c.gval(j, s, c.placed[j]));
                });
                double U2, Mb2;
                c.blk.detsum_max(fs2, gm2, U2, Mb2);
                if (U2 - c.k * Mb2 > J) {
                    c.for_jobs([&](int j, int s) {
                        (void)s;
                        c.nfin[j] = c.placed[j];
                        c.ybest[j] = c.ycur[j];
                    });
                    took = true;
                }
            }
            __syncthreads();
            if (!took) break;
            dens_best = false;
            rep_best = false;
            dskip_best = false;
        }
    }
    /* ---- P2 (twin: the P2 block): (a) density order, (b) weight order,
     *      (c) class-wise inside the P1 profile — first that places every
     *      round, else the P1 placement ---- */
    auto p2_ok = [&]() {
        int64_t bad_l = 0;
        c.for_jobs([&](int j, int s) { (void)s; bad_l += (c.placed[j] != c.nfin[j]); });
        return c.blk.sum(bad_l) == 0;
    };
    ok2 = false;
    if (dens_best) { /* (a) is the P1 placement itself */
        c.for_jobs([&](int j, int s) { (void)s; c.y2[j] = c.ybest[j]; });
        ok2 = true;
        if (rep_best) status |= SW_STATUS_P2_REPAIRED;
    }
    for (int att = 0; att < 2 && !ok2; ++att) {
        if (att == 0 && dskip_best) continue;
        c.pack(att == 0 ? 4 : 2, c.nfin, c.y2, c.placed);
        ok2 = p2_ok();
        if (!ok2 && att == 0) { /* (a') density with its width profile repaired */
            ok2 = c.repair_pack(c.nfin, c.y2, c.placed, c.ycur, c.placed2);
            if (ok2) {
                c.for_jobs([&](int j, int s) { (void)s; c.y2[j] = c.ycur[j]; });
                status |= SW_STATUS_P2_REPAIRED;
            }
        }
        if (ok2 && att == 1) status |= SW_STATUS_P2_WEIGHT_ORDER;
    }
    if (!ok2) {
        int32_t wprev = 0;
        while (true) {
            int32_t wl = 0x7FFFFFFF;
            c.for_jobs([&](int j, int s) {
                const int32_t w = c.jc(j, s).w;
                if (c.nfin[j] > 0 && w > wprev && w < wl) wl = w;
            });
            const int32_t wc = c.blk.min32(wl);
            if (wc == 0x7FFFFFFF) break;
            __syncthreads(); /* the previous class's pack has read caps */
            if (threadIdx.x < 64) c.caps[threadIdx.x] = 0;
            __syncthreads();
            c.for_jobs([&](int j, int s) {
                if (c.nfin[j] > 0 && c.jc(j, s).w == wc) {
                    const uint64_t m = c.ybest[j];
                    for (int t = 0; t < c.T; ++t)
                        if ((m >> t) & 1ull) atomicAdd(&c.caps[t], 1);
                }
            });
            c.pwc = wc;
            c.pack(5, c.nfin, c.y2, c.placed);
            wprev = wc;
        }
        ok2 = p2_ok();
        if (ok2) status |= SW_STATUS_P2_CLASSWISE;
    }
    SW_STAMP(4);
    if (!ok2) status |= SW_STATUS_P2_FALLBACK;

    /* ---- emit ---- */
    int64_t any_l = 0;
    double fs = 0.0, gm = 0.0, p2 = 0.0;
    const int T = c.T;
    uint8_t* plan = B.plan + I->plan_off;
    c.for_jobs([&](int j, int s) {
        const uint64_t m = ok2 ? c.y2[j] : c.ybest[j];
        const int cnt = __popcll(m);
        any_l += (cnt > 0);
        fs = fs + c.fval(j, s, cnt);
        gm = sw_max(gm, c.gval(j, s, cnt));
        double term = 0.0;
        if (cnt > 0) {
            /* Σ_t t·bit_t of the mask: bit b of t weighted 2^b, six popcounts */
            const int64_t Ssum = (int64_t)__popcll(m & 0xAAAAAAAAAAAAAAAAull) +
                                 2 * (int64_t)__popcll(m & 0xCCCCCCCCCCCCCCCCull) +
                                 4 * (int64_t)__popcll(m & 0xF0F0F0F0F0F0F0F0ull) +
                                 8 * (int64_t)__popcll(m & 0xFF00FF00FF00FF00ull) +
                                 16 * (int64_t)__popcll(m & 0xFFFF0000FFFF0000ull) +
                                 32 * (int64_t)__popcll(m & 0xFFFFFFFF00000000ull);
            term = ((double)Ssum / (double)cnt) * c.p_in[j];
        }
        p2 = p2 + term;
        B.planned[jo + j] = cnt;
        B.masks[jo + j] = m; /* for the P2 exchange kernel (sw_p2x_kernel.hip) */
    });
    /* the four emit results in one reduction; its barrier: every mask row
     * is final */
    double U, Mact, P2;
    int64_t any_n;
    c.blk.detsum2_max_cnt(fs, p2, gm, (int32_t)any_l, U, P2, Mact, any_n);
    const bool any = any_n > 0;
    if (!any) status |= SW_STATUS_NO_PLANNED;
    /* The plan bytes (shockwave.py:390-398 reads x[j][t]) with aligned
     * 16-byte stores, each thread expanding 16 consecutive bytes from the
     * round masks (a chunk spans at most ⌈16/T⌉ + 1 jobs), byte stores only
     * for the unaligned head and tail — instead of every thread storing its
     * own jobs' bytes one at a time (strided byte stores that inflated
     * WRITE_SIZE by ~1.6x). */
    emit_plan_bytes(plan, ok2 ? c.y2 : c.ybest, N, T);
    SW_STAMP(5);
    if (threadIdx.x == 0) {
        sw_out_dev o;
        o.objective = U - c.k * Mact;
        o.utility = U;
        o.makespan = Mact;
        o.p2_objective = P2;
        o.bound = bound;
        o.iters = (int32_t)c.passes;
        o.status = status | (sw_p1_uncertified(o.objective, bound) ? SW_STATUS_P1_UNCERTIFIED : 0);
        B.out[inst_] = o;
#ifdef SW_STAMPS
        if (B.stamps) {
            uint64_t* st = B.stamps + (size_t)inst_ * SW_STAMP_SLOTS;
            st[6] = ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                    (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
            st[7] = rt0_;
            st[14] = __builtin_amdgcn_s_memrealtime();
        }
#endif
    }
}

}  // namespace

/* One workgroup per instance.  A persistent work-queue variant (each
 * workgroup pulling instances from a device counter) removed the dispatch
 * gaps between workgroups on a CU but not the tail, which is set by the
 * expensive instances taken last, and its loop cost registers: the same
 * throughput and a slower single solve. */
template <int KT, bool ONE>
__global__ __launch_bounds__(SW_BLOCK) void sw_plan_kernel(sw_batch_dev B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sw_smem[];
    /* the slow-path launch after sw_pack_kernel: only the marked instances
     * (the rest were solved, and exchanged, there) */
    if (B.only_slow && !(B.out[blockIdx.x].status & SW_STATUS_SLOW_MARK)) return;
    solve_instance<KT, ONE>(B, sw_smem, blockIdx.x);
    if constexpr (ONE) {
        /* one launch for the whole batch: the instance's P2 exchange step
         * right after its emit, in the same workgroup and LDS (the solve's
         * state is dead by now), so that one instance's exchange overlaps
         * other instances' solves instead of waiting for the slowest solve
         * of the batch (sw_p2x_inst.h) */
        if (B.fuse_p2x) {
            __syncthreads();
            sw_p2x_instance(B, B.p2ws, sw_smem, blockIdx.x);
        }
    }
}

template <int KT>
__global__ __launch_bounds__(SW_BLOCK, 4) void sw_level_kernel(sw_batch_dev B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sw_smem[];
    level_instance<KT>(B, sw_smem, blockIdx.x);
}

/* ≤ 64 VGPRs, ~37 KB of LDS: four 512-thread workgroups per CU.  The
 * instance's P2 exchange step follows its emit in the same workgroup (the
 * pack state is dead by then, its LDS is the step's): the pack's round loop
 * keeps one wave of eight busy, the exchange all eight, so on a CU whose
 * workgroups are in different phases the exchanges fill the issue slots the
 * round loops leave idle — where two kernels ran the loops of every instance
 * first and all the exchanges after them. */
__global__ __launch_bounds__(SW_BLOCK, 8) void sw_pack_kernel(sw_batch_dev B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sw_smem[];
    const uint64_t* ym = pack_instance(B, sw_smem, blockIdx.x);
    if (ym) pack_tail(B, ym, sw_smem, blockIdx.x); /* uniform: marked instances return */
}

/* LDS bytes the kernel needs (solve_instance checks its carve-up against it). */
extern "C" size_t sw_plan_kernel_lds_bytes(int one) { return sw_plan_lds_bytes(one != 0); }

/* The split path for on-chip batches (every instance N ≤ SW_LDS_JOBS and
 * T ≤ 32): level search, then pack + emit, then the full kernel for the
 * instances the pack kernel marked (B->only_slow set by the caller). */
/* Every instance's exchange step runs inside these launches: the pack
 * kernel's instances at its end, the marked ones at the end of the full
 * kernel (p2x_lds: the step's LDS for the batch's largest instance). */
extern "C" hipError_t sw_launch_split(sw_batch_dev* B, size_t p2x_lds, hipStream_t stream) {
    dim3 grid(B->count), block(SW_BLOCK);
    B->only_slow = 0;
    B->fuse_p2x = 1;
    hipLaunchKernelGGL((sw_level_kernel<32>), grid, block, sw_level_lds_bytes(), stream, *B);
    B->lds_bytes = (int32_t)std::max(sw_pack_lds_bytes(), p2x_lds);
    hipLaunchKernelGGL(sw_pack_kernel, grid, block, (size_t)B->lds_bytes, stream, *B);
    B->only_slow = 1;
    hipLaunchKernelGGL((sw_plan_kernel<32, true>), grid, block, std::max(sw_plan_lds_bytes(true), p2x_lds),
                       stream, *B);
    B->only_slow = 0;
    return hipGetLastError();
}

extern "C" hipError_t sw_launch_plan(const sw_batch_dev* B, int KT, int one, size_t lds,
                                     hipStream_t stream) {
    dim3 grid(B->count), block(SW_BLOCK);
    if (KT == 32) {
        if (one) hipLaunchKernelGGL((sw_plan_kernel<32, true>), grid, block, lds, stream, *B);
        else hipLaunchKernelGGL((sw_plan_kernel<32, false>), grid, block, lds, stream, *B);
    } else {
        /* T > 32: key rows live in the HBM workspace (a 4×64 register row
         * would not fit the on-chip budget) */
        hipLaunchKernelGGL((sw_plan_kernel<64, false>), grid, block, lds, stream, *B);
    }
    return hipGetLastError();
}
