/*
 * sw_kernels.hip — the MI355X (gfx950) plan-solve kernel.
 *
 * One 1024-thread workgroup (16 wave64) solves one instance end to end:
 *   setup     per-job constants, fp32 ranking-key rows (the fused
 *             log-utility-gradient × fairness-weight step), A = max_j a_j
 *   P1        level search over the makespan M; at each level a price
 *             bisection over the fp32 key bits (the Fisher-market price of a
 *             GPU-round), a job-ordered tie group and a width tail;
 *             then packing into rounds, re-solved on a smaller budget when
 *             widths fragment rounds                        (shockwave.py:330-388)
 *   P2        priority placement of the planned rounds    (shockwave.py:281-328)
 *   emit      plan bytes, planned-round counts, objective  (shockwave.py:390-398)
 * The algorithm is specified by, and bit-identical to, oracle/plan_twin.c:
 * each function below names the twin function it mirrors.  DESIGN.md §3
 * describes it; §4 gives the layout and the roofline.
 *
 * Instances with N ≤ 1024 (every reference configuration: 50–900 jobs) keep
 * their whole state on chip: the job's key row in VGPRs (one job per
 * thread), everything else in LDS.  Larger instances (the 10k-job C4 shape)
 * keep per-job state in an HBM workspace (L2-resident) instead.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shockwave_amd.h"
#include "sw_arith.h"
#include "sw_block.h"
#include "sw_device.h"

namespace {

struct SelEval {
    double U, Mact, J, ubound;
};

__device__ __forceinline__ uint32_t next_pow2(uint32_t v) {
    uint32_t p = 1;
    while (p < v) p <<= 1;
    return p;
}

template <int KT, bool ONE>
struct Ctx {
    /* instance scalars (uniform) */
    int32_t N, T, G, nb, q;
    int64_t C;
    double k, A;
    int64_t passes;
    const sw_inst_dev* inst;
    const double* beta; /* LDS */
    const double* ell;  /* LDS */
    sw_scratch* S;
    /* inputs (instance-relative) */
    const int32_t* w_in;
    const double* p_in;
    /* per-job state (LDS when ONE, HBM workspace otherwise) */
    uint8_t *ncur, *lcur, *tkcur, *nbest, *placed, *placed2, *nfin;
    /* per-position state of the packer */
    uint8_t *rpos, *wpos, *selp;
    int32_t* ordj;
    uint64_t *ycur, *ybest, *y2;
    uint64_t *shi, *slo;
    /* small LDS arrays */
    int32_t *H, *SH;
    int64_t* need;
    int64_t* misc;
    /* this thread's job (ONE) */
    sw_jobc jc0;
    float kr[KT];
    /* global per-job data (!ONE) */
    float* gkeys;
    sw_jobc* gjc;

    __device__ __forceinline__ int jlo() const { return (int)threadIdx.x * q; }
    __device__ __forceinline__ int jhi() const {
        int h = jlo() + q;
        return h < N ? h : N;
    }
    __device__ __forceinline__ const sw_jobc& jc(int j) const {
        if constexpr (ONE) {
            (void)j;
            return jc0;
        } else {
            return gjc[j];
        }
    }
    __device__ __forceinline__ int Tj(int j) const { return jc(j).w <= G ? T : 0; }
    __device__ __forceinline__ double fval(int j, int n) const {
        return sw_f(&jc(j), n, nb, beta, ell);
    }
    __device__ __forceinline__ double gval(int j, int n) const { return sw_g(&jc(j), n); }

    __device__ __forceinline__ uint32_t kbits(int j, int n) const {
        if constexpr (ONE) {
            (void)j;
            uint32_t v = 0;
#pragma unroll
            for (int i = 0; i < KT; ++i) v = (i == n) ? sw_fbits_of(kr[i]) : v;
            return v;
        } else {
            return sw_fbits_of(gkeys[(size_t)j * KT + n]);
        }
    }
    /* twin: lforce */
    __device__ __forceinline__ int lforce(int j, double M) const {
        const sw_jobc& c = jc(j);
        int tj = Tj(j), cnt = 0;
        if constexpr (ONE) {
#pragma unroll
            for (int n = 0; n < KT; ++n) cnt += (n < tj && sw_g(&c, n) > M);
        } else {
            for (int n = 0; n < tj; ++n) cnt += (sw_g(&c, n) > M);
        }
        return cnt;
    }
    /* twin: cnt_gt / cnt_ge */
    template <bool GE>
    __device__ __forceinline__ int cnt(int j, uint32_t rho, int l) const {
        int tj = Tj(j), c = 0;
        if constexpr (ONE) {
#pragma unroll
            for (int n = 0; n < KT; ++n) {
                uint32_t b = sw_fbits_of(kr[n]);
                bool hit = GE ? (b >= rho) : (b > rho);
                c += (n >= l && n < tj && hit);
            }
        } else {
            const float* row = gkeys + (size_t)j * KT;
            for (int n = l; n < tj; ++n) {
                uint32_t b = sw_fbits_of(row[n]);
                c += GE ? (b >= rho) : (b > rho);
            }
        }
        return c;
    }

    /* twin: build() — constants and key rows */
    __device__ __forceinline__ void setup() {
        double amax = 0.0;
        for (int j = jlo(); j < jhi(); ++j) amax = sw_max(amax, jc(j).a);
        A = block_max_d(amax, S);
        for (int j = jlo(); j < jhi(); ++j) {
            const sw_jobc& c = jc(j);
            double prev = sw_f(&c, 0, nb, beta, ell), vm = 0.0;
            if constexpr (ONE) {
#pragma unroll
                for (int n = 0; n < KT; ++n) {
                    float kv = 0.0f;
                    if (n < T) {
                        double cur = sw_f(&c, n + 1, nb, beta, ell);
                        double v = sw_pos(cur - prev);
                        vm = (n == 0) ? v : sw_min(vm, v);
                        kv = sw_key(vm, c.w, A);
                        prev = cur;
                    }
                    kr[n] = kv;
                }
            } else {
                float* row = gkeys + (size_t)j * KT;
                for (int n = 0; n < T; ++n) {
                    double cur = sw_f(&c, n + 1, nb, beta, ell);
                    double v = sw_pos(cur - prev);
                    vm = (n == 0) ? v : sw_min(vm, v);
                    row[n] = sw_key(vm, c.w, A);
                    prev = cur;
                }
            }
        }
        __syncthreads();
    }

    /* twin: select_level */
    __device__ __forceinline__ SelEval select_level(double M, bool is_inf) {
        int64_t wf = 0, wall = 0;
        for (int j = jlo(); j < jhi(); ++j) {
            int l = is_inf ? 0 : lforce(j, M);
            lcur[j] = (uint8_t)l;
            wf += (int64_t)jc(j).w * l;
            wall += (int64_t)jc(j).w * (Tj(j) - l);
        }
        int64_t Wf, Wall;
        block_sum2(wf, wall, &Wf, &Wall, S);
        passes++;
        SelEval ev;
        if (Wf > C) {
            ev.U = 0; ev.Mact = 0; ev.J = -1e308; ev.ubound = 0;
            return ev;
        }
        int64_t bud = C - Wf;
        double rho_d = 0.0;
        int64_t wgt_star;
        if (Wall <= bud) {
            for (int j = jlo(); j < jhi(); ++j) {
                ncur[j] = (uint8_t)Tj(j);
                tkcur[j] = (uint8_t)(Tj(j) - lcur[j]);
            }
            wgt_star = Wall;
        } else {
            uint32_t lo = 0, hi = SW_KEY_INF_BITS;
            while (lo < hi) {
                uint32_t mid = lo + ((hi - lo) >> 1);
                int64_t wg = 0;
                for (int j = jlo(); j < jhi(); ++j)
                    wg += (int64_t)jc(j).w * cnt<false>(j, mid, lcur[j]);
                wg = block_sum(wg, S);
                passes++;
                if (wg <= bud) hi = mid; else lo = mid + 1;
            }
            const uint32_t rho = lo;
            rho_d = (double)sw_float_of(rho);
            int64_t wt_l = 0;
            int32_t tie_w_l = 0;
            for (int j = jlo(); j < jhi(); ++j) {
                int tk = cnt<false>(j, rho, lcur[j]);
                tkcur[j] = (uint8_t)tk;
                wt_l += (int64_t)jc(j).w * tk;
                int tie = cnt<true>(j, rho, lcur[j]) - tk;
                tie_w_l += jc(j).w * tie;
            }
            const int64_t wt = block_sum(wt_l, S);
            wgt_star = wt;
            const int64_t rem = bud - wt;
            int32_t tot;
            int64_t excl = block_exscan_i32(tie_w_l, &tot, S);
            int64_t used_l = 0;
            for (int j = jlo(); j < jhi(); ++j) {
                const int tk = tkcur[j];
                const int tie = cnt<true>(j, rho, lcur[j]) - tk;
                const int64_t wj = jc(j).w;
                int tt;
                if (excl + wj * tie <= rem) tt = tie;
                else if (excl <= rem) tt = (int)((rem - excl) / wj);
                else tt = 0;
                ncur[j] = (uint8_t)(lcur[j] + tk + tt);
                used_l += wj * tt;
                excl += wj * tie;
            }
            const int64_t used = block_sum(used_l, S);
            passes++;
            int64_t rem2 = rem - used;
            while (rem2 > 0) {
                uint64_t best = 0;
                for (int j = jlo(); j < jhi(); ++j) {
                    int nj = ncur[j];
                    if (nj < Tj(j) && (int64_t)jc(j).w <= rem2) {
                        uint64_t key = ((uint64_t)kbits(j, nj) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)j);
                        best = key > best ? key : best;
                    }
                }
                best = block_max_u64(best, S);
                passes++;
                if (best == 0) break;
                const int jb = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu));
                if (jb >= jlo() && jb < jhi()) ncur[jb] = (uint8_t)(ncur[jb] + 1);
                rem2 -= w_in[jb];
            }
        }
        double fs = 0.0, gm = 0.0;
        for (int j = jlo(); j < jhi(); ++j) {
            fs = fs + fval(j, ncur[j]);
            gm = sw_max(gm, gval(j, ncur[j]));
        }
        ev.U = block_detsum(fs, S);
        ev.Mact = block_max_d(gm, S);
        ev.J = ev.U - k * ev.Mact;
        double ub = 0.0;
        for (int j = jlo(); j < jhi(); ++j) ub = ub + fval(j, lcur[j] + tkcur[j]);
        ev.ubound = block_detsum(ub, S) + (rho_d * A) * (double)(bud - wgt_star);
        passes++;
        return ev;
    }

    __device__ __forceinline__ void keep_best(const SelEval& e, SelEval& best) {
        if (e.J > best.J || (e.J == best.J && e.Mact < best.Mact)) {
            best = e;
            for (int j = jlo(); j < jhi(); ++j) nbest[j] = ncur[j];
        }
    }

    /* twin: feasible_level */
    __device__ __forceinline__ bool feasible_level(double M) {
        int64_t wf = 0;
        for (int j = jlo(); j < jhi(); ++j) wf += (int64_t)jc(j).w * lforce(j, M);
        wf = block_sum(wf, S);
        passes++;
        return wf <= C;
    }

    /* twin: levels_between */
    __device__ __forceinline__ int64_t levels_between(double a, double b) {
        int64_t c = 0;
        for (int j = jlo(); j < jhi(); ++j) {
            const sw_jobc& cj = jc(j);
            int tj = Tj(j);
            if constexpr (ONE) {
#pragma unroll
                for (int n = 0; n <= KT; ++n) {
                    double v = sw_g(&cj, n);
                    c += (n <= tj && v > a && v < b);
                }
            } else {
                for (int n = 0; n <= tj; ++n) {
                    double v = sw_g(&cj, n);
                    c += (v > a && v < b);
                }
            }
        }
        c = block_sum(c, S);
        passes++;
        return c;
    }

    /* twin: level_search — best counts land in nbest; returns the bound */
    __device__ __forceinline__ double level_search() {
        SelEval best = select_level(0.0, true);
        for (int j = jlo(); j < jhi(); ++j) nbest[j] = ncur[j];
        const double U_inf = best.U, M_free = best.Mact, ub_inf = best.ubound;
        double M_lo = M_free;
        if (N > 0 && k > 0.0) {
            double lb = 0.0;
            for (int j = jlo(); j < jhi(); ++j) lb = sw_max(lb, gval(j, Tj(j)));
            lb = block_max_d(lb, S);
            uint64_t lo = sw_bits(lb), hi = sw_bits(M_free);
            while (lo < hi) {
                uint64_t mid = lo + ((hi - lo) >> 1);
                if (feasible_level(sw_from_bits(mid))) hi = mid; else lo = mid + 1;
            }
            M_lo = sw_from_bits(lo);
            SelEval ev = select_level(M_lo, false);
            keep_best(ev, best);
            const double width = (U_inf - ev.U) / k;
            double a = M_lo, b = sw_min(M_free, M_lo + width);
            for (int it = 0; it < SW_GS_ITERS; ++it) {
                if (!(a < b)) break;
                if (levels_between(a, b) == 0) break;
                const double m1 = a + (b - a) * SW_GS_A;
                const double m2 = a + (b - a) * SW_GS_B;
                SelEval e1 = select_level(m1, false);
                keep_best(e1, best);
                SelEval e2 = select_level(m2, false);
                keep_best(e2, best);
                if (e1.J >= e2.J) b = m2; else a = m1;
            }
        }
        __syncthreads();
        return ub_inf - k * M_lo;
    }

    /* Bitonic sort of (shi, slo) descending over NP entries, staged in LDS. */
    __device__ __forceinline__ void bitonic_desc(int NP) {
        for (int kk = 2; kk <= NP; kk <<= 1) {
            for (int jj = kk >> 1; jj > 0; jj >>= 1) {
                for (int i = threadIdx.x; i < NP; i += SW_BLOCK) {
                    int ixj = i ^ jj;
                    if (ixj > i) {
                        uint64_t ah = shi[i], al = slo[i], bh = shi[ixj], bl = slo[ixj];
                        bool a_gt = (ah > bh) || (ah == bh && al > bl);
                        bool up = ((i & kk) == 0);
                        /* descending overall: in "up" blocks larger first */
                        bool swap = up ? !a_gt : a_gt;
                        if (swap) {
                            shi[i] = bh; slo[i] = bl; shi[ixj] = ah; slo[ixj] = al;
                        }
                    }
                }
                __syncthreads();
            }
        }
    }

    /*
     * twin: pack — place nin[j] rounds per job into T rounds of capacity G.
     * MODE 1: P1 packing order (makespan-critical first, then marginal key);
     * MODE 2: P2 order (p_j / n_j desc).  Writes masks y[job], placed[job].
     */
    template <int MODE>
    __device__ __forceinline__ void pack(const uint8_t* nin, uint64_t* y, uint8_t* placed_out) {
        __syncthreads();
        double Mb = 0.0;
        if (MODE != 2) {
            for (int j = jlo(); j < jhi(); ++j) Mb = sw_max(Mb, gval(j, nin[j]));
            Mb = block_max_d(Mb, S);
        }
        const int NP = (int)next_pow2((uint32_t)(N > 0 ? N : 1));
        for (int i = threadIdx.x; i < NP; i += SW_BLOCK) { shi[i] = 0; slo[i] = 0; }
        __syncthreads();
        int act_l = 0;
        for (int j = jlo(); j < jhi(); ++j) {
            y[j] = 0;
            const int nj = nin[j];
            if (nj > 0) {
                uint64_t k1;
                uint32_t k2;
                if (MODE != 2) {
                    /* twin: orders A (MODE 1) and B (MODE 3) */
                    double lvl = gval(j, nj - 1);
                    bool crit = k > 0.0 && lvl > Mb;
                    k1 = crit ? (SW_CRIT_BIT | sw_bits(lvl)) : (MODE == 3 ? (uint64_t)jc(j).w : 0);
                    k2 = kbits(j, nj - 1);
                } else {
                    k1 = sw_bits(p_in[j] / (double)nj);
                    k2 = 0;
                }
                shi[j] = k1;
                slo[j] = ((uint64_t)k2 << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)j);
                act_l++;
            }
        }
        const int A_ = (int)block_sum(act_l, S);
        bitonic_desc(NP);
        const int q2 = (A_ + SW_BLOCK - 1) / SW_BLOCK;
        const int plo = (int)threadIdx.x * q2;
        const int phi = plo + q2 < A_ ? plo + q2 : A_;
        for (int i = plo; i < phi; ++i) {
            const int j = (int)(0xFFFFFFFFu - (uint32_t)(slo[i] & 0xFFFFFFFFu));
            ordj[i] = j;
            rpos[i] = nin[j];
            wpos[i] = (uint8_t)w_in[j];
            selp[i] = 0;
        }
        __syncthreads();
        for (int t = 0; t < T; ++t) {
            const int R = T - t;
            int64_t cap = G;
            if ((int)threadIdx.x <= R) { H[threadIdx.x] = 0; SH[threadIdx.x] = 0; }
            __syncthreads();
            for (int i = plo; i < phi; ++i) {
                int rr = rpos[i] < R ? rpos[i] : R;
                atomicAdd(&H[rr], (int32_t)wpos[i]);
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                int64_t S0 = 0, S1 = 0;
                for (int m = R - 1; m >= 0; --m) {
                    const int v = m + 1;
                    S0 += H[v];
                    S1 += (int64_t)v * H[v];
                    need[m] = (S1 - (int64_t)m * S0) - (int64_t)G * (R - 1 - m);
                }
            }
            __syncthreads();
            /* tiers (twin: m loop with q = need[m] - red) */
            int mstart = R - 1;
            while (true) {
                if (threadIdx.x == 0) {
                    int mf = -1;
                    int64_t qf = 0, red = 0;
                    for (int v = mstart + 1; v <= R; ++v) red += SH[v];
                    for (int m = mstart; m >= 0; --m) {
                        int64_t qq = need[m] - red;
                        if (qq > 0) { mf = m; qf = qq; break; }
                        red += SH[m];
                    }
                    misc[0] = mf;
                    misc[1] = qf;
                }
                __syncthreads();
                const int m = (int)misc[0];
                const int64_t qv = misc[1];
                __syncthreads();
                if (m < 0) break;
                int32_t lv = 0;
                for (int i = plo; i < phi; ++i) {
                    int rr = rpos[i] < R ? rpos[i] : R;
                    if (!selp[i] && rr > m) lv += wpos[i];
                }
                int32_t tot;
                int64_t ex = block_exscan_i32(lv, &tot, S);
                int64_t took_l = 0;
                for (int i = plo; i < phi; ++i) {
                    int rr = rpos[i] < R ? rpos[i] : R;
                    if (!selp[i] && rr > m) {
                        if (ex < qv && ex + wpos[i] <= cap) {
                            selp[i] = 1;
                            atomicAdd(&SH[rr], (int32_t)wpos[i]);
                            took_l += wpos[i];
                        }
                        ex += wpos[i];
                    }
                }
                cap -= block_sum(took_l, S);
                mstart = m - 1;
            }
            /* fill */
            {
                int32_t lv = 0;
                for (int i = plo; i < phi; ++i)
                    if (!selp[i] && rpos[i] > 0) lv += wpos[i];
                int32_t tot;
                int64_t ex = block_exscan_i32(lv, &tot, S);
                int64_t took_l = 0;
                for (int i = plo; i < phi; ++i) {
                    if (!selp[i] && rpos[i] > 0) {
                        if (ex + wpos[i] <= cap) { selp[i] = 1; took_l += wpos[i]; }
                        ex += wpos[i];
                    }
                }
                cap -= block_sum(took_l, S);
            }
            /* width tail */
            while (cap > 0) {
                uint64_t best = 0;
                for (int i = plo; i < phi; ++i)
                    if (!selp[i] && rpos[i] > 0 && (int64_t)wpos[i] <= cap) {
                        uint64_t key = (uint64_t)(0xFFFFFFFFu - (uint32_t)i);
                        best = key > best ? key : best;
                    }
                best = block_max_u64(best, S);
                if (best == 0) break;
                const int pick = (int)(0xFFFFFFFFu - (uint32_t)best);
                if (pick >= plo && pick < phi) selp[pick] = 1;
                cap -= wpos[pick];
            }
            for (int i = plo; i < phi; ++i) {
                if (selp[i]) {
                    y[ordj[i]] |= (1ull << t);
                    rpos[i] = (uint8_t)(rpos[i] - 1);
                    selp[i] = 0;
                }
            }
            __syncthreads();
        }
        for (int j = jlo(); j < jhi(); ++j) placed_out[j] = 0;
        __syncthreads();
        for (int i = plo; i < phi; ++i) placed_out[ordj[i]] = (uint8_t)(nin[ordj[i]] - rpos[i]);
        __syncthreads();
    }
};

template <int KT, bool ONE>
__device__ __forceinline__ void solve_instance(const sw_batch_dev& B, unsigned char* smem) {
    const sw_inst_dev* I = &B.inst[blockIdx.x];
    Ctx<KT, ONE> c;
    c.inst = I;
    c.N = I->N;
    c.T = I->T;
    c.G = I->G;
    c.nb = I->nb;
    c.C = (int64_t)I->G * I->T;
    c.k = I->k;
    c.passes = 0;
    c.q = (c.N + SW_BLOCK - 1) / SW_BLOCK;
    const int N = c.N;
    const int64_t jo = I->job_off;
    c.w_in = B.w + jo;
    c.p_in = B.p + jo;

    /* LDS carve-up (16-byte aligned pieces) */
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        unsigned char* p = smem + off;
        off += (bytes + 15) & ~(size_t)15;
        return p;
    };
    c.S = (sw_scratch*)carve(sizeof(sw_scratch));
    double* bt = (double*)carve(sizeof(double) * 2 * SW_BMAX);
    c.beta = bt;
    c.ell = bt + SW_BMAX;
    c.H = (int32_t*)carve(sizeof(int32_t) * (SW_TMAX + 2));
    c.SH = (int32_t*)carve(sizeof(int32_t) * (SW_TMAX + 2));
    c.need = (int64_t*)carve(sizeof(int64_t) * SW_TMAX);
    c.misc = (int64_t*)carve(sizeof(int64_t) * 8);
    if (threadIdx.x < SW_BMAX) {
        bt[threadIdx.x] = I->beta[threadIdx.x];
        bt[SW_BMAX + threadIdx.x] = I->ell[threadIdx.x];
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
        c.rpos = carve(NJ);
        c.wpos = carve(NJ);
        c.selp = carve(NJ);
        c.ordj = (int32_t*)carve(sizeof(int32_t) * NJ);
        c.ycur = (uint64_t*)carve(sizeof(uint64_t) * NJ);
        c.ybest = (uint64_t*)carve(sizeof(uint64_t) * NJ);
        c.y2 = (uint64_t*)carve(sizeof(uint64_t) * NJ);
        c.shi = (uint64_t*)carve(sizeof(uint64_t) * NJ);
        c.slo = (uint64_t*)carve(sizeof(uint64_t) * NJ);
        c.gkeys = nullptr;
        c.gjc = nullptr;
        const int j = (int)threadIdx.x;
        if (j < N) {
            c.jc0 = sw_make_jobc(N, c.T, I->delta, B.w[jo + j], B.d[jo + j], B.F[jo + j],
                                 B.E[jo + j], B.R[jo + j], B.p[jo + j]);
        } else {
            c.jc0 = sw_make_jobc(1, 1, 1.0, 1, 1.0, 0, 1, 0.0, 0.0);
        }
    } else {
        uint8_t* u8 = B.ws.u8 + SW_WS_U8 * jo;
        c.ncur = u8 + 0 * (size_t)N;
        c.lcur = u8 + 1 * (size_t)N;
        c.tkcur = u8 + 2 * (size_t)N;
        c.nbest = u8 + 3 * (size_t)N;
        c.placed = u8 + 4 * (size_t)N;
        c.nfin = u8 + 5 * (size_t)N;
        c.rpos = u8 + 6 * (size_t)N;
        c.wpos = u8 + 7 * (size_t)N;
        c.selp = u8 + 8 * (size_t)N;
        c.placed2 = u8 + 9 * (size_t)N;
        uint64_t* m64 = B.ws.u64 + 4 * jo;
        c.ycur = m64;
        c.ybest = m64 + N;
        c.y2 = m64 + 2 * (size_t)N;
        c.ordj = (int32_t*)(m64 + 3 * (size_t)N); /* N int32 fit in N u64 */
        c.shi = B.ws.sort + 4 * jo;
        c.slo = c.shi + 2 * (size_t)N;
        c.gkeys = B.ws.keys + (size_t)KT * jo;
        c.gjc = B.ws.jc + jo;
        for (int j = c.jlo(); j < c.jhi(); ++j)
            c.gjc[j] = sw_make_jobc(N, c.T, I->delta, B.w[jo + j], B.d[jo + j], B.F[jo + j],
                                    B.E[jo + j], B.R[jo + j], B.p[jo + j]);
    }
    __syncthreads();

    c.setup();

    /* ---- P1: level search + packing with budget re-solve (twin: twin_plan_solve) ---- */
    int32_t status = 0;
    double bound = 0.0, Jbest = 0.0;
    for (int it = 0; it < SW_REPACK_ITERS; ++it) {
        const double b0 = c.level_search();
        if (it == 0) bound = b0;
        /* order A; order B only if A left rounds unplaced (twin: ord loop) */
        int64_t deficit = 0;
        double Jp = 0.0;
        for (int ord = 0; ord < 2; ++ord) {
            uint8_t* pl = ord ? c.placed2 : c.placed;
            if (ord == 0) c.template pack<1>(c.nbest, c.ycur, pl);
            else c.template pack<3>(c.nbest, c.y2, pl);
            int64_t def_l = 0;
            double fs = 0.0, gm = 0.0;
            for (int j = c.jlo(); j < c.jhi(); ++j) {
                def_l += (int64_t)c.jc(j).w * (c.nbest[j] - pl[j]);
                fs = fs + c.fval(j, pl[j]);
                gm = sw_max(gm, c.gval(j, pl[j]));
            }
            const int64_t dfc = block_sum(def_l, c.S);
            const double Jo = block_detsum(fs, c.S) - c.k * block_max_d(gm, c.S);
            c.passes++;
            if (ord == 0 || Jo > Jp) {
                Jp = Jo;
                deficit = dfc;
                if (ord == 1) {
                    for (int j = c.jlo(); j < c.jhi(); ++j) {
                        c.placed[j] = c.placed2[j];
                        c.ycur[j] = c.y2[j];
                    }
                }
            }
            if (ord == 0 && dfc == 0) break;
        }
        if (it == 0 || Jp > Jbest) {
            Jbest = Jp;
            for (int j = c.jlo(); j < c.jhi(); ++j) {
                c.nfin[j] = c.placed[j];
                c.ybest[j] = c.ycur[j];
            }
        }
        if (deficit == 0) break;
        status |= SW_STATUS_P1_REPACKED;
        c.C -= deficit;
    }
    /* ---- P2 (twin: priority placement of the same counts) ---- */
    c.template pack<2>(c.nfin, c.y2, c.placed);
    int64_t bad_l = 0;
    for (int j = c.jlo(); j < c.jhi(); ++j) bad_l += (c.placed[j] != c.nfin[j]);
    const bool ok2 = block_sum(bad_l, c.S) == 0;
    if (!ok2) status |= SW_STATUS_P2_FALLBACK;

    /* ---- emit ---- */
    int64_t any_l = 0;
    double fs = 0.0, gm = 0.0, p2 = 0.0;
    const int T = c.T;
    uint8_t* plan = B.plan + I->plan_off;
    for (int j = c.jlo(); j < c.jhi(); ++j) {
        const uint64_t m = ok2 ? c.y2[j] : c.ybest[j];
        const int cnt = __popcll(m);
        any_l += (cnt > 0);
        fs = fs + c.fval(j, cnt);
        gm = sw_max(gm, c.gval(j, cnt));
        double term = 0.0;
        if (cnt > 0) {
            int64_t Ssum = 0;
            for (int t = 0; t < T; ++t) Ssum += ((m >> t) & 1ull) ? t : 0;
            term = ((double)Ssum / (double)cnt) * c.p_in[j];
        }
        p2 = p2 + term;
        for (int t = 0; t < T; ++t) plan[(size_t)j * T + t] = (uint8_t)((m >> t) & 1ull);
        B.planned[jo + j] = cnt;
    }
    const bool any = block_sum(any_l, c.S) > 0;
    if (!any) status |= SW_STATUS_NO_PLANNED;
    const double U = block_detsum(fs, c.S);
    const double Mact = block_max_d(gm, c.S);
    const double P2 = block_detsum(p2, c.S);
    if (threadIdx.x == 0) {
        sw_out_dev o;
        o.objective = U - c.k * Mact;
        o.utility = U;
        o.makespan = Mact;
        o.p2_objective = P2;
        o.bound = bound;
        o.iters = (int32_t)c.passes;
        o.status = status;
        B.out[blockIdx.x] = o;
    }
}

}  // namespace

template <int KT, bool ONE>
__global__ __launch_bounds__(SW_BLOCK) void sw_plan_kernel(sw_batch_dev B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sw_smem[];
    solve_instance<KT, ONE>(B, sw_smem);
}

/* LDS bytes the kernel needs (must match the carve-up above). */
extern "C" size_t sw_plan_kernel_lds_bytes(int one) {
    auto r16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    size_t s = r16(sizeof(sw_scratch)) + r16(sizeof(double) * 2 * SW_BMAX) +
               2 * r16(sizeof(int32_t) * (SW_TMAX + 2)) + r16(sizeof(int64_t) * SW_TMAX) +
               r16(sizeof(int64_t) * 8);
    if (one) {
        const size_t NJ = SW_LDS_JOBS;
        s += 10 * r16(NJ) + r16(4 * NJ) + 5 * r16(8 * NJ);
    }
    return s;
}

extern "C" hipError_t sw_launch_plan(const sw_batch_dev* B, int KT, int one, size_t lds,
                                     hipStream_t stream) {
    dim3 grid(B->count), block(SW_BLOCK);
    if (KT == 32) {
        if (one) hipLaunchKernelGGL((sw_plan_kernel<32, true>), grid, block, lds, stream, *B);
        else hipLaunchKernelGGL((sw_plan_kernel<32, false>), grid, block, lds, stream, *B);
    } else {
        if (one) hipLaunchKernelGGL((sw_plan_kernel<64, true>), grid, block, lds, stream, *B);
        else hipLaunchKernelGGL((sw_plan_kernel<64, false>), grid, block, lds, stream, *B);
    }
    return hipGetLastError();
}
