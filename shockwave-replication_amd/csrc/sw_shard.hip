/*
 * sw_shard.hip — sharded single-instance plan solve on MI355X
 * (include/shockwave_amd.h sw_dist_*).
 *
 * One process per GPU holds a contiguous slice of the jobs (sw_shard_range).
 * The controller (sw_shard_ctl.h, the algorithm of oracle/plan_twin.c as a
 * sequence of steps) runs on the host of every rank; this file is its GPU
 * engine.  Each step is
 *      one or two kernels over the rank's jobs in HBM
 *   →  one collective on the handle's stream (RCCL over xGMI, or host
 *      callbacks)
 *   →  a few bytes back to the host (pinned), one stream sync.
 * The placement steps never come back to the host: local keys → all-gather
 * → all-pairs rank sort → block-wide round loop, all on the stream.
 *
 * Layout in HBM (per rank, NL local jobs, T rounds):
 *   jc[NL] (sw_jobc, 64 B)   keys[NL][T] fp32   l, taken, 5 count arrays [NL] i32
 *   3 round-bitmask arrays [NL] u64   plan[NL][T] u8   planned[NL] i32
 *   red[128] i64 (step results)   exchange blocks for the gathers
 *   placement: send[P] / all[W·P] entries (24 B), chunk-sorted keys and
 *   entries [W·P rounded up to 1024], order[W·P]
 *
 * Kernels and what bounds them (all latency-bound at C4's 1,250 jobs per
 * rank; DESIGN.md §7 has the per-step budget):
 *   k_force / k_take / k_between / k_tail_best   thread per job, binary
 *        searches on the monotone g and key rows, wave reductions + atomics
 *   k_probe    thread per (job, round) item: one binary search over the ≤63
 *        ascending thresholds, an LDS histogram, a suffix sum on the host —
 *        K price/level probes per pass (K-ary search)
 *   k_assign   thread per job: the job-ordered tie group, block offsets
 *        from k_take's per-block tie sums plus a block scan
 *   k_eval     per-job values (thread per job) into LDS, then a thread per
 *        deterministic-sum lane sums its jobs left to right (sw_detsum's
 *        chunks), so the gathered lanes reproduce the single-instance sums
 *        bit for bit; one launch per reduction step
 *   k_pack_chunk_sort / k_pack_merge_rank   the global placement order: LDS
 *        bitonic sort per 1024-entry chunk, ranks by binary searches in the
 *        other sorted chunks
 *   k_pack_rounds   the round loop of the placement (sw_pack.h)
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <new>
#include <string>
#include <vector>

#include "../../include/shockwave_amd.h"
#include "sw_arith.h"
#include "sw_block.h"
#include "sw_device.h"
#include "sw_handle.h"
#include "sw_p2x.h"
#include "sw_p2x_dev.h"
#include "sw_pack.h"
#include "sw_reround_dev.h"
#include "sw_shard_ctl.h"
#include "sw_validate.h"

#ifdef SW_STAMPS
/* diagnostic builds: k_pack_rounds phase cycles (sw_pack.h SWP_STAMP) */
__device__ uint64_t g_sw_pack_stamps[24]; /* swp[0..7] phases, [17..19] counters */
#endif

namespace {

constexpr int kTB = 256;  /* threads per block of the per-job kernels */
constexpr int kRed = 320; /* entries of a step-result slice (a probe's SW_SHARD_K + 1 bins) */
constexpr int kRing = 64; /* step-result slices cleared together      */
constexpr int kProbeBlocks = 256; /* grid of the K-ary price probes (SW_PROBE_BLOCKS overrides; 0 = full) */
int probe_blocks(unsigned pb) {
    static const int v = [] {
        const char* e = getenv("SW_PROBE_BLOCKS");
        return e ? atoi(e) : kProbeBlocks;
    }();
    return (v <= 0 || pb <= (unsigned)v) ? (int)pb : v;
}
/* a pack's per-round capacities, passed by value (no staging copy) */
struct CapsArg {
    int32_t v[SW_TMAX];
    int32_t has; /* 0: capacity G in every round */
};

struct sw_pack_ent {
    uint64_t khi, klo; /* order key (desc); klo low 32 bits = ~job */
    uint32_t st;       /* rounds | width << 8 (0 = not placed)      */
    uint32_t pad;
};

/* kernel view of one rank's shard (passed by value) */
struct ShardDev {
    int32_t NL, T, G, nb, LW, rank;
    int64_t off, N, q, P;
    /* the share placement's shares on this rank (sw_share_count): nsub of
     * them, share s holding the local jobs [s·Ps, (s + 1)·Ps) and its
     * placement entries at [s·Pp, s·Pp + Ps) (Pp: Ps rounded up to the sort's
     * chunk) */
    int32_t nsub;
    int64_t Ps, Pp;
    double k;
    double beta[SW_BMAX], ell[SW_BMAX], slope[SW_BMAX];
    const sw_jobc* jc;
    float* keys;
    const double* p;
    int32_t* l;
    int32_t* taken;
    int32_t* tie; /* w·(count(key ≥ ρ) − taken), stored by k_take */
    long long* tieblk; /* Σ tie per k_take block (k_assign's offsets) */
    double* xa;   /* per-job values of the last reduction (two rows of NL) */
    int32_t* arr[SW_A_COUNT];
    uint64_t* y[SW_Y_COUNT];
    uint8_t* plan;
    int32_t* planned;
    long long* red; /* i64 / u64-bit step results */
    /* fused publish (world 1): the kernel's last block stores the step result
     * into pinned host memory and releases the flag itself, instead of a
     * k_publish launch behind it (dst = nullptr: not armed) */
    struct {
        uint32_t* dst;
        unsigned long long* flag;
        unsigned long long seq;
        const uint32_t* src;
        const int* xerr;
        int nwords;
    } pub;
};

/* Device-side state of a solve's common path (fast_solve): every decision the
 * controller (sw_shard_ctl.h) makes on that path, taken by the kernels from
 * the step results in device memory instead of by the host.  escape != 0:
 * the solve left the common path (a width tail, a level search that needs
 * its branch and bound, a share pack that strands rounds, invalid inputs);
 * the host then solves it again with the host-driven controller. */
struct FastCtl {
    long long C, bud, Wall, wt, rem, used;
    int all, escape, did_between, tail_steps; /* tail_steps: the width tail's steps (k_fast_tail) */
    double k, A, M_lo, U, Mact, ubound, Umax, bmax;
};

/* The last step of a device-chained search, applied by the kernel that
 * consumes its answer (fast_solve) instead of a k_search_update launch:
 * every block steps X_{nr−1} = x (its bins / gathered lists), block 0 stores
 * X_nr at xo.  x = nullptr: no search to finish. */
struct SearchTail {
    const unsigned long long* x;
    unsigned long long* xo;
    const long long* bins;
    const unsigned long long* lists;
    int W;
};
__device__ uint64_t search_tail(const SearchTail& t);

struct Thresholds {
    uint64_t v[SW_SHARD_K]; /* u32 key bits or fp64 bits, ascending */
    uint64_t lo;            /* the bracket's lower end (bin 0 counts the items ≥ it) */
    int32_t K;
};

__device__ __forceinline__ int tj_of(const ShardDev& S, const sw_jobc& c) { return c.w <= S.G ? S.T : 0; }

__device__ __forceinline__ int g_count_gt(const sw_jobc& c, int hi, double x) {
    int lo = 0;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sw_g(&c, mid) > x) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int g_count_ge(const sw_jobc& c, int hi, double x) {
    int lo = 0;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sw_g(&c, mid) >= x) lo = mid + 1; else hi = mid;
    }
    return lo;
}
/* #{n ∈ [l, tj) : key(n) > ρ (≥ ρ)} — keys are nonincreasing along the row */
template <bool GE>
__device__ __forceinline__ int key_count(const float* row, int l, int tj, uint32_t rho) {
    int lo = l, hi = tj;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const uint32_t b = sw_fbits_of(row[mid]);
        if (GE ? (b >= rho) : (b > rho)) lo = mid + 1; else hi = mid;
    }
    return lo - l;
}

__device__ __forceinline__ void red_add(long long* dst, long long v) {
    v = wave_sum(v);
    if (lane_id() == 0 && v != 0) atomicAdd((unsigned long long*)dst, (unsigned long long)v);
}
__device__ __forceinline__ void red_umax(long long* dst, uint64_t v) {
    v = wave_max(v);
    if (lane_id() == 0 && v != 0) atomicMax((unsigned long long*)dst, (unsigned long long)v);
}

/* The step result to the host (k_publish's stores, by one whole block): the
 * words read at device scope (other blocks' atomics and stores), then the
 * error word, a system-scope fence and the flag's release.  Plain vector
 * stores, no scalar-cache writes. */
__device__ __forceinline__ void pub_store(const ShardDev& S) {
    for (int i = threadIdx.x; i < S.pub.nwords; i += blockDim.x)
        S.pub.dst[i] = __hip_atomic_load(S.pub.src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) S.pub.dst[S.pub.nwords] = S.pub.xerr ? (uint32_t)*S.pub.xerr : 0u;
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(S.pub.flag, S.pub.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int kRedCtr = 300; /* a step-result slot no step uses: the last-block counter */
static_assert(SW_SHARD_K + 1 <= kRedCtr && kRedCtr < kRed, "the probe bins stay below the counter slot");
/* At the end of a step kernel, by every thread that did not return: when
 * armed, the last block to finish (counter red[kRedCtr], zero in every fresh
 * step slice) publishes.  Uniform over the grid: S.pub is a kernel argument. */
__device__ __forceinline__ void pub_tail(const ShardDev& S) {
    if (!S.pub.dst) return;
    __shared__ int last_;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0)
        last_ = atomicAdd((unsigned long long*)(S.red + kRedCtr), 1ull) == (unsigned long long)(gridDim.x - 1);
    __syncthreads();
    if (!last_) return;
    __threadfence();
    pub_store(S);
}

/* ---- setup ---------------------------------------------------------------- */

__global__ __launch_bounds__(kTB) void k_setup(ShardDev S, sw_jobc* jc, const int32_t* w,
                                               const double* d, const int32_t* F,
                                               const int32_t* E, const double* R, double delta) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    uint64_t amax = 0, lb = 0, top = 0, bad = 0;
    if (i < S.NL) {
        /* the per-job checks of sw_validate_problem, on the device: device-
         * resident inputs (sw_dist_plan_solve_dev) never visit the host */
        const double pj = S.p[i];
        bad = w[i] < 1 || E[i] < 1 || F[i] < 0 || F[i] > E[i] || (w[i] <= S.G && w[i] > SW_MAX_WIDTH) ||
              !(d[i] > 0.0) || !(d[i] < 1e308) || !(R[i] == R[i] && R[i] < 1e308 && R[i] > -1e308) ||
              !(pj >= 0.0) || !(pj < 1e308);
        if (!bad) {
            const sw_jobc c = sw_make_jobc((int32_t)S.N, S.T, delta, w[i], d[i], F[i], E[i], R[i], pj);
            jc[i] = c;
            amax = sw_bits(c.a); /* a, g ≥ 0: bit order = value order */
            lb = sw_bits(sw_g(&c, tj_of(S, c)));
            top = sw_bits(sw_g(&c, 0));
        }
    }
    red_umax(S.red + 0, amax);
    red_umax(S.red + 1, lb);
    red_umax(S.red + 2, bad);
    red_umax(S.red + 3, top);
    pub_tail(S);
}

/* key rows (twin: build), A read from the all-reduced step result */
/* one wave per job, lane n = the job's (n+1)-th round: f(n + 1) − f(n) per
 * lane, the running minimum over n as a wave prefix-min scan (min is exact,
 * so any scan order gives the sequential loop's values), the fp32 keys
 * stored coalesced.  (A thread per job walked its 30 rounds in sequence:
 * 16 µs per C4 solve, the job loop spread over only NL / 256 workgroups.) */
/* fc (fast_solve): thread 0 of block 0 also sets up the level search
 * (k_fast_lvl_init's work, from the same setup result) */
__device__ void fast_lvl_init(FastCtl* c, const long long* R0, unsigned long long* sr, long long C, double k);
__global__ __launch_bounds__(kTB) void k_keys(ShardDev S, FastCtl* fc = nullptr, unsigned long long* sr = nullptr,
                                             long long C = 0, double kk = 0.0) {
    if (fc && blockIdx.x == 0 && threadIdx.x == 0) fast_lvl_init(fc, S.red, sr, C, kk);
    const int64_t i = ((int64_t)blockIdx.x * kTB + threadIdx.x) >> 6;
    if (i >= S.NL) return; /* uniform over the wave */
    const int n = lane_id();
    const double A = sw_from_bits((uint64_t)S.red[0]);
    const sw_jobc c = S.jc[i];
    const double ks = sw_key_scale(c.w, A);
    double v = 0.0;
    if (n < S.T) {
        const double prev = sw_f(&c, n, S.nb, S.beta, S.ell, S.slope);
        const double cur = sw_f(&c, n + 1, S.nb, S.beta, S.ell, S.slope);
        v = sw_pos(cur - prev);
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double u = __shfl_up(v, o, 64);
        if (n >= o) v = sw_min(u, v);
    }
    if (n < S.T) S.keys[(size_t)i * S.T + n] = sw_key(v, ks);
}

/* ---- SELECT steps ----------------------------------------------------------- */

struct FastCtl;
__device__ void fast_price_init(FastCtl* c, long long Wf, long long Wall, unsigned long long Mbits,
                                unsigned long long* sp);

/* Mdev (fast_solve): M = the level search's answer, its state's lo bits.
 * fpi (fast_solve at world 1, where the force's sums need no collective):
 * the last block to finish also sets up the price search (k_fast_price_init's
 * work, one launch fewer) */
__global__ __launch_bounds__(kTB) void k_force(ShardDev S, double M, int is_inf,
                                               const unsigned long long* Mdev = nullptr, SearchTail st = {},
                                               FastCtl* fpi = nullptr, unsigned long long* sp = nullptr) {
    if (st.x) M = sw_from_bits(search_tail(st));
    else if (Mdev) M = sw_from_bits(Mdev[0]);
    const int i = blockIdx.x * kTB + threadIdx.x;
    long long wf = 0, wall = 0;
    if (i < S.NL) {
        const sw_jobc c = S.jc[i];
        const int tj = tj_of(S, c);
        const int l = is_inf ? 0 : g_count_gt(c, tj, M);
        S.l[i] = l;
        wf = (long long)c.w * l;
        wall = (long long)c.w * (tj - l);
    }
    red_add(S.red + 0, wf);
    red_add(S.red + 1, wall);
    if (fpi) { /* uniform: a kernel argument */
        __shared__ int last_;
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0)
            last_ = atomicAdd((unsigned long long*)(S.red + kRedCtr), 1ull) == (unsigned long long)(gridDim.x - 1);
        __syncthreads();
        if (last_ && threadIdx.x == 0) {
            __threadfence();
            const long long Wf = __hip_atomic_load(S.red + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const long long Wall = __hip_atomic_load(S.red + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            fast_price_init(fpi, Wf, Wall, sw_bits(M), sp);
        }
        return;
    }
    pub_tail(S);
}

/* K probes at once: item (job, n) adds w to bin #{m : thr_m < v(n)} (v =
 * the key, or g for the level probes); the count for probe m is the suffix
 * Σ_{b > m} bin[b].  Bin 0 holds only the items at or above the bracket's
 * lower end lob, so Σ_b bin[b] is that end's count (sw_shard_ops.count_gt's
 * out[K]).  Thread per item: the whole grid is busy. */
template <bool LEVEL>
__device__ __forceinline__ void probe_body(const ShardDev& S, const uint64_t* thr, int K, uint64_t lob,
                                           int32_t* bins) {
    /* grid-stride over the items (NL·T < 2^31): a bounded grid keeps the
     * block → global flush at ≤ kProbeBlocks·K atomics per probe */
    const int items = S.NL * S.T;
    int32_t wtop = 0; /* items above every threshold: wave-summed, one atomic per wave */
    for (int e = (int)blockIdx.x * kTB + (int)threadIdx.x; e < items; e += (int)gridDim.x * kTB) {
        const int i = e / S.T, n = e - i * S.T;
        const int32_t w = S.jc[i].w;
        const int tj = w <= S.G ? S.T : 0;
        bool live;
        int lo = 0, hi = K;
        uint64_t vb = 0;
        if (LEVEL) {
            live = n < tj;
            if (live) {
                const sw_jobc c = S.jc[i];
                const double v = sw_g(&c, n);
                vb = sw_bits(v);
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (sw_from_bits(thr[mid]) < v) lo = mid + 1; else hi = mid;
                }
            }
        } else {
            live = n >= S.l[i] && n < tj;
            if (live) {
                const uint32_t b = sw_fbits_of(S.keys[(size_t)i * S.T + n]);
                vb = b;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if ((uint32_t)thr[mid] < b) lo = mid + 1; else hi = mid;
                }
            }
        }
        if (live && lo == K) wtop += w;
        else if (live && (lo > 0 || vb >= lob)) atomicAdd(&bins[lo], w);
    }
    wtop = wave_sum_i32(wtop);
    if (lane_id() == 0 && wtop != 0) atomicAdd(&bins[K], wtop);
    __syncthreads();
    if (threadIdx.x <= K && bins[threadIdx.x] != 0)
        atomicAdd((unsigned long long*)(S.red + threadIdx.x), (unsigned long long)bins[threadIdx.x]);
}

/* thresholds given by the host (controller-driven search step) */
template <bool LEVEL>
__global__ __launch_bounds__(kTB) void k_probe(ShardDev S, Thresholds th) {
    __shared__ int32_t bins[SW_SHARD_K + 1];
    __shared__ uint64_t thr[SW_SHARD_K];
    if (threadIdx.x <= SW_SHARD_K) bins[threadIdx.x] = 0;
    if (threadIdx.x < th.K) thr[threadIdx.x] = th.v[threadIdx.x];
    __syncthreads();
    probe_body<LEVEL>(S, thr, th.K, th.lo, bins);
}

/* ---- device-chained K-ary search (op_search) ---------------------------------
 * The controller's swc_search loop (sw_shard_ctl.h) with its state in device
 * memory: sr[0] = lo, sr[1] = hi, sr[2] = budget (i64), sr[3] = rounds taken,
 * sr[4] = clo = Σ w·#{v ≥ lo}, sr[5] = chi = Σ w·#{v > hi} (−1: unknown),
 * kSt words per state.  Each round is k_probe_dev → (collectives) → the step
 * applied in the next round's kernel (or k_search_update after the last),
 * with no host round trip.  A round's kind follows from its state
 * (sw_search_mode): probe K thresholds into bins, or gather the bracket's
 * items into the rank's list (SW_GATHER_CAP pairs), whose step resolves the
 * answer; a closed bracket does nothing, so the host enqueues a bound on the
 * rounds. */
constexpr int kSt = 8;                            /* words of a search state */
constexpr int kGl = 2 * (SW_GATHER_CAP + 1);      /* words of a rank's item list: count, pad, (v, w) pairs */
/* rounds fast_solve enqueues per search: C4's level search closes in two (a
 * probe, a gather), its price search in three (two probes, a gather); a
 * search still open after them sends the solve to the host path */
constexpr int kFastRounds = 3;
struct SearchPts {
    int32_t K;
    uint64_t a, b, d;
};
__device__ __forceinline__ SearchPts search_pts(uint64_t lo, uint64_t hi) {
    SearchPts q;
    const uint64_t span = hi - lo;
    q.K = lo >= hi ? 0 : (span < (uint64_t)SW_SHARD_K ? (int32_t)span : SW_SHARD_K);
    q.d = (uint64_t)q.K + 1u;
    q.a = lo >= hi ? 0 : span / q.d;
    q.b = lo >= hi ? 0 : span % q.d;
    return q;
}
__device__ __forceinline__ uint64_t search_pt(uint64_t lo, const SearchPts& q, int i) {
    const uint64_t m = (uint64_t)(i + 1);
    return lo + q.a * m + (q.b * m) / q.d;
}
__device__ __forceinline__ int search_mode(const unsigned long long* x) {
    return sw_search_mode(x[0], x[1], (int64_t)x[4], (int64_t)x[5]);
}

__global__ void k_search_init(unsigned long long* sr, unsigned long long lo, unsigned long long hi,
                              long long bud, long long chi) {
    if (threadIdx.x == 0) {
        sr[0] = lo; sr[1] = hi; sr[2] = (unsigned long long)bud; sr[3] = 0;
        sr[4] = ~0ull; sr[5] = (unsigned long long)chi; sr[6] = 0; sr[7] = 0;
    }
}

/* One probe step of swc_search on a state x from the all-reduced bins of the
 * round that probed it: counts cnt[i] = Σ_{b > i} bins[b]; the first i with
 * cnt ≤ budget closes the bracket, whose ends keep their counts.  One wave:
 * lane i loads bins[i + 1], a shuffle suffix scan forms cnt[i], a ballot
 * finds the first i.  Returns the new state in lane 0's out. */
__device__ __forceinline__ void search_step_wave(const unsigned long long* x, const long long* bins,
                                                 unsigned long long* out) {
    constexpr int PL = (SW_SHARD_K + 63) / 64; /* thresholds per lane: i = PL·lane + j */
    const uint64_t lo = x[0], hi = x[1];
    const int64_t bud = (int64_t)x[2];
    const SearchPts q = search_pts(lo, hi);
    const int lane = lane_id();
    if (q.K == 0) {
        if (lane < kSt) out[lane] = x[lane];
        return;
    }
    /* cnt[i] = Σ_{b > i} bins[b]: each lane's suffix over its PL bins, then
     * an exclusive suffix scan of the lane totals (the same integers) */
    int64_t c[PL];
    int64_t tot = 0;
#pragma unroll
    for (int j = PL - 1; j >= 0; --j) {
        const int i = PL * lane + j;
        tot += (i < q.K) ? (int64_t)bins[i + 1] : 0;
        c[j] = tot;
    }
    int64_t after = tot; /* Σ over the lanes above this one, by a shuffle suffix scan */
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t v = __shfl_down(after, o, 64);
        after += (lane + o < 64) ? v : 0;
    }
    after -= tot;
    int fj = PL;
#pragma unroll
    for (int j = PL - 1; j >= 0; --j)
        if (PL * lane + j < q.K && c[j] + after <= bud) fj = j;
    const uint64_t ok = __ballot(fj < PL);
    const int fl = ok ? __builtin_ctzll(ok) : 0;
    const int f = ok ? PL * fl + __shfl(fj, fl, 64) : q.K;
    /* the counts at the new ends: cnt[f] (f < K) and cnt[f − 1] (f > 0) */
    auto cnt_at = [&](int i) -> int64_t {
        const int jj = i % PL;
        int64_t v = after;
#pragma unroll
        for (int j = 0; j < PL; ++j) v += (j == jj) ? c[j] : 0;
        return __shfl(v, i / PL, 64);
    };
    const int64_t chi_n = f < q.K ? cnt_at(f) : (int64_t)x[5];
    const int64_t clo_n = f > 0 ? cnt_at(f - 1) : cnt_at(0) + (int64_t)bins[0]; /* lo stays: bin 0 + cnt[0] */
    if (lane == 0) {
        uint64_t nlo = lo, nhi = hi;
        if (f < q.K) {
            nhi = search_pt(lo, q, f);
            if (f > 0) nlo = search_pt(lo, q, f - 1) + 1u;
        } else {
            nlo = search_pt(lo, q, q.K - 1) + 1u;
        }
        out[0] = nlo;
        out[1] = nhi;
        out[2] = x[2];
        out[3] = x[3] + 1;
        out[4] = (unsigned long long)clo_n;
        out[5] = (unsigned long long)chi_n;
        out[6] = 0;
        out[7] = 0;
    }
}

/* The gather step of a state x (mode 2): the items of every rank's list
 * (lists: W blocks of kGl words, rank order) resolve the answer as
 * sw_search_resolve does — each item's sum over all items, then a minimum —
 * by the whole block; the closed state into out (block-shared, kSt words).
 * sm: ≥ 2·SW_GATHER_CAP + 2 words of shared scratch. */
__device__ void search_resolve_block(const unsigned long long* x, const unsigned long long* lists, int W,
                                     unsigned long long* out, unsigned long long* sm) {
    unsigned long long* rv = sm;
    long long* rw = reinterpret_cast<long long*>(sm + SW_GATHER_CAP);
    __shared__ int rn;
    __shared__ unsigned long long rbest;
    __shared__ long long rslo;
    const uint64_t lo = x[0], hi = x[1];
    const long long bud = (long long)x[2], chi = (long long)x[5];
    if (threadIdx.x == 0) { rn = 0; rbest = hi; rslo = 0; }
    __syncthreads();
    int base = 0;
    for (int r = 0; r < W; ++r) { /* the lists' counts are uniform loads */
        const unsigned long long* L = lists + (size_t)r * kGl;
        int c = (int)L[0];
        c = c < SW_GATHER_CAP - base ? c : SW_GATHER_CAP - base; /* ≤ the cap by the mode's rule */
        for (int e = threadIdx.x; e < c; e += blockDim.x) {
            rv[base + e] = L[2 + 2 * e];
            rw[base + e] = (long long)L[3 + 2 * e];
        }
        base += c;
    }
    __syncthreads();
    const int n = base;
    unsigned long long best = hi;
    long long slo = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const unsigned long long vi = rv[i];
        long long si = chi;
        for (int k = 0; k < n; ++k) si += rv[k] > vi ? rw[k] : 0;
        if (si <= bud && vi < best) best = vi;
        slo += vi > lo ? rw[i] : 0;
    }
    best = wave_min_u64(best);
    slo = wave_sum(slo);
    if (lane_id() == 0) {
        atomicMin(&rbest, best);
        if (slo) atomicAdd((unsigned long long*)&rslo, (unsigned long long)slo);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long b = rbest;
        if (chi + rslo <= bud) b = lo; /* lo ≤ every item */
        out[0] = b;
        out[1] = b;
        out[2] = x[2];
        out[3] = x[3] + 1;
        out[4] = ~0ull;
        out[5] = ~0ull;
        out[6] = 0;
        out[7] = 0;
    }
    __syncthreads();
}

/* The step of the round that ran on state x (its bins / its gathered lists)
 * into out (block-shared), by the whole block. */
__device__ __forceinline__ void search_step_block(const unsigned long long* x, const long long* bins,
                                                  const unsigned long long* lists, int W, unsigned long long* out,
                                                  unsigned long long* sm) {
    const int m = search_mode(x);
    if (m == 2) {
        search_resolve_block(x, lists, W, out, sm);
        return;
    }
    if (threadIdx.x < 64) {
        if (m == 1) search_step_wave(x, bins, out);
        else if (threadIdx.x < kSt) out[threadIdx.x] = x[threadIdx.x];
    }
    __syncthreads();
}

/* Items of the bracket [lo, hi] into this rank's list gl (count at gl[0];
 * pairs beyond the cap are counted, not stored). */
template <bool LEVEL>
__device__ __forceinline__ void gather_body(const ShardDev& S, uint64_t lo, uint64_t hi, unsigned long long* gl) {
    const int items = S.NL * S.T;
    for (int e = (int)blockIdx.x * kTB + (int)threadIdx.x; e < items; e += (int)gridDim.x * kTB) {
        const int i = e / S.T, n = e - i * S.T;
        const int32_t w = S.jc[i].w;
        const int tj = w <= S.G ? S.T : 0;
        uint64_t v = 0;
        bool in = false;
        if (LEVEL) {
            if (n < tj) {
                const sw_jobc c = S.jc[i];
                v = sw_bits(sw_g(&c, n));
                in = v >= lo && v <= hi;
            }
        } else if (n >= S.l[i] && n < tj) {
            v = sw_fbits_of(S.keys[(size_t)i * S.T + n]);
            in = v >= lo && v <= hi;
        }
        if (in) {
            const unsigned long long k = atomicAdd(gl, 1ull);
            if (k < (unsigned long long)SW_GATHER_CAP) {
                gl[2 + 2 * k] = v;
                gl[3 + 2 * k] = (unsigned long long)(long long)w;
            }
        }
    }
}

/* Round r of the chained search: first the step of round r − 1 (its state
 * xin, its all-reduced bins prev or its gathered lists gprev) — every block
 * computes it, block 0 stores the result in xout — then this round on the
 * new state: K probes into S.red, or the bracket's items into gl.  Fusing
 * the step into the next round saves a kernel launch per round; round 0
 * passes prev = nullptr and runs on xin as it is. */
template <bool LEVEL>
__global__ __launch_bounds__(kTB) void k_probe_dev(ShardDev S, const unsigned long long* xin,
                                                   unsigned long long* xout, const long long* prev,
                                                   unsigned long long* gl, const unsigned long long* gprev, int W) {
    __shared__ int32_t bins[SW_SHARD_K + 1];
    __shared__ unsigned long long sm[2 * SW_GATHER_CAP]; /* the resolve's items, then the thresholds */
    __shared__ unsigned long long xs[kSt];
    if (prev == nullptr) {
        if (threadIdx.x < kSt) xs[threadIdx.x] = xin[threadIdx.x];
        __syncthreads();
    } else {
        search_step_block(xin, prev, gprev, W, xs, sm);
    }
    if (prev != nullptr && blockIdx.x == 0 && threadIdx.x < kSt) xout[threadIdx.x] = xs[threadIdx.x];
    const int mode = search_mode(xs);
    if (mode == 0) return; /* bracket closed: uniform over the grid */
    const uint64_t lo = xs[0], hi = xs[1];
    if (mode == 2) {
        gather_body<LEVEL>(S, lo, hi, gl);
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) gl[0] = 0; /* a later gather round appends from 0 */
    const SearchPts q = search_pts(lo, hi);
    uint64_t* thr = reinterpret_cast<uint64_t*>(sm);
    if (threadIdx.x <= SW_SHARD_K) bins[threadIdx.x] = 0;
    if ((int)threadIdx.x < q.K) {
        const uint64_t v = search_pt(lo, q, (int)threadIdx.x);
        thr[threadIdx.x] = LEVEL ? v : (uint64_t)(uint32_t)v; /* price bits are u32 */
    }
    __syncthreads();
    probe_body<LEVEL>(S, thr, q.K, lo, bins);
}

/* the last round's step, in place (one block) */
__global__ __launch_bounds__(kTB) void k_search_update(unsigned long long* sr, const long long* bins,
                                                      const unsigned long long* lists, int W, ShardDev S) {
    __shared__ unsigned long long sm[2 * SW_GATHER_CAP];
    __shared__ unsigned long long xs[kSt];
    search_step_block(sr, bins, lists, W, xs, sm);
    if (threadIdx.x < kSt) sr[threadIdx.x] = xs[threadIdx.x];
    if (S.pub.dst) { /* the state to the host (fused publish) */
        __threadfence();
        __syncthreads();
        pub_store(S);
    }
}

__device__ uint64_t search_tail(const SearchTail& t) {
    __shared__ unsigned long long sm[2 * SW_GATHER_CAP];
    __shared__ unsigned long long xs[kSt];
    search_step_block(t.x, t.bins, t.lists, t.W, xs, sm);
    if (blockIdx.x == 0 && threadIdx.x < kSt) t.xo[threadIdx.x] = xs[threadIdx.x];
    return xs[0];
}

/* The width tail of SELECT at world 1 (swc_select's loop: while room is
 * left, the job whose next key is largest among those that fit — key << 32 |
 * ~job, k_tail_best's order — takes one more round), by one workgroup over
 * every job, before the SELECT evaluation.  fc->tail_steps = the steps the
 * controller counts: one per tail_best, plus the widths' gather on the first
 * round taken. */
constexpr int kTailTB = 1024;
__global__ __launch_bounds__(kTailTB) void k_fast_tail(ShardDev S, FastCtl* fc, const long long* R3) {
    __shared__ unsigned long long wb[kTailTB / 64];
    __shared__ unsigned long long bb;
    const int tid = threadIdx.x;
    if (fc->all || fc->escape) { /* uniform */
        if (tid == 0) fc->tail_steps = 0;
        return;
    }
    long long rem2 = fc->rem - R3[0];
    int steps = 0, took = 0;
    while (rem2 > 0) {
        unsigned long long best = 0;
        for (int i = tid; i < S.NL; i += kTailTB) {
            const sw_jobc c = S.jc[i];
            const int n = S.arr[SW_A_N][i];
            if (n < tj_of(S, c) && (long long)c.w <= rem2) {
                const unsigned long long kk = ((unsigned long long)sw_fbits_of(S.keys[(size_t)i * S.T + n]) << 32) |
                                              (unsigned long long)(0xFFFFFFFFu - (uint32_t)(S.off + i));
                best = kk > best ? kk : best;
            }
        }
        best = wave_max(best);
        if (lane_id() == 0) wb[wave_id()] = best;
        __syncthreads();
        if (tid == 0) {
            unsigned long long b = 0;
            for (int w = 0; w < kTailTB / 64; ++w) b = wb[w] > b ? wb[w] : b;
            bb = b;
        }
        __syncthreads();
        best = bb;
        ++steps;
        if (best == 0) break; /* uniform */
        const int jb = (int)((long long)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFu)) - S.off);
        if (tid == 0) S.arr[SW_A_N][jb] += 1;
        rem2 -= S.jc[jb].w;
        took = 1;
        __syncthreads(); /* the count is read by every thread next step */
    }
    if (tid == 0) fc->tail_steps = steps + took;
}

/* the items of [lo, hi] into gl alone (op_gather) */
template <bool LEVEL>
__global__ __launch_bounds__(kTB) void k_gather(ShardDev S, uint64_t lo, uint64_t hi, unsigned long long* gl) {
    gather_body<LEVEL>(S, lo, hi, gl);
}

/* c (fast_solve): the interval (M_lo, M_lo + wmax] of FastCtl, nothing to
 * count when wmax ≤ 0 */
__global__ __launch_bounds__(kTB) void k_between(ShardDev S, double a, double b, const FastCtl* c = nullptr) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    long long cnt = 0;
    bool run = true;
    if (c) {
        a = c->M_lo;
        b = c->bmax;
        run = c->did_between != 0;
    }
    if (c && i < S.NL) S.arr[SW_A_NB][i] = S.arr[SW_A_N][i]; /* fast_solve: swc_level_search's copy */
    if (run && i < S.NL) {
        const sw_jobc c = S.jc[i];
        const int n1 = tj_of(S, c) + 1;
        const int d = g_count_gt(c, n1, a) - g_count_ge(c, n1, b);
        cnt = d > 0 ? d : 0;
    }
    red_add(S.red + 0, cnt);
    pub_tail(S);
}

__global__ __launch_bounds__(kTB) void k_take_all(ShardDev S) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    if (i >= S.NL) return;
    const int tj = tj_of(S, S.jc[i]);
    S.arr[SW_A_N][i] = tj;
    S.taken[i] = tj - S.l[i];
}

/* rdev / fc (fast_solve): ρ = the price search's answer; when every item
 * fits (fc->all) the step is k_take_all's (n := T_j, taken := T_j − l) */
__global__ __launch_bounds__(kTB) void k_take(ShardDev S, uint32_t rho, const unsigned long long* rdev = nullptr,
                                              const FastCtl* fc = nullptr, SearchTail st = {}) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    if (st.x) rho = (uint32_t)search_tail(st);
    else if (rdev) rho = (uint32_t)rdev[0];
    const bool all = fc && fc->all;
    long long wt = 0, tie = 0;
    if (i < S.NL) {
        const sw_jobc c = S.jc[i];
        const int tj = tj_of(S, c), l = S.l[i];
        const float* row = S.keys + (size_t)i * S.T;
        const int tk = all ? tj - l : key_count<false>(row, l, tj, rho);
        S.taken[i] = tk;
        wt = (long long)c.w * tk;
        tie = all ? 0 : (long long)c.w * (key_count<true>(row, l, tj, rho) - tk);
        S.tie[i] = (int32_t)tie;
        if (all) S.arr[SW_A_N][i] = tj;
    }
    red_add(S.red + 0, wt);
    red_add(S.red + 1, tie);
    /* this block's tie weight, for k_assign's block offsets */
    __shared__ long long ws[kTB / 64];
    const long long bt = wave_sum(tie);
    if (lane_id() == 0) ws[wave_id()] = bt;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long s = 0;
        for (int w = 0; w < kTB / 64; ++w) s += ws[w];
        S.tieblk[blockIdx.x] = s;
    }
    pub_tail(S);
}

/* tie group in job order (twin: the excl loop of select_level): thread per
 * job, the grid of k_take.  Block b's offset is excl0 plus the tie weights
 * k_take summed for blocks 0 … b−1, then a block scan: the same integer
 * prefix as a walk over the jobs in order, without one workgroup walking
 * them all. */
/* fc / g (fast_solve): rem = bud − Σ_ranks wt and excl0 = Σ of the tie
 * weights of the ranks before this one, from k_take's gathered results g
 * (2 per rank); nothing to assign when every item fits */
__global__ __launch_bounds__(kTB) void k_assign(ShardDev S, long long rem, long long excl0,
                                                FastCtl* fc = nullptr, const long long* g = nullptr,
                                                int world = 1) {
    if (fc) {
        if (fc->all) return; /* used = 0 (the zeroed step slot) */
        long long wt = 0, ex = 0;
        for (int r = 0; r < world; ++r) {
            wt += g[2 * r];
            if (r < S.rank) ex += g[2 * r + 1];
        }
        rem = fc->bud - wt;
        excl0 = ex;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            fc->wt = wt;
            fc->rem = rem;
        }
    }
    __shared__ long long ws[kTB / 64];
    __shared__ long long boff;
    long long pb = 0;
    for (int b = (int)threadIdx.x; b < (int)blockIdx.x; b += kTB) pb += S.tieblk[b];
    pb = wave_sum(pb);
    if (lane_id() == 0) ws[wave_id()] = pb;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long s = excl0;
        for (int w = 0; w < kTB / 64; ++w) s += ws[w];
        boff = s;
    }
    __syncthreads();
    const int i = blockIdx.x * kTB + threadIdx.x;
    const long long t = i < S.NL ? (long long)S.tie[i] : 0;
    const long long inc = wave_incscan(t);
    if (lane_id() == 63) ws[wave_id()] = inc;
    __syncthreads();
    long long before = boff;
    for (int w = 0; w < wave_id(); ++w) before += ws[w];
    long long used = 0;
    if (i < S.NL) {
        const long long excl = before + inc - t;
        const long long wj = S.jc[i].w;
        const int tie = (int)(t / wj);
        int tt;
        if (excl + t <= rem) tt = tie;
        else if (excl <= rem) tt = (int)((rem - excl) / wj);
        else tt = 0;
        S.arr[SW_A_N][i] = S.l[i] + S.taken[i] + tt;
        used = wj * tt;
    }
    red_add(S.red + 0, used);
    pub_tail(S);
}

__global__ __launch_bounds__(kTB) void k_tail_best(ShardDev S, long long rem2) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    uint64_t best = 0;
    if (i < S.NL) {
        const sw_jobc c = S.jc[i];
        const int n = S.arr[SW_A_N][i];
        if (n < tj_of(S, c) && (long long)c.w <= rem2)
            best = ((uint64_t)sw_fbits_of(S.keys[(size_t)i * S.T + n]) << 32) |
                   (uint64_t)(0xFFFFFFFFu - (uint32_t)(S.off + i));
    }
    red_umax(S.red + 0, best);
}

__global__ void k_tail_apply(ShardDev S, int i) { S.arr[SW_A_N][i] += 1; }

/* raises (sw_shard_ops.raise_stats): red[0] = ~ the first global job with
 * g(nfin) = M (max of ~index; 0 if none here), red[1] = #{g = M}, red[2] =
 * max bits of {g < M}, red[3] = max bits of g (g ≥ 0: bits order as
 * values), red[4] = Σ w·nfin */
__global__ __launch_bounds__(kTB) void k_raise_stats(ShardDev S, double M) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    uint64_t first = 0, mlt = 0, mall = 0;
    long long cnt = 0, load = 0;
    if (i < S.NL) {
        const sw_jobc c = S.jc[i];
        const int n = S.arr[SW_A_NFIN][i];
        const double g = sw_g(&c, n);
        if (g == M) {
            first = ~(uint64_t)(S.off + i);
            cnt = 1;
        } else if (g < M) {
            mlt = sw_bits(g);
        }
        mall = sw_bits(g);
        load = (long long)c.w * n;
    }
    red_umax(S.red + 0, first);
    red_add(S.red + 1, cnt);
    red_umax(S.red + 2, mlt);
    red_umax(S.red + 3, mall);
    red_add(S.red + 4, load);
    pub_tail(S);
}

/* raises (sw_shard_ops.raise_best): the best untried candidate's key */
struct RaiseTried {
    long long j[SW_RAISE_TRIES];
    int n;
};
__global__ __launch_bounds__(kTB) void k_raise_best(ShardDev S, double M, long long i1, double M2, RaiseTried rt) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    uint64_t key = 0;
    if (i < S.NL) {
        const sw_jobc c = S.jc[i];
        const int n = S.arr[SW_A_NFIN][i];
        const long long j = S.off + i;
        bool skip = n >= tj_of(S, c);
        for (int q = 0; q < rt.n; ++q) skip |= rt.j[q] == j;
        if (!skip) {
            const double Mo = j == i1 ? M2 : M;
            key = sw_fill_key(sw_raise_gain(sw_f(&c, n, S.nb, S.beta, S.ell, S.slope),
                                            sw_f(&c, n + 1, S.nb, S.beta, S.ell, S.slope), sw_g(&c, n + 1), Mo, M,
                                            S.k),
                              j, 0);
        }
    }
    red_umax(S.red, key);
    pub_tail(S);
}

/* fill of stranded capacity (sw_shard_ops.fill_best / fill_apply) */
struct FillLoad {
    long long v[SW_TMAX]; /* GPUs in use per round, all ranks */
};

__global__ __launch_bounds__(kTB) void k_fill_best(ShardDev S, FillLoad L) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    uint64_t best = 0;
    if (i < S.NL) {
        const sw_jobc c = S.jc[i];
        const int n = S.arr[SW_A_NFIN][i];
        if (n < tj_of(S, c)) {
            const uint64_t m = S.y[SW_Y_BEST][i];
            int tf = -1;
            for (int t = 0; t < S.T; ++t)
                if (!((m >> t) & 1ull) && (long long)c.w <= (long long)S.G - L.v[t]) { tf = t; break; }
            if (tf >= 0)
                best = sw_fill_key(sw_f(&c, n + 1, S.nb, S.beta, S.ell, S.slope) -
                                       sw_f(&c, n, S.nb, S.beta, S.ell, S.slope),
                                   S.off + i, tf);
        }
    }
    red_umax(S.red + 0, best);
}

__global__ void k_fill_apply(ShardDev S, int i, int t) {
    S.y[SW_Y_BEST][i] |= 1ull << t;
    S.arr[SW_A_NFIN][i] += 1;
}

/* ---- reductions with deterministic lane sums ------------------------------- */

/* A reduction step in ONE kernel.  Block b owns the deterministic-sum lanes
 * [b·lpb, (b+1)·lpb) of this rank (lane ℓ sums the jobs [ℓ·q, ℓ·q + q),
 * sw_detsum's chunks): its threads compute the per-job values of those
 * lanes' jobs (thread per job) into LDS, then lpb threads sum each lane left
 * to right — so the gathered lanes reproduce the single-instance sums bit for
 * bit.  max g and the integer sum go to red[0] / red[1] by atomics; the last
 * block to finish (counter red[kRedCtr]) copies them behind the lanes.
 * out = [A lanes][B lanes][gm][isum].  SW_EV_FINAL also writes the plan row
 * and count of each job. */
/* sel = kEvSelUmax (fast_solve): SW_EV_SELECT's A, B, max g and a third
 * lane sum C = f(T_j) (SW_EV_UMAX's A) in one pass, out = [A][B][gm][isum][C] */
constexpr int kEvSelUmax = 7;
__global__ __launch_bounds__(kTB) void k_eval(ShardDev S, int sel, const int32_t* arr,
                                             const uint64_t* ysrc, int arr_a, int arr_b, int lpb,
                                             double* out) {
    __shared__ double xs[3][kTB];
    __shared__ long long wred[kTB / 64];
    __shared__ unsigned long long wmax[kTB / 64];
    __shared__ int last;
    const int64_t q = S.q;
    const int64_t lane0 = (int64_t)blockIdx.x * lpb;
    const int64_t i = lane0 * q + (int64_t)threadIdx.x; /* local job of this thread */
    double fa = 0.0, fb = 0.0, fc = 0.0, gm = 0.0;
    long long is = 0;
    if ((int64_t)threadIdx.x < (int64_t)lpb * q && i < S.NL) {
        const sw_jobc c = S.jc[i];
        if (sel == SW_EV_SELECT || sel == kEvSelUmax) {
            const int n = S.arr[SW_A_N][i];
            fa = sw_f(&c, n, S.nb, S.beta, S.ell, S.slope);
            fb = sw_f(&c, S.l[i] + S.taken[i], S.nb, S.beta, S.ell, S.slope);
            gm = sw_g(&c, n);
            if (sel == kEvSelUmax) fc = sw_f(&c, tj_of(S, c), S.nb, S.beta, S.ell, S.slope);
        } else if (sel == SW_EV_GMAX) {
            gm = sw_g(&c, arr[i]);
        } else if (sel == SW_EV_PACKED) {
            const int pl = arr[i];
            fa = sw_f(&c, pl, S.nb, S.beta, S.ell, S.slope);
            gm = sw_g(&c, pl);
            is = (long long)c.w * (S.arr[SW_A_NB][i] - pl);
        } else if (sel == SW_EV_P2OK) {
            is = S.arr[SW_A_PL][i] != S.arr[SW_A_NFIN][i];
        } else if (sel == SW_EV_UNPLACED) {
            is = S.arr[arr_a][i] != S.arr[arr_b][i];
        } else if (sel == SW_EV_UMAX) {
            fa = sw_f(&c, tj_of(S, c), S.nb, S.beta, S.ell, S.slope);
        } else { /* SW_EV_FINAL */
            const uint64_t m = ysrc[i];
            const int cn = __popcll(m);
            long long Ssum = 0;
            uint8_t* row = S.plan + (size_t)i * S.T;
            for (int t = 0; t < S.T; ++t) {
                const uint32_t bit = (uint32_t)((m >> t) & 1ull);
                Ssum += bit ? t : 0;
                row[t] = (uint8_t)bit;
            }
            S.planned[i] = cn;
            fa = sw_f(&c, cn, S.nb, S.beta, S.ell, S.slope);
            fb = cn > 0 ? ((double)Ssum / (double)cn) * S.p[i] : 0.0;
            gm = sw_g(&c, cn);
            is = cn > 0;
        }
    }
    xs[0][threadIdx.x] = fa;
    xs[1][threadIdx.x] = fb;
    xs[2][threadIdx.x] = fc;
    /* block max / sum, one atomic each per block */
    const unsigned long long gb = wave_max((unsigned long long)sw_bits(gm)); /* g ≥ 0: bit order = value order */
    const long long sb = wave_sum(is);
    if (lane_id() == 0) { wmax[wave_id()] = gb; wred[wave_id()] = sb; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = 0;
        long long t = 0;
        for (int w = 0; w < kTB / 64; ++w) { m = wmax[w] > m ? wmax[w] : m; t += wred[w]; }
        if (m) atomicMax((unsigned long long*)(S.red + 0), m);
        if (t) atomicAdd((unsigned long long*)(S.red + 1), (unsigned long long)t);
    }
    /* lane sums, left to right over the lane's jobs present on this rank */
    const int64_t lane = lane0 + (int64_t)threadIdx.x;
    if ((int)threadIdx.x < lpb && lane < S.LW) {
        const int64_t jb = lane * q, je = min((int64_t)S.NL, jb + q);
        double a = 0.0, b = 0.0, cc = 0.0;
        for (int64_t j = jb; j < je; ++j) {
            a = a + xs[0][j - lane0 * q];
            b = b + xs[1][j - lane0 * q];
            cc = cc + xs[2][j - lane0 * q];
        }
        out[lane] = a;
        out[S.LW + lane] = b;
        if (sel == kEvSelUmax) out[2 * S.LW + 2 + lane] = cc;
    }
    /* the last block publishes max g and the sum behind the lanes */
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0)
        last = atomicAdd((unsigned long long*)(S.red + kRedCtr), 1ull) == (unsigned long long)(gridDim.x - 1);
    __syncthreads();
    if (last && threadIdx.x == 0) {
        __threadfence();
        const unsigned long long g = __hip_atomic_load((unsigned long long*)(S.red + 0), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t = __hip_atomic_load((unsigned long long*)(S.red + 1), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
        out[2 * S.LW] = sw_from_bits(g);
        reinterpret_cast<long long*>(out)[2 * S.LW + 1] = (long long)t;
    }
    if (last && S.pub.dst) { /* the lanes and the two results to the host */
        __threadfence();
        __syncthreads();
        pub_store(S);
    }
}

/* ---- device-side control of the common path (fast_solve) -------------------------
 * One-wave kernels between the step kernels: each takes the controller's
 * decisions (sw_shard_ctl.h) from the step results in device memory, so the
 * host enqueues the whole solve and reads one result. */

/* sw_shard_tree on one wave: lane l holds lane 64·w + l of chunk w (lane
 * partial ℓ of the gathered eval blocks: rank ℓ / LW, offset ℓ mod LW), each
 * chunk halved by shuffles (p[i] + p[i + h], the same operands as the host
 * loop), then the eight chunk sums by the same halving.  Wave-uniform result. */
__device__ __forceinline__ double wave_tree512(const double* blocks, int blk, int LW, int off) {
    const int lane = lane_id();
    double ws[SW_DET_LANES / 64];
#pragma unroll
    for (int w = 0; w < SW_DET_LANES / 64; ++w) {
        const int idx = 64 * w + lane, r = idx / LW, o = idx - r * LW;
        double v = blocks[(size_t)r * blk + (size_t)off + o];
#pragma unroll
        for (int h = 32; h >= 1; h >>= 1) v = v + __shfl_down(v, h, 64);
        ws[w] = __shfl(v, 0, 64);
    }
#pragma unroll
    for (int h = SW_DET_LANES / 128; h >= 1; h >>= 1)
#pragma unroll
        for (int i = 0; i < h; ++i) ws[i] = ws[i] + ws[i + h];
    return ws[0];
}

/* max g and Σ isum over the gathered eval blocks (op_eval's host loop) */
__device__ __forceinline__ void blocks_gm_isum(const double* blocks, int blk, int LW, int W, double& gm,
                                               long long& is) {
    gm = 0.0;
    is = 0;
    for (int r = 0; r < W; ++r) {
        const double* b = blocks + (size_t)r * blk;
        gm = sw_max(gm, b[2 * LW]);
        is += reinterpret_cast<const long long*>(b)[2 * LW + 1];
    }
}

/* after setup: the level search's bracket [lb, top) and budget C */
__device__ void fast_lvl_init(FastCtl* c, const long long* R0, unsigned long long* sr, long long C, double k) {
    FastCtl z;
    memset(&z, 0, sizeof(z));
    z.C = C;
    z.k = k;
    z.A = sw_from_bits((uint64_t)R0[0]);
    z.escape = R0[2] != 0; /* invalid inputs: the host path reports them */
    *c = z;
    sr[0] = (unsigned long long)R0[1];
    sr[1] = (unsigned long long)R0[3];
    sr[2] = (unsigned long long)C;
    sr[3] = 0;
    sr[4] = ~0ull; /* clo unknown; chi = 0: no item lies above top */
    sr[5] = 0;
    sr[6] = 0;
    sr[7] = 0;
}

/* after the forcing step at M_lo (swc_select): budget, every item fits or
 * the price search's bracket [0, SW_KEY_INF_BITS) */
__device__ void fast_price_init(FastCtl* c, long long Wf, long long Wall, unsigned long long Mbits,
                                unsigned long long* sp) {
    c->M_lo = sw_from_bits(Mbits);
    if (Wf > c->C) c->escape = 1; /* not at M_lo: a guard */
    const long long bud = c->C - Wf;
    const int all = Wall <= bud || Wf > c->C;
    c->bud = bud;
    c->Wall = Wall;
    c->all = all;
    sp[0] = 0;
    sp[1] = all ? 0ull : (unsigned long long)SW_KEY_INF_BITS;
    sp[2] = (unsigned long long)bud;
    sp[3] = 0;
    sp[4] = ~0ull; /* clo unknown; chi = 0: no key lies above SW_KEY_INF_BITS */
    sp[5] = 0;
    sp[6] = 0;
    sp[7] = 0;
}
__global__ void k_fast_price_init(FastCtl* c, const long long* R1, const unsigned long long* srl,
                                  unsigned long long* sp) {
    if (threadIdx.x == 0) fast_price_init(c, R1[0], R1[1], srl[0], sp);
}

/* after the SELECT and UMAX evaluations: U, max g, the Lagrangian bound, the
 * utility optimum and the interval the level search counts next
 * (swc_select / swc_level_search); a width tail leaves the common path */
/* Every gathered view is consumed by the kernel right after its gather (the
 * peer transport's region half is rewritten two exchanges later). */
__global__ __launch_bounds__(64) void k_fast_sel_ctl(FastCtl* c, const long long* R3, const double* sel,
                                                     const unsigned long long* sp, int W, int LW) {
    const int blk = 3 * LW + 2; /* [A][B][gm][isum][C] (kEvSelUmax) */
    const double U = wave_tree512(sel, blk, LW, 0);
    const double Bt = wave_tree512(sel, blk, LW, LW);
    const double Um = wave_tree512(sel, blk, LW, 2 * LW + 2);
    if (lane_id() != 0) return;
    double gm;
    long long is;
    blocks_gm_isum(sel, blk, LW, W, gm, is);
    const int all = c->all;
    if (W > 1 && !all && c->rem - R3[0] > 0) c->escape = 1; /* the width tail above world 1: host path */
    const double rho_d = all ? 0.0 : (double)sw_float_of((uint32_t)sp[0]);
    const long long wgt = all ? c->Wall : c->wt;
    c->U = U;
    c->Mact = gm;
    c->ubound = Bt + (rho_d * c->A) * (double)(c->bud - wgt);
    c->Umax = Um;
    const double wmax = (Um - U) / c->k;
    c->did_between = wmax > 0.0;
    c->bmax = c->M_lo + wmax;
}

/* after the PACKED evaluation: rounds the share placement stranded */
__global__ __launch_bounds__(64) void k_fast_packed(FastCtl* c, const double* packed, int W, int LW) {
    if (lane_id() != 0) return;
    double gp;
    long long dfc;
    blocks_gm_isum(packed, 2 * LW + 2, LW, W, gp, dfc);
    if (dfc != 0) c->escape = 1; /* the share repair, the gathered orders: host path */
}

/* the solve's result: P1 from the level search, P2 and the plan from the
 * final evaluation (sw_shard_solve's common path), to pinned host memory
 * (words: objective, utility, makespan, p2, bound as f64; iters, status,
 * escape, transport error as i32), then the flag's release */
struct FastOut {
    double objective, utility, makespan, p2, bound;
    int32_t iters, status, escape, xerr;
};
__global__ __launch_bounds__(64) void k_fast_final(const FastCtl* c, const long long* R4,
                                                   const long long* R5, const double* fin,
                                                   const unsigned long long* srl, const unsigned long long* sp,
                                                   int W, int LW, FastOut* hout, unsigned long long* hflag,
                                                   unsigned long long hseq, const int* xerr, const long long* Rd,
                                                   int extra_iters = 0, int extra_status = 0) {
    const int blk = 2 * LW + 2;
    const double U = wave_tree512(fin, blk, LW, 0);
    const double P2 = wave_tree512(fin, blk, LW, LW);
    if (lane_id() != 0) return;
    double gm;
    long long any;
    blocks_gm_isum(fin, blk, LW, W, gm, any);
    FastOut o;
    /* 1 = the host-driven controller solves it again; 2 = only the share
     * placement stranded rounds: the host repairs the shares and the rest of
     * the path runs again on this state (fast_resume) */
    const bool other = c->escape || (c->did_between && R4 && R4[0] != 0) /* the branch and bound */
                       || srl[0] < srl[1] || (!c->all && sp[0] < sp[1]); /* a search needed more rounds */
    o.escape = other ? 1 : (Rd && Rd[0] != 0) ? 2 : 0;
    o.utility = U;
    o.p2 = P2;
    o.makespan = gm;
    o.objective = U - c->k * gm;
    o.bound = c->ubound - c->k * c->M_lo;
    int32_t st = extra_status;
    if (R5[0] > 0) st |= SW_STATUS_P2_EXCHANGED;
    if (any == 0) st |= SW_STATUS_NO_PLANNED;
    if (sw_p1_uncertified(o.objective, o.bound)) st |= SW_STATUS_P1_UNCERTIFIED;
    o.status = st;
    /* setup, level rounds, force, [price rounds, take, assign], SELECT, UMAX,
     * [between], share pack, PACKED, exchange, FINAL (swc_* step counts) */
    o.iters = (int32_t)(1 + (long long)srl[3] + 1 + (c->all ? 0 : (long long)sp[3] + 2 + c->tail_steps) + 2 +
                        (c->did_between ? 1 : 0) + 4 + extra_iters);
    o.xerr = xerr ? *xerr : 0;
    *hout = o;
    __threadfence_system();
    __hip_atomic_store(hflag, hseq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* ---- placement ---------------------------------------------------------------- */

/* this rank's entries (twin: the k1/k2 of each pack caller) */
/* mode 1/3 P1 orders A/B, 2 P2 weight order, 4 P2 density order, 5 the
 * class-wise P2 repack of width wc (unit widths) */
/* sub: the shares' layout (entry s·Pp + k = job s·Ps + k, padding zero);
 * else entry i = job i of [0, P).  Jobs outside [jlo, jhi) take no entry. */
__global__ __launch_bounds__(kTB) void k_pack_keys(ShardDev S, int mode, const int32_t* src,
                                                   double Mb, int wc, sw_pack_ent* out, int sub = 0,
                                                   int jlo = 0, int jhi = 0x7FFFFFFF) {
    const int e = blockIdx.x * kTB + threadIdx.x;
    int64_t i = e;
    if (sub) {
        if (e >= (int64_t)S.nsub * S.Pp) return;
        const int64_t sh = e / S.Pp, k = e - sh * S.Pp;
        i = k < S.Ps ? sh * S.Ps + k : (int64_t)S.NL; /* padding: no job */
    } else if (e >= S.P) {
        return;
    }
    sw_pack_ent ent;
    ent.khi = 0; ent.klo = 0; ent.st = 0; ent.pad = 0;
    if (i < S.NL && i >= jlo && i < jhi) {
        const sw_jobc c = S.jc[i];
        const int n = (mode == 5 && c.w != wc) ? 0 : src[i];
        if (n > 0) {
            uint64_t k1;
            uint32_t k2;
            if (mode == 4) {
                k1 = sw_ratio_key(S.p[i] / (double)(n * c.w));
                k2 = 0;
            } else if (mode != 2 && mode != 5) {
                const double lvl = sw_g(&c, n - 1);
                const bool crit = S.k > 0.0 && lvl > Mb;
                k1 = crit ? (SW_CRIT_BIT | sw_bits(lvl)) : (mode == 3 ? (uint64_t)c.w : 0);
                k2 = sw_fbits_of(S.keys[(size_t)i * S.T + n - 1]);
            } else {
                k1 = sw_ratio_key(S.p[i] / (double)n);
                k2 = 0;
            }
            ent.khi = k1;
            ent.klo = ((uint64_t)k2 << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(S.off + i));
            ent.st = (uint32_t)n | ((mode == 5 ? 1u : (uint32_t)c.w) << 8);
        }
    }
    out[e] = ent;
}

/* width-class profile: red[t] = #{local j : src_j > 0, w_j = wc, bit t of
 * ys_j}; red[64] = max over local j with src_j > 0 and w_j > wc of ~w_j;
 * red[65] = #{local j : src_j > 0, w_j = wc}, red[66] = Σ over them of
 * src_j − ps_j (ps = nullptr: 0).  hist: red[v − 1] = #{local j : src_j = v,
 * w_j = wc} instead of the round counts (SW_CLASS_HIST) */
__global__ __launch_bounds__(kTB) void k_class_caps(ShardDev S, const int32_t* src,
                                                    const uint64_t* ys, int wc, const int32_t* ps,
                                                    int hist) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    uint64_t m = 0, nx = 0;
    long long mem = 0, dfc = 0;
    if (i < S.NL && src[i] > 0) {
        const int w = S.jc[i].w;
        if (w == wc) {
            m = hist ? (1ull << (src[i] - 1)) : ys[i];
            mem = 1;
            dfc = ps ? (long long)(src[i] - ps[i]) : 0;
        }
        if (w > wc) nx = 0xFFFFFFFFull - (uint64_t)w;
    }
    for (int t = 0; t < S.T; ++t) red_add(S.red + t, (long long)((m >> t) & 1ull));
    red_umax(S.red + 64, nx);
    red_add(S.red + 65, mem);
    red_add(S.red + 66, dfc);
}

/* the loads Σ w·src of this rank's shares (the share placement) → red[s];
 * a block's jobs lie in at most two shares (Ps ≥ kTB whenever nsub > 1) */
__global__ __launch_bounds__(kTB) void k_load(ShardDev S, const int32_t* src) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    long long v = 0;
    if (i < S.NL) v = (long long)S.jc[i].w * src[i];
    const int s0 = S.nsub > 1 ? (int)(((int64_t)blockIdx.x * kTB) / S.Ps) : 0;
    const int sh = (S.nsub > 1 && i < S.NL) ? (int)(i / S.Ps) : s0;
    red_add(S.red + s0, sh == s0 ? v : 0);
    if (S.nsub > 1) red_add(S.red + s0 + 1, sh != s0 ? v : 0);
    pub_tail(S);
}

/* Every share's capacity of every round (sw_share_caps, restated): loads[V]
 * are the shares' loads in share order (gathered), this rank's shares are
 * rank·nsub … rank·nsub + nsub − 1.  caps[s·64 + t]; caps[SW_VSHARES·64] = 1
 * when the shares exist (0 < L ≤ G·T), else 0.  One wave; exact 64-bit
 * integers (G·T < 2^31, so S·L_r < 2^62; above that no shares). */
/* sw_share_caps of share v on one wave: lane t < T gets round t's capacity;
 * false when the shares do not exist.  Lane r < V computes share r's budget
 * (one 64-bit division each instead of a loop of them per lane). */
__device__ __forceinline__ bool share_caps_wave(const long long* loads, int V, int v, int T, long long G,
                                                int32_t& cap) {
    const int lane = lane_id();
    const long long Lr = lane < V ? loads[lane] : 0;
    long long L = Lr;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) L += __shfl_xor(L, o, 64);
    const long long C = G * (long long)T;
    cap = 0;
    if (!(L > 0 && L <= C && T >= 1 && C < (1ll << 31))) return false;
    const long long Sl = C - L;
    const long long gi = lane < V ? Sl * Lr / L : 0; /* share lane's ⌊S·L_r/L⌋ */
    long long given = gi;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) given += __shfl_xor(given, o, 64);
    const long long rest = Sl - given;
    const long long B = Lr + gi + (lane < rest ? 1 : 0); /* share lane's budget */
    long long m = lane < v ? B % T : 0; /* the extras of the shares before v */
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m += __shfl_xor(m, o, 64);
    const long long cursor = m % T;
    const long long Bv = __shfl(B, v, 64);
    const long long base = Bv / T, ext = Bv % T;
    const long long d = ((long long)lane - cursor + T) % T;
    cap = (int32_t)(base + (d < ext ? 1 : 0));
    return true;
}

__global__ __launch_bounds__(64) void k_share_caps(const long long* loads, int V, int rank, int nsub, int T,
                                                   long long G, int32_t* caps) {
    const int lane = lane_id();
    for (int s = 0; s < nsub; ++s) {
        int32_t c;
        const bool ok = share_caps_wave(loads, V, rank * nsub + s, T, G, c);
        if (s == 0 && lane == 0) caps[SW_VSHARES * 64] = ok ? 1 : 0;
        if (ok && lane < T) caps[s * 64 + lane] = c;
    }
}

__global__ __launch_bounds__(kTB) void k_copy_words(uint32_t* dst, const uint32_t* src, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kTB + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

/* per-solve state: every count array, every bitmask, l and taken = 0, and the
 * step-result ring (S.red at its base) */
__global__ __launch_bounds__(kTB) void k_zero_state(ShardDev S) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    if (i < kRing * kRed) S.red[i] = 0;
    if (i >= S.NL) return;
#pragma unroll
    for (int a = 0; a < SW_A_COUNT; ++a) S.arr[a][i] = 0;
#pragma unroll
    for (int a = 0; a < SW_Y_COUNT; ++a) S.y[a][i] = 0;
    S.l[i] = 0;
    S.taken[i] = 0;
}

struct alignas(16) key2 {
    uint64_t h, l;
};

/* Global placement order of the gathered entries, by sorting: each
 * kSortChunk-entry chunk is bitonic-sorted (descending; inactive entries as
 * (0, 0), which every active key exceeds, sort last), then each active
 * entry's global rank is its chunk position plus, for every other chunk, the
 * number of its keys above the entry's key (a binary search in that sorted
 * chunk).  Keys are unique, so the ranks of the active entries are a
 * permutation of [0, A); order[rank] = entry. */
constexpr int kSortChunk = 256;
constexpr int kSortThreads = kSortChunk; /* one entry per thread */
__device__ __forceinline__ bool key_gt(const key2& a, const key2& b) {
    return a.h > b.h || (a.h == b.h && a.l > b.l);
}
/* One entry per thread, in registers.  Stage (kk, jj) pairs position p with
 * p ^ jj: partners within a wave (jj < 64) trade through cross-lane shuffles,
 * with no barrier; the 10 stages with jj ≥ 64 through LDS.  Both partners
 * evaluate the same exchange test on the same pair (a = the lower position's
 * entry), so they agree on it, and the network and its exchanges are the
 * LDS-only form's: the same sorted chunk.  (The LDS-only form, 512 threads
 * with one pair each and a barrier per stage, took 19–20 µs per 10k-entry
 * sort)
 * nact (optional): the entries are compacted, the first *nact active —
 * chunks past them have nothing to sort */
__global__ __launch_bounds__(kSortThreads) void k_pack_chunk_sort(const sw_pack_ent* all, int64_t M,
                                                                   key2* skeys, int32_t* sidx,
                                                                   const int32_t* nact = nullptr) {
    __shared__ key2 k[kSortChunk];
    __shared__ int32_t ix[kSortChunk];
    const int64_t c0 = (int64_t)blockIdx.x * kSortChunk;
    const int64_t na = nact ? (int64_t)*nact : M;
    if (c0 >= na) return;
    const int p = threadIdx.x;
    key2 v;
    v.h = 0; v.l = 0;
    const int64_t e = c0 + p;
    if (e < M && e < na && all[e].st != 0) { v.h = all[e].khi; v.l = all[e].klo; }
    int32_t vi = (int32_t)e;
    for (int kk = 2; kk <= kSortChunk; kk <<= 1) {
        for (int jj = kk >> 1; jj > 0; jj >>= 1) {
            key2 o;
            int32_t oi;
            if (jj >= 64) {
                k[p] = v;
                ix[p] = vi;
                __syncthreads();
                o = k[p ^ jj];
                oi = ix[p ^ jj];
                __syncthreads();
            } else {
                o.h = __shfl_xor(v.h, jj, 64);
                o.l = __shfl_xor(v.l, jj, 64);
                oi = __shfl_xor(vi, jj, 64);
            }
            const bool lower = (p & jj) == 0;
            const bool desc = (p & kk) == 0;
            const key2& a = lower ? v : o;
            const key2& b = lower ? o : v;
            if (desc ? key_gt(b, a) : key_gt(a, b)) { v = o; vi = oi; }
        }
    }
    skeys[c0 + p] = v;
    sidx[c0 + p] = vi;
}

/* One thread per (entry, chunk): lane q of an entry's group of kMergeG
 * searches chunk q (11 halving steps for the number of its keys above the
 * entry's key: the descending chunk's prefix where ck[i] > v), and the group
 * sums its counts with shuffles.  One thread per entry searching every chunk
 * in turn put ~110 scattered L2 loads per thread on the 40 CUs its 10k
 * threads fill (15 µs per C4 sort; 23 µs with the searches interleaved); the
 * (entry, chunk) grid spreads them over the chip. */
constexpr int kMergeG = 64; /* lanes per entry, a wave (more chunks: lane q searches q, q + 64, …) */
/* cpg > 0: the chunks form groups of cpg (the share placement's shares),
 * each ranked on its own into order[its first entry …] */
__global__ __launch_bounds__(kTB) void k_pack_merge_rank(const key2* skeys, const int32_t* sidx,
                                                         int nchunks, int32_t* order,
                                                         const int32_t* nact = nullptr, int cpg = 0) {
    const int64_t g = (int64_t)blockIdx.x * kTB + threadIdx.x;
    if (nact) nchunks = (int)((*nact + kSortChunk - 1) / kSortChunk);
    const int64_t s = g / kMergeG; /* groups of kMergeG lanes lie inside one wave */
    const int q = (int)(g % kMergeG);
    const bool live = s < (int64_t)nchunks * kSortChunk;
    key2 v;
    v.h = 0; v.l = 0;
    if (live) v = skeys[s];
    const int c = (int)(s / kSortChunk);
    const int c0 = cpg > 0 ? c - c % cpg : 0, c1 = cpg > 0 ? c0 + cpg : nchunks;
    int64_t cnt = 0;
    if (live && (v.h | v.l) != 0)
        for (int qq = c0 + q; qq < c1; qq += kMergeG) { /* the group's chunks q, q + kMergeG, … */
            if (qq == c) continue;
            const key2* ck = skeys + (int64_t)qq * kSortChunk;
            int pos = 0;
#pragma unroll
            for (int step = kSortChunk; step > 0; step >>= 1) {
                const int i = pos + step - 1;
                if (i < kSortChunk && key_gt(ck[i], v)) pos += step;
            }
            cnt += pos;
        }
    int pos = (int)cnt;
#pragma unroll
    for (int o = kMergeG / 2; o > 0; o >>= 1) pos += __shfl_xor(pos, o, 64);
    if (!live || q != 0 || (v.h == 0 && v.l == 0)) return; /* inactive or padding */
    order[(int64_t)c0 * kSortChunk + s - (int64_t)c * kSortChunk + pos] = sidx[s];
}

/* the round loop over the global order; writes this rank's rows */
/* has_caps: per-round capacities in capsL (the share placement's shares, a
 * class-wise repack's class capacities), else G */
template <int E, class BLK>
__device__ __forceinline__ void pack_rounds_body(const ShardDev& S, const sw_pack_ent* all, int A,
                                                 const int32_t* order, uint64_t* ydst, int32_t* pdst,
                                                 bool has_caps, BLK& blk, sw_pack_lds* PL,
                                                 const int32_t* capsL) {
    const int tid = threadIdx.x;
    uint32_t st[E];
    uint64_t mk[E];
    int32_t ent[E];
    const int Am = A > 0 ? A - 1 : 0; /* clamped, unconditional loads: no per-position waits */
#pragma unroll
    for (int i = 0; i < E; ++i) ent[i] = order[min(E * tid + i, Am)];
#pragma unroll
    for (int i = 0; i < E; ++i) {
        const uint32_t v = A > 0 ? all[ent[i]].st : 0u;
        st[i] = E * tid + i < A ? v : 0u;
        ent[i] = E * tid + i < A ? ent[i] : -1;
    }
#ifdef SW_STAMPS
    sw_pack_rounds<E>(blk, PL, A, S.T, S.G, st, mk, has_caps ? capsL : nullptr, g_sw_pack_stamps);
#else
    sw_pack_rounds<E>(blk, PL, A, S.T, S.G, st, mk, has_caps ? capsL : nullptr);
#endif
#pragma unroll
    for (int i = 0; i < E; ++i) {
        if (ent[i] < 0) continue;
        const int64_t j = (int64_t)(0xFFFFFFFFu - (uint32_t)(all[ent[i]].klo & 0xFFFFFFFFu));
        if (j >= S.off && j < S.off + S.NL) {
            ydst[j - S.off] = mk[i];
            pdst[j - S.off] = (int32_t)(all[ent[i]].st & 0xFFu) - (int32_t)pk_r(st[i]);
        }
    }
}

/* The round loop with E positions per thread.  The launch sizes E from the
 * entries M, but only the ACTIVE entries (jobs with rounds to place — about
 * 3/8 of a C4 instance's jobs) take positions, and every pass of the loop
 * walks all E.  So the host launches the variant for M and, when M is large,
 * a smaller one too; each counts the active entries A and runs only when
 * alo < A ≤ E·NT (one runs, the other returns at once).  Separate kernels
 * keep each variant's registers to its own E.  NT threads per workgroup:
 * 1,024 threads with 4 positions each (4 waves per SIMD, 67 VGPRs) placed
 * C4's 3,748 active jobs in 198 µs against 172 µs for 512 threads with 8
 * (DESIGN.md §6.1): the 16-wave block reductions cost more than the shorter
 * walks save, so every variant runs SW_BLOCK threads. */
template <int E, int NT>
__global__ __launch_bounds__(NT) void k_pack_rounds(ShardDev S, const sw_pack_ent* all,
                                                    int64_t M, const int32_t* order,
                                                    uint64_t* ydst, int32_t* pdst,
                                                    CapsArg caps, int alo, int zero,
                                                    const int32_t* capsd = nullptr) {
    __shared__ sw_xchg_t<NT / 64> X;
    __shared__ sw_pack_lds PL;
    __shared__ int32_t capsL[64];
    sw_blk_t<NT / 64> blk;
    blk.X = &X;
    blk.par = 0;
    const int tid = threadIdx.x;
    const bool has = caps.has || capsd; /* capsd: one share, workgroup 0 (k_pack_rounds_wave) */
    if (has && tid < S.T) capsL[tid] = capsd ? capsd[tid] : caps.v[tid];
    if (capsd && capsd[SW_VSHARES * 64] == 0) return; /* no shares: the wave variant cleared the rows */
    int act = 0;
    for (int64_t e = tid; e < M; e += NT) act += all[e].st != 0;
    const int A = blk.sum32(act); /* its barrier publishes capsL */
    if (A <= alo || A > E * NT) return; /* the other variant places these */
    if (zero) /* a whole placement (not one width class): every row of this rank */
        for (int i = tid; i < S.NL; i += NT) { ydst[i] = 0; pdst[i] = 0; }
    pack_rounds_body<E>(S, all, A, order, ydst, pdst, has, blk, &PL, capsL);
}

/* The same round loop on ONE wave (sw_pack_rounds_wave, sw_pack.h): E1
 * positions per lane, position p = E1·lane + i, no barriers — for placements
 * with at most kWaveA active entries, where the block loop's two barriers per
 * scan cost more than the wave's longer per-lane walks (the share placement
 * of a rank's own jobs at W ≥ 2, the class repacks).  A runtime E1 over four
 * instantiations: one wave per CU, so the widest one's registers cost
 * nothing. */
constexpr int kWaveE = 64;
template <int E1>
__device__ __forceinline__ void pack_rounds_wave_body(const ShardDev& S, const sw_pack_ent* all, int A,
                                                      const int32_t* order, uint64_t* ydst, int32_t* pdst,
                                                      const int32_t* capsL, sw_pack_lds* PL, uint64_t* xmk) {
    const int lane = lane_id();
    uint32_t st[E1];
    int32_t ent[E1];
#pragma unroll
    for (int i = 0; i < E1; ++i) {
        const int p = E1 * lane + i;
        ent[i] = p < A ? order[p] : -1;
    }
#pragma unroll
    for (int i = 0; i < E1; ++i) st[i] = ent[i] >= 0 ? all[ent[i]].st : 0u;
    sw_pack_rounds_wave<E1>(PL, S.T, S.G, st, xmk, capsL);
#pragma unroll
    for (int i = 0; i < E1; ++i) {
        if (ent[i] < 0) continue;
        const sw_pack_ent& e = all[ent[i]];
        const int64_t j = (int64_t)(0xFFFFFFFFu - (uint32_t)(e.klo & 0xFFFFFFFFu));
        if (j >= S.off && j < S.off + S.NL) {
            ydst[j - S.off] = xmk[E1 * lane + i];
            pdst[j - S.off] = (int32_t)(e.st & 0xFFu) - (int32_t)pk_r(st[i]);
        }
    }
}

/* amax: the largest active count this kernel places (≤ 64·kWaveE); the block
 * variants (k_pack_rounds, alo = amax) place larger ones */
/* The share placement's form (capsd != nullptr, one workgroup per share):
 * workgroup b places share b — entries [b·M, b·M + M), its order at b·M, its
 * capacities capsd[b·64 …] (all rows of the share cleared when the shares do
 * not exist, capsd[SW_VSHARES·64] = 0) — and clears only the share's rows. */
__device__ __forceinline__ void share_rows(const ShardDev& S, const int32_t* capsd, int zero, int& r0, int& r1) {
    r0 = 0;
    r1 = zero ? S.NL : 0;
    if (capsd) {
        r0 = (int)min((int64_t)S.NL, (int64_t)blockIdx.x * S.Ps);
        r1 = (int)min((int64_t)S.NL, (int64_t)(blockIdx.x + 1) * S.Ps);
    }
}

__global__ __launch_bounds__(64) void k_pack_rounds_wave(ShardDev S, const sw_pack_ent* all, int64_t M,
                                                         const int32_t* order, uint64_t* ydst, int32_t* pdst,
                                                         CapsArg caps, int amax, int zero,
                                                         const int32_t* capsd = nullptr) {
    __shared__ sw_pack_lds PL;
    __shared__ int32_t capsL[64];
    __shared__ uint64_t xmk[64 * kWaveE];
    const int lane = lane_id();
    const int64_t eb = (int64_t)blockIdx.x * M; /* this workgroup's entries and order */
    order += eb;
    const bool has = caps.has || capsd;
    if (has && lane < S.T) capsL[lane] = capsd ? capsd[blockIdx.x * 64 + lane] : caps.v[lane];
    int r0, r1;
    share_rows(S, capsd, zero, r0, r1);
    if (capsd && capsd[SW_VSHARES * 64] == 0) { /* no shares: nothing placed */
        for (int i = r0 + lane; i < r1; i += 64) { ydst[i] = 0; pdst[i] = 0; }
        return;
    }
    int act = 0;
    for (int64_t e = lane; e < M; e += 64) act += all[eb + e].st != 0;
    const int A = wave_sum_i32(act);
    if (A > amax) return; /* the block variant places these */
    /* a whole placement (not one width class): every row of this rank, or of the share */
    for (int i = r0 + lane; i < r1; i += 64) { ydst[i] = 0; pdst[i] = 0; }
    __threadfence_block(); /* the zero rows land before the placed rows below */
    wave_sync();           /* capsL */
    const int32_t* cl = has ? capsL : nullptr;
    if (A <= 64 * 8) pack_rounds_wave_body<8>(S, all, A, order, ydst, pdst, cl, &PL, xmk);
    else if (A <= 64 * 16) pack_rounds_wave_body<16>(S, all, A, order, ydst, pdst, cl, &PL, xmk);
    else if (A <= 64 * 32) pack_rounds_wave_body<32>(S, all, A, order, ydst, pdst, cl, &PL, xmk);
    else pack_rounds_wave_body<64>(S, all, A, order, ydst, pdst, cl, &PL, xmk);
}

/* Active entries up to which the one-wave loop places (SW_SHARD_WAVE_A
 * overrides; 0 = never).  Measured on C4's share placement (MI355X,
 * profiles/r7c4w1_*): 1,900 active entries per rank (W = 2) take 214 µs in
 * the wave loop (E1 = 32) against 149 µs in the 512-thread loop, 3,748 (W = 1)
 * 0.98 ms per solve against 0.75 — its LDS histogram atomics serialise over
 * the lanes of the wave — so it is kept to E1 = 8, where the block loop's
 * two barriers per scan are most of a round's cost. */
int wave_pack_max() {
    static const int v = [] {
        const char* e = getenv("SW_SHARD_WAVE_A");
        const int x = e ? atoi(e) : 512;
        return x < 0 ? 0 : (x > 64 * kWaveE ? 64 * kWaveE : x);
    }();
    return v;
}

/* The round loop for up to 8·NT active entries with E = 2, 4 or 8 positions
 * per thread chosen by A at run time (one launch; the E = 8 body sets the
 * registers, well inside the budget) — and with EB = 20 up to 20·NT in the
 * same launch (one workgroup per placement, so the wider body's registers
 * cost no occupancy; a second kernel that only counted A and returned was
 * 5 µs per C4 placement): the per-position loops of every pass
 * walk what the entries need, not what M allows — a rank's share placement
 * has M = its job count but A = its jobs with rounds (≈ 3/8 of them at C4). */
template <int NT, int EB>
__global__ __launch_bounds__(NT) void k_pack_rounds_sel(ShardDev S, const sw_pack_ent* all, int64_t M,
                                                        const int32_t* order, uint64_t* ydst, int32_t* pdst,
                                                        CapsArg caps, int alo, int zero,
                                                        const int32_t* capsd = nullptr) {
    __shared__ sw_xchg_t<NT / 64> X;
    __shared__ sw_pack_lds PL;
    __shared__ int32_t capsL[64];
    sw_blk_t<NT / 64> blk;
    blk.X = &X;
    blk.par = 0;
    const int tid = threadIdx.x;
    const int64_t eb = (int64_t)blockIdx.x * M; /* this workgroup's entries and order (k_pack_rounds_wave) */
    order += eb;
    const bool has = caps.has || capsd;
    if (has && tid < S.T) capsL[tid] = capsd ? capsd[blockIdx.x * 64 + tid] : caps.v[tid];
    if (capsd && capsd[SW_VSHARES * 64] == 0) { /* no shares: nothing placed */
        int r0, r1;
        share_rows(S, capsd, zero, r0, r1);
        for (int i = r0 + tid; i < r1; i += NT) { ydst[i] = 0; pdst[i] = 0; }
        return;
    }
    int act = 0;
    for (int64_t e = tid; e < M; e += NT) act += all[eb + e].st != 0;
    const int A = blk.sum32(act); /* its barrier publishes capsL */
    if (A <= alo || A > (EB > 8 ? EB : 8) * NT) return; /* another variant places these */
    int r0, r1;
    share_rows(S, capsd, zero, r0, r1);
    /* a whole placement (not one width class): every row of this rank, or of the share */
    for (int i = r0 + tid; i < r1; i += NT) { ydst[i] = 0; pdst[i] = 0; }
    if (A <= 2 * NT) pack_rounds_body<2>(S, all, A, order, ydst, pdst, has, blk, &PL, capsL);
    else if (A <= 4 * NT) pack_rounds_body<4>(S, all, A, order, ydst, pdst, has, blk, &PL, capsL);
    else if (EB <= 8 || A <= 8 * NT)
        pack_rounds_body<8>(S, all, A, order, ydst, pdst, has, blk, &PL, capsL);
    else
        pack_rounds_body<(EB > 8 ? EB : 8)>(S, all, A, order, ydst, pdst, has, blk, &PL, capsL);
}

/* The share placement's round loops in ONE launch (capsd: the shares'
 * capacities, k_share_caps): workgroup b places share b — entries
 * [b·M, b·M + M), its order at b·M — on its one-wave loop when the share has
 * at most wa active entries (wave 0 alone, sw_pack_rounds_wave), else on the
 * block loop with E = 2, 4 or 8 positions per thread.  One launch for both
 * forms: as two launches (k_pack_rounds_wave, then k_pack_rounds_sel for the
 * shares above wa) the C4 placement paid both kernels' ~68 µs in turn
 * (profiles/r8c4a_*). */
/* loads (the gathered share loads, V of them): each workgroup computes its
 * share's capacities itself (share_caps_wave) and stores them to capsd for
 * the host's share repair, instead of a k_share_caps launch before it */
/* dfc (fast_solve): Σ w·(nsrc − placed) over the share's rows — the
 * PACKED evaluation's stranded rounds — added to *dfc by each workgroup */
__global__ __launch_bounds__(SW_BLOCK) void k_pack_rounds_share(ShardDev S, const sw_pack_ent* all, int64_t M,
                                                                const int32_t* order, uint64_t* ydst,
                                                                int32_t* pdst, int32_t* capsd, int wa,
                                                                const long long* loads, int V,
                                                                const int32_t* nsrc = nullptr,
                                                                long long* dfc = nullptr) {
    __shared__ sw_xchg_t<SW_BLOCK / 64> X;
    __shared__ sw_pack_lds PL;
    __shared__ int32_t capsL[64];
    __shared__ int okL;
    __shared__ uint64_t xmk[64 * 8];
    sw_blk_t<SW_BLOCK / 64> blk;
    blk.X = &X;
    blk.par = 0;
    const int tid = threadIdx.x;
    const int64_t eb = (int64_t)blockIdx.x * M;
    order += eb;
    if (tid < 64) {
        int32_t c;
        const bool ok = share_caps_wave(loads, V, S.rank * S.nsub + blockIdx.x, S.T, S.G, c);
        if (tid < S.T) {
            capsL[tid] = c;
            capsd[blockIdx.x * 64 + tid] = c;
        }
        if (tid == 0) {
            okL = ok;
            if (blockIdx.x == 0) capsd[SW_VSHARES * 64] = ok ? 1 : 0;
        }
    }
    int r0, r1;
    share_rows(S, capsd, 1, r0, r1);
    for (int i = r0 + tid; i < r1; i += SW_BLOCK) { ydst[i] = 0; pdst[i] = 0; }
    __syncthreads(); /* capsL, okL */
    if (okL) { /* no shares: nothing placed */
        int act = 0;
        for (int64_t e = tid; e < M; e += SW_BLOCK) act += all[eb + e].st != 0;
        const int A = blk.sum32(act); /* its barrier orders the cleared rows first */
        if (A <= wa && A <= 64 * 8) {
            if (wave_id() == 0) pack_rounds_wave_body<8>(S, all, A, order, ydst, pdst, capsL, &PL, xmk);
        } else if (A <= 2 * SW_BLOCK) {
            pack_rounds_body<2>(S, all, A, order, ydst, pdst, true, blk, &PL, capsL);
        } else if (A <= 4 * SW_BLOCK) {
            pack_rounds_body<4>(S, all, A, order, ydst, pdst, true, blk, &PL, capsL);
        } else if (A <= 8 * SW_BLOCK) {
            pack_rounds_body<8>(S, all, A, order, ydst, pdst, true, blk, &PL, capsL);
        }
    }
    if (!dfc) return;
    __syncthreads(); /* the share's rows are final (device-scope loads below: no stale L1 lines) */
    long long v = 0;
    for (int i = r0 + tid; i < r1; i += SW_BLOCK)
        v += (long long)S.jc[i].w *
             (nsrc[i] - __hip_atomic_load(pdst + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    v = wave_sum(v);
    __shared__ long long vs[SW_BLOCK / 64];
    if (lane_id() == 0) vs[wave_id()] = v;
    __syncthreads();
    if (tid == 0) {
        long long t = 0;
        for (int w = 0; w < SW_BLOCK / 64; ++w) t += vs[w];
        if (t) atomicAdd((unsigned long long*)dfc, (unsigned long long)t);
    }
}

/* ---- P2 exchange step (sw_p2x_dev.h) on the gathered placement ------------------ */

/* one gathered entry per job (the pack's gather buffer, reused) */
struct p2x_ent {
    uint64_t m; /* round mask of the P2 placement */
    double p;   /* priority                       */
    int32_t n, w;
};
static_assert(sizeof(p2x_ent) == sizeof(sw_pack_ent), "p2x entries reuse the pack's gather buffer");

/* bcnt (world 1: the entries are the gathered ones): also k_p2x_cnt's work
 * — each workgroup's active entries, and the zeroed width map and counts */
__global__ __launch_bounds__(kTB) void k_p2x_ent(ShardDev S, const uint64_t* y, const int32_t* n,
                                                 p2x_ent* out, int32_t* bcnt = nullptr, uint32_t* wmap = nullptr,
                                                 int32_t* wcnt = nullptr) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    p2x_ent e;
    e.m = 0; e.p = 0.0; e.n = 0; e.w = 0;
    if (i < S.NL) {
        e.m = y[i]; e.p = S.p[i]; e.n = n[i]; e.w = S.jc[i].w;
    }
    if (i < S.P) out[i] = e;
    if (!bcnt) return;
    if (blockIdx.x == 0 && threadIdx.x < 8) wmap[threadIdx.x] = 0u;
    if (blockIdx.x == 0) wcnt[threadIdx.x] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) wcnt[256] = 0;
    const int w = __popcll(__ballot(i < S.P && e.n > 0));
    __shared__ int32_t ws_[kTB / 64];
    if (lane_id() == 0) ws_[wave_id()] = w;
    __syncthreads();
    if (threadIdx.x == 0) {
        int c = 0;
        for (int k = 0; k < kTB / 64; ++k) c += ws_[k];
        bcnt[blockIdx.x] = c;
    }
}

/* ---- the step's set-up by several workgroups (sw_p2x_pre, sw_p2x_dev.h):
 * the single-workgroup step then starts from the prepared classes,
 * positions, bitsets and first edge costs instead of building them itself
 * (C4: a 4,096-entry rank sort and four full edge builds in one workgroup,
 * ~190 of its ~225 µs).  Same values, so the same result bit for bit. */

/* the active entries compacted in job order into the X arrays (as k_p2x
 * does), by the grid: k_p2x_cnt counts each block's active entries,
 * k_p2x_compact places them (each block's offset = the counts before it),
 * and collects the widths present (wmap) */
__global__ __launch_bounds__(kTB) void k_p2x_cnt(const p2x_ent* all, int64_t M, int32_t* bcnt,
                                                 uint32_t* wmap, int32_t* wcnt) {
    const int64_t j = (int64_t)blockIdx.x * kTB + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < 8) wmap[threadIdx.x] = 0u; /* k_p2x_compact ORs into it */
    if (blockIdx.x == 0) wcnt[threadIdx.x] = 0; /* …and adds widths / its finish counter (wcnt[256]) */
    if (blockIdx.x == 0 && threadIdx.x == 0) wcnt[256] = 0;
    const int a = (j < M && all[j].n > 0) ? 1 : 0;
    const int w = __popcll(__ballot(a));
    __shared__ int32_t ws_[kTB / 64];
    if (lane_id() == 0) ws_[wave_id()] = w;
    __syncthreads();
    if (threadIdx.x == 0) {
        int c = 0;
        for (int i = 0; i < kTB / 64; ++i) c += ws_[i];
        bcnt[blockIdx.x] = c;
    }
}

/* …and the width classes (ascending) with their sizes and offsets in hdr,
 * computed by the last workgroup to finish from the width bitmap wmap and
 * the workgroups' width counts wcnt[w] (no separate launch, no second pass
 * over the entries) */
__global__ __launch_bounds__(kTB) void k_p2x_compact(const p2x_ent* all, int64_t M, const int32_t* bcnt,
                                                     unsigned char* ws, uint32_t* wmap, int32_t* hdr,
                                                     int32_t* wcnt, int T) {
    __shared__ int32_t base_, wsum[kTB / 64];
    __shared__ uint32_t bm[8]; /* this block's widths, one global OR per word */
    __shared__ int32_t wh[256]; /* this block's active entries per width */
    __shared__ int last_;
    const int64_t j = (int64_t)blockIdx.x * kTB + threadIdx.x;
    if (threadIdx.x < 8) bm[threadIdx.x] = 0u;
    wh[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        int b = 0;
        for (unsigned i = 0; i < blockIdx.x; ++i) b += bcnt[i];
        base_ = b;
        if (blockIdx.x == gridDim.x - 1) hdr[SW_P2X_HDR_A] = b + bcnt[blockIdx.x];
    }
    p2x_ent e;
    e.m = 0; e.p = 0.0; e.n = 0; e.w = 0;
    if (j < M) e = all[j];
    const bool act = e.n > 0;
    const uint64_t bal = __ballot(act);
    const int lane = lane_id();
    if (lane == 0) wsum[wave_id()] = __popcll(bal);
    __syncthreads();
    if (act) {
        atomicOr(&bm[(e.w >> 5) & 7], 1u << (e.w & 31));
        atomicAdd(&wh[e.w & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x < 8 && bm[threadIdx.x]) atomicOr(&wmap[threadIdx.x], bm[threadIdx.x]);
    if (wh[threadIdx.x]) atomicAdd(&wcnt[threadIdx.x], wh[threadIdx.x]);
    if (act) {
        int a = base_ + __popcll(bal & ((1ull << lane) - 1ull));
        for (int i = 0; i < wave_id(); ++i) a += wsum[i];
        sw_p2x_arrays X;
        X.cc = reinterpret_cast<double*>(ws);
        X.cm = reinterpret_cast<uint64_t*>(X.cc + M);
        X.cw = reinterpret_cast<int32_t*>(X.cm + M);
        X.cj = X.cw + M;
        X.cw[a] = e.w;
        X.cj[a] = (int32_t)j;
        X.cc[a] = e.p / (double)e.n;
        X.cm[a] = e.m;
    }
    /* the last workgroup to finish: the classes */
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last_ = atomicAdd(&wcnt[256], 1) == (int)gridDim.x - 1;
    __syncthreads();
    if (!last_ || threadIdx.x != 0) return;
    __threadfence();
    uint32_t wm[8];
    int K = 0;
    for (int i = 0; i < 8; ++i) {
        wm[i] = __hip_atomic_load(&wmap[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        K += __builtin_popcount(wm[i]);
    }
    int32_t cls[SW_P2X_KMAX];
    if (K > SW_P2X_KMAX) {
        K = -1;
    } else {
        K = 0;
        for (int i = 0; i < 8; ++i)
            for (uint32_t b = wm[i]; b; b &= b - 1) cls[K++] = 32 * i + __builtin_ctz(b);
    }
    hdr[SW_P2X_HDR_K] = K;
    int o = 0, b = 0;
    for (int k = 0; k < SW_P2X_KMAX; ++k) {
        const int m = (K >= 0 && k < K) ? __hip_atomic_load(&wcnt[cls[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                        : 0;
        hdr[SW_P2X_HDR_WC + k] = (K >= 0 && k < K) ? cls[k] : 0;
        hdr[SW_P2X_HDR_M + k] = m;
        hdr[SW_P2X_HDR_OFF + k] = o;
        hdr[SW_P2X_HDR_NW + k] = (m + 63) / 64;
        hdr[SW_P2X_HDR_BOFF + k] = b;
        o += m;
        b += ((m + 63) / 64) * T; /* word offsets, as sw_p2x_block's boff */
    }
    hdr[SW_P2X_HDR_OFF + SW_P2X_KMAX] = o;
}

/* the rank-sort keys (class asc, sw_p2x_ckey(c) desc, job asc), as
 * descending (~hi, ~lo) keys for k_pack_chunk_sort; key a = active entry a */
__global__ __launch_bounds__(kTB) void k_p2x_keys(const unsigned char* ws, int64_t M, const int32_t* hdr,
                                                  sw_pack_ent* keys) {
    const int64_t i = (int64_t)blockIdx.x * kTB + threadIdx.x;
    const int K = hdr[SW_P2X_HDR_K], A = hdr[SW_P2X_HDR_A];
    if (i >= A || K <= 0) return;
    const double* cc = reinterpret_cast<const double*>(ws);
    const int32_t* cw = reinterpret_cast<const int32_t*>(ws + (size_t)M * 16);
    const int32_t* cj = cw + M;
    int k = 0;
    while (k < K - 1 && hdr[SW_P2X_HDR_WC + k] != cw[i]) ++k;
    const uint64_t ck = sw_p2x_ckey(cc[i]);
    const uint64_t hi = ((uint64_t)k << 61) | (~ck & ((1ull << 61) - 1));
    const uint64_t lo = ((uint64_t)(uint32_t)cj[i] << 32) | (uint32_t)i;
    sw_pack_ent e;
    e.khi = ~hi;
    e.klo = ~lo;
    e.st = 1u;
    e.pad = 0u;
    keys[i] = e;
}

/* positions and bitsets: one wave per 64-rank word slot (class k, word w):
 * lane r takes position off[k] + 64·w + r (ord, pc) and each round's word is
 * one ballot (the layout of sw_p2x_block: word w of round t at boff[k]·T +
 * w·T + t) */
__global__ __launch_bounds__(kTB) void k_p2x_pre_bits(const int32_t* hdr, const int32_t* order,
                                                      const unsigned char* ws, int64_t M, int T,
                                                      int32_t* ord, double* pc, uint64_t* B) {
    const int K = hdr[SW_P2X_HDR_K];
    if (K <= 0) return;
    const double* cc = reinterpret_cast<const double*>(ws);
    const uint64_t* cm = reinterpret_cast<const uint64_t*>(cc + M);
    const int lane = lane_id();
    int sl = (int)((blockIdx.x * kTB + threadIdx.x) >> 6);
    int k = 0;
    while (k < K && sl >= hdr[SW_P2X_HDR_NW + k]) sl -= hdr[SW_P2X_HDR_NW + k++];
    if (k >= K) return;
    const int r = 64 * sl + lane;
    const int p = hdr[SW_P2X_HDR_OFF + k] + r;
    uint64_t m = 0;
    if (r < hdr[SW_P2X_HDR_M + k]) {
        const int a = order[p];
        ord[p] = a;
        pc[p] = cc[a];
        m = cm[a];
    }
    uint64_t* Bk = B + (size_t)hdr[SW_P2X_HDR_BOFF + k] + (size_t)sl * T;
    for (int t = 0; t < T; ++t) {
        const uint64_t word = __ballot((m >> t) & 1ull);
        if (lane == 0) Bk[t] = word;
    }
}

/* the first edge costs of every load size F (each class width): entry
 * (ki, t, u), the cheapest class k with w_k | F, F / w_k ≤ SW_P2X_QMAX
 * (ascending k on ties), without δ — oracle/p2x_twin.c build_w */
/* sw_p2x_cost (sw_p2x.h) on one wave: lane i holds word i of the and-not
 * words in scan order (ascending words when u < t, descending when u > t),
 * 64 words per pass; the q picks are located by a ballot over the lanes'
 * running popcounts, each pick's rank read back to lane 0, which sums c in
 * selection order from 0.0 as the sequential form does.  Wave-uniform
 * result.  (Thread-per-entry, the longest scan — 60 words of a C4 class in
 * one thread, one L2 round trip per word — set the set-up kernel's 32 µs.) */
__device__ __forceinline__ double p2x_cost_wave(const uint64_t* Bt, const uint64_t* Bu, int nw, int ws, int q,
                                                int t, int u, const double* c) {
    const int lane = lane_id();
    const bool lo = u < t;
    double s = 0.0;
    int got = 0;
    for (int base = 0; base < nw && got < q; base += 64) {
        const int i = base + lane;
        const int w = lo ? i : nw - 1 - i; /* the word this lane holds */
        const uint64_t x = i < nw ? (Bt[(size_t)w * ws] & ~Bu[(size_t)w * ws]) : 0ull;
        const int cnt = __popcll(x);
        const int inc = wave_incscan_i32(cnt);
        const int tot = __builtin_amdgcn_readlane(inc, 63);
        const int need = q - got < tot ? q - got : tot;
        for (int g = 0; g < need; ++g) {
            /* the lane holding this pass's pick g: the first with inc > g */
            const int owner = (int)__builtin_ctzll(__ballot(inc > g));
            int rank = 0;
            if (lane == owner) {
                uint64_t y = x;
                for (int d = g - (inc - cnt); d > 0; --d) /* skip the picks before g in this word */
                    y = lo ? (y & (y - 1)) : (y & ~(1ull << (63 - __builtin_clzll(y))));
                rank = 64 * w + (lo ? __builtin_ctzll(y) : 63 - __builtin_clzll(y));
            }
            rank = __builtin_amdgcn_readlane(rank, owner);
            s = s + c[rank];
        }
        got += need;
    }
    return got == q ? s * (double)(u - t) : SW_P2X_NONE;
}

/* one wave per entry (ki, t, u) */
__global__ __launch_bounds__(kTB) void k_p2x_pre_w(const int32_t* hdr, const double* pc,
                                                   const uint64_t* B, int T, double* Wb, int8_t* Wk) {
    const int K = hdr[SW_P2X_HDR_K];
    const int64_t e = ((int64_t)blockIdx.x * kTB + threadIdx.x) >> 6;
    if (K <= 0 || e >= (int64_t)K * T * T) return; /* uniform over the wave */
    const int ki = (int)(e / (T * T)), tu = (int)(e % (T * T)), t = tu / T, u = tu % T;
    const int F = hdr[SW_P2X_HDR_WC + ki];
    double best = SW_P2X_NONE;
    int bk = -1;
    if (t != u)
        for (int k = 0; k < K; ++k) {
            const int wk = hdr[SW_P2X_HDR_WC + k];
            if (wk > F || F % wk != 0 || F / wk > SW_P2X_QMAX) continue;
            const uint64_t* Bk = B + (size_t)hdr[SW_P2X_HDR_BOFF + k];
            const double cost = p2x_cost_wave(Bk + t, Bk + u, hdr[SW_P2X_HDR_NW + k], T, F / wk, t, u,
                                              pc + hdr[SW_P2X_HDR_OFF + k]);
            if (cost < best) {
                best = cost;
                bk = k;
            }
        }
    if (lane_id() == 0) {
        Wb[e] = best;
        Wk[e] = (int8_t)bk;
    }
}

/* The step on the M gathered entries (entry j = job j), one workgroup, the
 * same on every rank; writes this rank's rows of ydst and the number of
 * cycles cancelled into red[0].  pre: the prepared set-up (k_p2x_pre*; the
 * X arrays are then already compacted in ws). */
/* skip (fast_solve): the share placement stranded rounds — leave the
 * placement as it is for the share repair that follows on the host */
__global__ __launch_bounds__(SW_BLOCK) void k_p2x(ShardDev S, const p2x_ent* all, int64_t M,
                                                  unsigned char* ws, uint64_t* ydst, sw_p2x_pre pre,
                                                  int prepared, const long long* skip = nullptr) {
    if (skip && skip[0] != 0) return; /* uniform */
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    sw_p2x_lds* L = reinterpret_cast<sw_p2x_lds*>(smem);
    unsigned char* var = smem + ((sizeof(sw_p2x_lds) + 15) & ~(size_t)15);
    sw_blk blk;
    blk.X = &L->X;
    blk.par = 0;
    sw_p2x_arrays X;
    X.cc = reinterpret_cast<double*>(ws);
    X.cm = reinterpret_cast<uint64_t*>(X.cc + M);
    X.cw = reinterpret_cast<int32_t*>(X.cm + M);
    X.cj = X.cw + M;
    int A;
    if (prepared) {
        A = pre.hdr[SW_P2X_HDR_A];
    } else {
        const int64_t q = (M + SW_BLOCK - 1) / SW_BLOCK;
        const int64_t j0 = (int64_t)threadIdx.x * q, j1 = j0 + q < M ? j0 + q : M;
        int act = 0;
        for (int64_t j = j0; j < j1; ++j) act += all[j].n > 0;
        int a = blk.exscan(act, A);
        for (int64_t j = j0; j < j1; ++j) {
            const p2x_ent e = all[j];
            if (e.n <= 0) continue;
            X.cw[a] = e.w;
            X.cj[a] = (int32_t)j;
            X.cc[a] = e.p / (double)e.n;
            X.cm[a] = e.m;
            ++a;
        }
        __syncthreads();
    }
    const int nc = sw_p2x_block<SW_WAVES, 8>(blk, L, var, X, A, S.T, S.G, nullptr,
                                             prepared ? &pre : nullptr);
    if (nc > 0)
        for (int i = threadIdx.x; i < A; i += SW_BLOCK) {
            const int64_t j = X.cj[i];
            if (j >= S.off && j < S.off + S.NL) ydst[j - S.off] = X.cm[i];
        }
    if (threadIdx.x == 0) S.red[0] = nc;
    if (S.pub.dst) { /* one workgroup: it is the last */
        __threadfence();
        __syncthreads();
        pub_store(S);
    }
}

/* ---- per-round re-optimisation (sw_reround_dev.h) on the gathered P1 plan ----
 * Two 24-byte gathers per job (the pack's entry size, so the peer regions
 * hold them): the inputs (d, R, p) and (mask, count, w, F, E); every rank
 * rebuilds every job's constants with sw_make_jobc — the same bits its owner
 * computed — and runs the step on one workgroup, then keeps its own rows. */
struct rr_in {
    double d, R, p;
};
struct rr_row {
    uint64_t m;
    int32_t n, w, F, E;
};
static_assert(sizeof(rr_in) == sizeof(sw_pack_ent) && sizeof(rr_row) == sizeof(sw_pack_ent),
              "re-optimisation entries use the pack's gather size");

__global__ __launch_bounds__(kTB) void k_rr_ent(ShardDev S, const int32_t* w, const int32_t* F,
                                                const int32_t* E, const double* d, const double* R,
                                                const double* pr, rr_in* in, rr_row* row) {
    const int i = blockIdx.x * kTB + threadIdx.x;
    if (i >= S.P) return;
    rr_in a;
    rr_row b;
    a.d = a.R = a.p = 0.0;
    b.m = 0; b.n = 0; b.w = 1; b.F = 0; b.E = 1;
    if (i < S.NL) {
        a.d = d[i]; a.R = R[i]; a.p = pr[i];
        b.m = S.y[SW_Y_BEST][i]; b.n = S.arr[SW_A_NFIN][i]; b.w = w[i]; b.F = F[i]; b.E = E[i];
    }
    in[i] = a;
    row[i] = b;
}

/* The step's view of the gathered instance: per-job values in the workspace
 * (JMAX = 0 form of sw_reround_dev.h). */
struct ShardRREnv {
    sw_blk& blk;
    int N, T, G, q, nb;
    double k;
    const double *beta, *ell, *slope;
    const sw_jobc* jcg;
    uint64_t* yg;
    int32_t* ng;
    double *gv, *g0, *g1;
    uint8_t *S, *Sb;
    uint32_t* items;
    double *iv, *dpA, *dpB;
    uint64_t* bits;
    __device__ ShardRREnv(sw_blk& b) : blk(b) {}
    template <class F>
    __device__ __forceinline__ void for_jobs(F&& f) {
        const int j0 = (int)threadIdx.x * q, j1 = j0 + q < N ? j0 + q : N;
        for (int j = j0; j < j1; ++j) f(j, 0);
    }
    __device__ __forceinline__ sw_jobc jc(int j) const { return jcg[j]; }
    __device__ __forceinline__ double f(const sw_jobc& c, int n) const {
        return sw_f(&c, n, nb, beta, ell, slope);
    }
    __device__ __forceinline__ bool tj(int j) const { return jcg[j].w <= G; }
    __device__ __forceinline__ uint64_t& y(int j) { return yg[j]; }
    __device__ __forceinline__ int cnt(int j) const { return ng[j]; }
    __device__ __forceinline__ void add_cnt(int j, int d) { ng[j] += d; }
    __device__ __forceinline__ double& V(int j, int) { return gv[j]; }
    __device__ __forceinline__ double& H0(int j, int) { return g0[j]; }
    __device__ __forceinline__ double& H1(int j, int) { return g1[j]; }
};

__global__ __launch_bounds__(SW_BLOCK) void k_rr(ShardDev S, double delta, const rr_in* in,
                                                 const rr_row* row, unsigned char* ws) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int N = (int)S.N;
    sw_blk blk;
    blk.X = reinterpret_cast<sw_xchg*>(smem);
    blk.par = 0;
    size_t off = (sizeof(sw_xchg) + 15) & ~(size_t)15;
    ShardRREnv e(blk);
    e.dpA = reinterpret_cast<double*>(smem + off);
    e.dpB = e.dpA + (SW_RR_CAPMAX + 1);
    e.bits = reinterpret_cast<uint64_t*>(e.dpB + (SW_RR_CAPMAX + 1));
    const size_t M = (size_t)(N > 0 ? N : 1);
    sw_jobc* jcg = reinterpret_cast<sw_jobc*>(ws);
    unsigned char* p = ws + ((M * sizeof(sw_jobc) + 15) & ~(size_t)15);
    e.yg = reinterpret_cast<uint64_t*>(p); p += 8 * M;
    e.gv = reinterpret_cast<double*>(p); p += 8 * M;
    e.g0 = reinterpret_cast<double*>(p); p += 8 * M;
    e.g1 = reinterpret_cast<double*>(p); p += 8 * M;
    e.iv = reinterpret_cast<double*>(p); p += 8 * SW_RR_WORDS;
    e.ng = reinterpret_cast<int32_t*>(p); p += 4 * M;
    e.items = reinterpret_cast<uint32_t*>(p); p += 4 * SW_RR_WORDS;
    e.S = p; p += M;
    e.Sb = p;
    e.jcg = jcg;
    e.N = N; e.T = S.T; e.G = S.G; e.k = S.k; e.nb = S.nb;
    e.q = (N + SW_BLOCK - 1) / SW_BLOCK;
    e.beta = S.beta; e.ell = S.ell; e.slope = S.slope;
    for (int j = threadIdx.x; j < N; j += SW_BLOCK) {
        const rr_in a = in[j];
        const rr_row b = row[j];
        jcg[j] = sw_make_jobc(N, S.T, delta, b.w, a.d, b.F, b.E, a.R, a.p);
        e.yg[j] = b.m;
        e.ng[j] = b.n;
    }
    __syncthreads();
    int64_t passes = 0;
    const int moves = sw_rr_run(e, passes);
    if (moves > 0)
        for (int i = threadIdx.x; i < S.NL; i += SW_BLOCK) {
            S.y[SW_Y_BEST][i] = e.yg[S.off + i];
            S.arr[SW_A_NFIN][i] = e.ng[S.off + i];
        }
    if (threadIdx.x == 0) S.red[0] = moves;
}

/* Step results to the host without a stream synchronisation: the words are
 * stored into fine-grained pinned host memory, then a sequence number is
 * released at system scope; the host spins on it (sw_shard_state::publish).
 * Plain vector stores (global_store), no scalar-cache writes. */
__global__ __launch_bounds__(256) void k_publish(const uint32_t* src, uint32_t* dst, int nwords,
                                                 unsigned long long* flag, unsigned long long seq,
                                                 const int* xerr) {
    for (int i = threadIdx.x; i < nwords; i += blockDim.x) dst[i] = src[i];
    /* one word after the data: the peer transport's sticky error (0 if none) */
    if (threadIdx.x == 0) dst[nwords] = xerr ? (uint32_t)*xerr : 0u;
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* ---- peer-memory step transport (sw_dist_enable_peer) ----------------------
 * Every rank's exchange region: kXHdr bytes of sequence flags (u64 per source
 * rank), then two halves (by sequence parity) of W slots.  A collective is one
 * single-workgroup kernel: this rank's payload is stored into slot `rank` of
 * the current half of EVERY rank's region (over xGMI for ranks on other GPUs),
 * a system-scope release of `seq` into each region's flag `rank` follows, then
 * lane 0 waits for all W flags of its own region to reach `seq` (bounded; a
 * timeout sets the sticky error word) and the workgroup combines the W slots
 * in rank order (all-reduce) or leaves them in place (all-gather: the half IS
 * the gathered array, rank r's block at r·bytes).  Parity halves: a peer can be
 * one exchange ahead but not two (exchange s + 2 needs this rank's flag s + 1,
 * released only after this rank consumed s), so no slot is overwritten while
 * it is read.  The payload is read completely before anything is combined, so
 * in-place all-reduces are safe. */
constexpr int kXHdr = 1024;
/* wall_clock64 ticks (100 MHz) a rank waits for its peers' flags: 10 s by
 * default, SW_PEER_TIMEOUT_MS overrides it (sw_dist_enable_peer).  A timeout
 * sets the sticky error word, which makes the handle unusable: the ranks left
 * the exchange at different sequence numbers, so every later solve on it
 * returns SW_ERR_RCCL until the handle is rebuilt (include/shockwave_amd.h). */
constexpr unsigned long long kXTimeoutDefault = 1000ull * 1000 * 1000;

struct PeerSet {
    unsigned char* base[SW_PEER_MAX_WORLD];
};

/* hdst / hflag (optional): the combined result (all-reduce) or the gathered
 * half (all-gather) also goes to pinned host memory, followed by the error
 * word and a system-scope release of hseq — the host-synchronised steps then
 * need no k_publish launch of their own */
__global__ __launch_bounds__(256) void k_xchg(PeerSet ps, const unsigned char* src, long long bytes,
                                              long long half, int rank, int W, unsigned long long seq,
                                              int op, int n, unsigned char* dst, int* xerr,
                                              uint32_t* hdst, unsigned long long* hflag,
                                              unsigned long long hseq, unsigned long long tmo) {
    const long long off = kXHdr + (long long)(seq & 1ull) * half + (long long)rank * bytes;
    if ((bytes & 15) == 0 && ((uintptr_t)src & 15) == 0) {
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        const long long n16 = bytes >> 4;
        for (long long i = threadIdx.x; i < n16; i += 256) {
            const uint4 v = s4[i];
            for (int p = 0; p < W; ++p) reinterpret_cast<uint4*>(ps.base[p] + off)[i] = v;
        }
    } else {
        const unsigned long long* s8 = reinterpret_cast<const unsigned long long*>(src);
        const long long n8 = bytes >> 3;
        for (long long i = threadIdx.x; i < n8; i += 256) {
            const unsigned long long v = s8[i];
            for (int p = 0; p < W; ++p) reinterpret_cast<unsigned long long*>(ps.base[p] + off)[i] = v;
        }
    }
    /* every thread makes its own payload stores visible at system scope
     * before the barrier: a system-scope release orders only the issuing
     * wave's outstanding stores, so the flag writers' releases below cannot
     * publish the other waves' payload on their own */
    __threadfence_system();
    __syncthreads();
    if ((int)threadIdx.x < W)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(ps.base[threadIdx.x]) + rank, seq,
                           __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    __shared__ int bad;
    if (threadIdx.x == 0) {
        int b = 0;
        const unsigned long long* fl = reinterpret_cast<const unsigned long long*>(ps.base[rank]);
        const uint64_t t0 = wall_clock64();
        for (int sr = 0; sr < W && !b; ++sr)
            while (__hip_atomic_load(fl + sr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
                if (wall_clock64() - t0 > tmo) { b = 1; break; }
                __builtin_amdgcn_s_sleep(1);
            }
        if (b) atomicExch(xerr, 1);
        bad = b;
    }
    __syncthreads();
    const unsigned char* mine = ps.base[rank] + kXHdr + (long long)(seq & 1ull) * half;
    for (int i = threadIdx.x; i < ((bad || op == 3) ? 0 : n); i += 256) {
        if (op == 0) {
            long long v = 0;
            for (int sr = 0; sr < W; ++sr) v += reinterpret_cast<const long long*>(mine + sr * bytes)[i];
            reinterpret_cast<long long*>(dst)[i] = v;
        } else if (op == 1) {
            unsigned long long v = 0;
            for (int sr = 0; sr < W; ++sr) {
                const unsigned long long x = reinterpret_cast<const unsigned long long*>(mine + sr * bytes)[i];
                v = x > v ? x : v;
            }
            reinterpret_cast<unsigned long long*>(dst)[i] = v;
        } else {
            double v = reinterpret_cast<const double*>(mine)[i];
            for (int sr = 1; sr < W; ++sr) {
                const double x = reinterpret_cast<const double*>(mine + sr * bytes)[i];
                v = x > v ? x : v;
            }
            reinterpret_cast<double*>(dst)[i] = v;
        }
    }
    if (hdst) {
        __syncthreads(); /* the combine is complete */
        const uint32_t* from = reinterpret_cast<const uint32_t*>(op == 3 ? mine : dst);
        const int words = op == 3 ? (int)((long long)W * bytes / 4) : 2 * n;
        if (!bad)
            for (int i = threadIdx.x; i < words; i += 256) hdst[i] = from[i];
        if (threadIdx.x == 0) hdst[words] = bad ? 1u : 0u;
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(hflag, hseq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

/* A per-process identity: 128 random bits drawn once per process, and the
 * kernel boot id (so equal nonces on two hosts cannot collide either). */
void process_identity(unsigned long long nonce[2], char* boot, size_t boot_len) {
    /* drawn once per process: a function-local static is initialised exactly
     * once even when ranks that are threads of one process call this at the
     * same time (C++11), so every such rank sees the same nonce */
    struct Nonce {
        unsigned long long n0 = 0, n1 = 0;
    };
    static const Nonce id = [] {
        Nonce n;
        FILE* f = fopen("/dev/urandom", "rb");
        if (!f || fread(&n.n0, sizeof(n.n0), 1, f) != 1 || fread(&n.n1, sizeof(n.n1), 1, f) != 1) {
            n.n0 = (unsigned long long)getpid() * 0x9E3779B97F4A7C15ull ^ (unsigned long long)time(nullptr);
            n.n1 = (unsigned long long)(uintptr_t)&process_identity;
        }
        if (f) fclose(f);
        if (n.n0 == 0 && n.n1 == 0) n.n0 = 1;
        return n;
    }();
    nonce[0] = id.n0;
    nonce[1] = id.n1;
    memset(boot, 0, boot_len);
    if (FILE* b = fopen("/proc/sys/kernel/random/boot_id", "r")) {
        if (!fgets(boot, (int)boot_len, b)) boot[0] = 0;
        fclose(b);
    }
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + kTB - 1) / kTB > 0 ? (n + kTB - 1) / kTB : 1); }

}  // namespace

/* ---- host side: the engine behind sw_shard_ops ------------------------------ */

struct sw_shard_state {
    sw_handle* h = nullptr;
    /* step results published by k_publish: fine-grained pinned host memory
     * (data, then the flag word), its device alias, the last sequence number */
    uint32_t* pub = nullptr;
    uint32_t* pub_dev = nullptr;
    size_t pub_words = 0;
    unsigned long long* pub_flag = nullptr;
    unsigned long long* pub_flag_dev = nullptr;
    unsigned long long pub_seq = 0;
    /* a step kernel armed to publish its own result (arm_pub): the sequence
     * number it releases and the device words it stores, consumed by the
     * publish() of the same words */
    unsigned long long armed_seq = 0;
    const void* armed_src = nullptr;
    size_t armed_bytes = 0;
    int32_t rank = 0, world = 1;
    ncclComm_t comm = nullptr;
    bool host_comm = false;
    sw_host_comm hc;
    /* peer-memory transport (sw_dist_enable_peer): own region, every rank's
     * region as mapped here, IPC mappings to close, half size, sequence,
     * sticky device error word, the largest total_jobs the regions fit */
    bool peer = false;
    unsigned char* xreg = nullptr;
    PeerSet ps{};
    void* opened[SW_PEER_MAX_WORLD] = {};
    long long xhalf = 0, xslot = 0;
    unsigned long long xseq = 0;
    int* xerr = nullptr;
    int64_t xmax_jobs = 0;
    unsigned long long xtimeout = kXTimeoutDefault;
    bool xfailed = false;
    /* current solve */
    int32_t NL = 0, T = 0;
    int64_t N = 0, off = 0, q = 1, P = 0, LW = 0;
    double delta = 0.0;
    ShardDev dv;
    /* device */
    DevBuf<int32_t> w, F, E, l, taken, tie, arr[SW_A_COUNT], planned, porder;
    DevBuf<double> xa;
    DevBuf<double> d, R, p, xrecv; /* gathers run in place: rank r's block is its send buffer */
    DevBuf<sw_jobc> jc;
    DevBuf<float> keys;
    DevBuf<uint64_t> y[SW_Y_COUNT];
    DevBuf<uint8_t> plan;
    DevBuf<long long> red, tieblk;
    DevBuf<sw_pack_ent> pall;
    DevBuf<unsigned char> p2ws; /* P2 exchange arrays (SW_P2X_ARR_BYTES per gathered entry), prepared set-up */
    DevBuf<sw_pack_ent> p2keys; /* the exchange's rank-sort keys (k_p2x_pre0) */
    DevBuf<unsigned char> rrin, rrrow, rrws; /* re-optimisation: gathered entries, workspace */
    DevBuf<unsigned long long> srch; /* device-chained search states (k_search_*): level [0, 2·kSt), price after */
    DevBuf<unsigned long long> glist, glall; /* the searches' item lists (level, price; kGl words each), all-gathered */
    DevBuf<FastCtl> fctl;            /* fast_solve's device-side controller state */
    DevBuf<key2> skeys;   /* chunk-sorted placement keys */
    DevBuf<int32_t> sidx; /* their entries */
    /* this solve's per-job inputs on the device: the buffers above after an
     * upload, or the caller's own HBM (sw_dist_plan_solve_dev) */
    const int32_t *in_w = nullptr, *in_F = nullptr, *in_E = nullptr;
    const double *in_d = nullptr, *in_R = nullptr, *in_p = nullptr;
    int ring_pos = kRing; /* next step-result slice (kRing = clear the ring first) */
    bool zero_pending = false;
    /* pinned staging */
    HostBuf<uint8_t> hx;
    DevBuf<int32_t> scapsd; /* every share's capacities of every round + the shares flag (k_share_caps) */
    std::vector<int32_t> w_all;
    std::vector<uint8_t> hgather;
};

namespace {

#define SH_HIP(S, call)                                                                    \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) {                                                            \
            (S)->h->err = std::string(#call) + ": " + hipGetErrorString(e_);               \
            return SW_ERR_HIP;                                                             \
        }                                                                                  \
    } while (0)

#define SH_NCCL(S, call)                                                                   \
    do {                                                                                   \
        ncclResult_t r_ = (call);                                                          \
        if (r_ != ncclSuccess) {                                                           \
            (S)->h->err = std::string(#call) + ": " + ncclGetErrorString(r_);              \
            return SW_ERR_RCCL;                                                            \
        }                                                                                  \
    } while (0)

#define SH_TRY(x)                \
    do {                         \
        int rc_ = (x);           \
        if (rc_ < 0) return rc_; \
    } while (0)

int host_fail(sw_shard_state* S, const char* what) {
    S->h->err = std::string("host collective failed: ") + what;
    return SW_ERR_RCCL;
}

/* Copies `bytes` (a multiple of 4) of device memory to `hout` once the
 * stream reaches this point: k_publish stores them into pinned host memory
 * and releases a sequence number, and the host spins on it instead of a
 * stream synchronisation (the wake-up of hipStreamSynchronize is the larger
 * part of a host-synchronised step's round trip).  A flag that does not
 * arrive within 30 s falls back to hipStreamSynchronize, which reports the
 * failed kernel. */
/* pinned buffers for `words` result words + the error word */
int publish_reserve(sw_shard_state* S, size_t words) {
    if (words + 1 > S->pub_words) { /* + the transport's error word */
        if (S->pub) (void)hipHostFree(S->pub);
        S->pub = nullptr;
        S->pub_words = 0;
        const size_t want = words + 1 < 2048 ? 2048 : words + 1;
        SH_HIP(S, hipHostMalloc((void**)&S->pub, want * 4, hipHostMallocMapped | hipHostMallocCoherent));
        SH_HIP(S, hipHostGetDevicePointer((void**)&S->pub_dev, S->pub, 0));
        S->pub_words = want;
    }
    if (!S->pub_flag) {
        SH_HIP(S, hipHostMalloc((void**)&S->pub_flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
        SH_HIP(S, hipHostGetDevicePointer((void**)&S->pub_flag_dev, S->pub_flag, 0));
        __atomic_store_n(S->pub_flag, 0ull, __ATOMIC_RELEASE);
        S->pub_seq = 0;
    }
    return SW_OK;
}

/* spin until sequence number seq is released, then copy the words out */
int publish_wait(sw_shard_state* S, unsigned long long seq, size_t words, size_t bytes, void* hout) {
    hipStream_t st = S->h->stream;
    auto t0 = std::chrono::steady_clock::now();
    uint32_t spins = 0;
    while (__atomic_load_n(S->pub_flag, __ATOMIC_ACQUIRE) < seq) {
        __builtin_ia32_pause();
        if (((++spins) & 0xFFFFu) == 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
            SH_HIP(S, hipStreamSynchronize(st));
            if (__atomic_load_n(S->pub_flag, __ATOMIC_ACQUIRE) < seq)
                return S->h->err = "publish: step result never arrived", SW_ERR_HIP;
            break;
        }
    }
    if (S->pub[words] != 0u) {
        S->xfailed = true; /* sticky: the ranks stopped at different exchanges */
        return S->h->err = "peer exchange: a rank's flag never arrived (timed out)", SW_ERR_RCCL;
    }
    memcpy(hout, S->pub, bytes);
    return SW_OK;
}

int publish(sw_shard_state* S, const void* dsrc, size_t bytes, void* hout) {
    const size_t words = (bytes + 3) / 4;
    if (bytes % 4 != 0) return S->h->err = "publish: size not a multiple of 4", SW_ERR_INVALID;
    if (S->armed_seq) { /* the step kernel publishes these words itself */
        const unsigned long long seq = S->armed_seq;
        S->armed_seq = 0;
        if (S->armed_src == dsrc && S->armed_bytes == bytes) return publish_wait(S, seq, words, bytes, hout);
        /* not these words: its release precedes the one below, which is waited for */
    }
    SH_TRY(publish_reserve(S, words));
    const unsigned long long seq = ++S->pub_seq;
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(256), 0, S->h->stream, (const uint32_t*)dsrc,
                       S->pub_dev, (int)words, S->pub_flag_dev, seq, (const int*)S->xerr);
    SH_HIP(S, hipGetLastError());
    return publish_wait(S, seq, words, bytes, hout);
}

/* Fused publish (world 1, no peer transport, no host collectives): the step
 * kernel launched next stores `bytes` of `dsrc` into the pinned buffer and
 * releases the flag from its last block (pub_tail / pub_store), so the
 * host's publish() of the same words only waits — no k_publish launch, whose
 * dispatch sat between the step kernel and the host on every
 * host-synchronised step (13 per C4 solve).  disarm_pub after the launch. */
int arm_pub(sw_shard_state* S, const void* dsrc, size_t bytes) {
    S->dv.pub.dst = nullptr;
    if (S->world != 1 || S->peer || S->host_comm || bytes % 4 != 0) return SW_OK;
    const size_t words = bytes / 4;
    SH_TRY(publish_reserve(S, words));
    S->armed_seq = ++S->pub_seq;
    S->armed_src = dsrc;
    S->armed_bytes = bytes;
    S->dv.pub.dst = S->pub_dev;
    S->dv.pub.flag = S->pub_flag_dev;
    S->dv.pub.seq = S->armed_seq;
    S->dv.pub.src = (const uint32_t*)dsrc;
    S->dv.pub.xerr = (const int*)S->xerr;
    S->dv.pub.nwords = (int)words;
    return SW_OK;
}
inline void disarm_pub(sw_shard_state* S) { S->dv.pub.dst = nullptr; }

/* One peer-transport collective (k_xchg) on the handle's stream. */
/* hout (optional): the result also comes to the host (fused publish) */
int peer_xchg(sw_shard_state* S, const void* src, size_t bytes, int op, int n, void* dst,
              void* hout = nullptr) {
    if ((long long)bytes > S->xslot)
        return S->h->err = "peer exchange: step payload exceeds the region slot", SW_ERR_CAPACITY;
    if (bytes % 8 != 0) return S->h->err = "peer exchange: size not a multiple of 8", SW_ERR_INVALID;
    const size_t obytes = op == 3 ? bytes * (size_t)S->world : (size_t)n * 8;
    unsigned long long hseq = 0;
    if (hout) {
        SH_TRY(publish_reserve(S, obytes / 4));
        hseq = ++S->pub_seq;
    }
    hipLaunchKernelGGL(k_xchg, dim3(1), dim3(256), 0, S->h->stream, S->ps, (const unsigned char*)src,
                       (long long)bytes, S->xhalf, (int)S->rank, (int)S->world, ++S->xseq, op, n,
                       (unsigned char*)dst, S->xerr, hout ? S->pub_dev : nullptr,
                       hout ? S->pub_flag_dev : nullptr, hseq, S->xtimeout);
    SH_HIP(S, hipGetLastError());
    if (hout) return publish_wait(S, hseq, obytes / 4, obytes, hout);
    return SW_OK;
}

/* this rank's view of the last peer all-gather (rank r's block at r·bytes) */
inline const void* peer_gathered(const sw_shard_state* S) {
    return S->xreg + kXHdr + (long long)(S->xseq & 1ull) * S->xhalf;
}

/* In-place all-reduce of n values on the device buffer `dbuf`, copied to
 * `hout`.  op: 0 = sum i64, 1 = max u64, 2 = max f64. */
int coll_reduce(sw_shard_state* S, void* dbuf, int n, int op, void* hout) {
    hipStream_t st = S->h->stream;
    const size_t bytes = (size_t)n * 8;
    /* through RCCL above world 1; at world 1 the all-reduce is the identity
     * and is skipped (RCCL's own copies cost ~30 µs per C4 solve there) */
    if (S->peer) return peer_xchg(S, dbuf, bytes, op, n, dbuf, hout);
    if (S->comm && S->world > 1) {
        const ncclDataType_t ty = op == 0 ? ncclInt64 : op == 1 ? ncclUint64 : ncclFloat64;
        SH_NCCL(S, ncclAllReduce(dbuf, dbuf, (size_t)n, ty, op == 0 ? ncclSum : ncclMax, S->comm, st));
    }
    SH_TRY(publish(S, dbuf, bytes, hout));
    if (S->world > 1 && S->host_comm && !S->peer) {
        int rc = op == 0 ? S->hc.allreduce_sum_i64(S->hc.ctx, (int64_t*)hout, n)
               : op == 1 ? S->hc.allreduce_max_u64(S->hc.ctx, (uint64_t*)hout, n)
                         : S->hc.allreduce_max_f64(S->hc.ctx, (double*)hout, n);
        if (rc) return host_fail(S, "all-reduce");
    }
    return SW_OK;
}

/* All-gather `bytes` per rank from dsend into drecv (device, rank order).
 * If hrecv is set, the gathered blocks are also copied to the host.  With the
 * peer transport the gathered blocks stay in this rank's exchange region:
 * *dview (if given) receives where they are on the device (drecv otherwise). */
int coll_gather(sw_shard_state* S, const void* dsend, void* drecv, size_t bytes, void* hrecv,
                const void** dview = nullptr) {
    hipStream_t st = S->h->stream;
    const size_t total = bytes * (size_t)S->world;
    if (dview) *dview = drecv;
    if (S->peer) {
        SH_TRY(peer_xchg(S, dsend, bytes, 3, 0, nullptr, hrecv));
        const void* g = peer_gathered(S);
        if (dview) *dview = g;
        else if (!hrecv) SH_HIP(S, hipMemcpyAsync(drecv, g, total, hipMemcpyDeviceToDevice, st));
        return SW_OK;
    }
    if (!S->host_comm) {
        const bool one = !S->comm || S->world == 1;
        /* no communicator: the gather is the identity; a gather read back by
         * the host is not needed on the device afterwards, so it is copied
         * down directly */
        if (one) {
            if (drecv != dsend && !hrecv)
                SH_HIP(S, hipMemcpyAsync(drecv, dsend, bytes, hipMemcpyDeviceToDevice, st));
        } else {
            SH_NCCL(S, ncclAllGather(dsend, drecv, bytes, ncclUint8, S->comm, st));
        }
        if (hrecv) SH_TRY(publish(S, one ? dsend : drecv, total, hrecv));
        return SW_OK;
    }
    /* host collectives: down, gather, up */
    if (S->hx.reserve(total)) return host_fail(S, "pinned staging");
    S->hgather.resize(total);
    SH_HIP(S, hipMemcpyAsync(S->hx.p, dsend, bytes, hipMemcpyDeviceToHost, st));
    SH_HIP(S, hipStreamSynchronize(st));
    std::vector<uint8_t> mine(S->hx.p, S->hx.p + bytes);
    if (S->hc.allgather(S->hc.ctx, mine.data(), S->hgather.data(), (int64_t)bytes))
        return host_fail(S, "all-gather");
    memcpy(S->hx.p, S->hgather.data(), total);
    SH_HIP(S, hipMemcpyAsync(drecv, S->hx.p, total, hipMemcpyHostToDevice, st));
    if (hrecv) memcpy(hrecv, S->hgather.data(), total);
    SH_HIP(S, hipStreamSynchronize(st)); /* staging is reused by the next step */
    return SW_OK;
}

/* Step-result slots: a ring of kRing zeroed slices of kRed entries.  Each
 * step takes the next slice (S->dv.red, passed to its kernels by value), so
 * the whole ring is cleared once per kRing steps instead of a memset per step. */
int zero_red(sw_shard_state* S, int n) {
    (void)n;
    S->dv.pub.dst = nullptr; /* a step's kernels publish only when armed for it */
    if (S->ring_pos >= kRing) {
        SH_HIP(S, hipMemsetAsync(S->red.p, 0, (size_t)kRing * kRed * 8, S->h->stream));
        S->ring_pos = 0;
    }
    S->dv.red = S->red.p + (size_t)S->ring_pos * kRed;
    S->ring_pos++;
    return SW_OK;
}

#define LAUNCH(S, ...)                                   \
    do {                                                 \
        hipLaunchKernelGGL(__VA_ARGS__);                 \
        SH_HIP(S, hipGetLastError());                    \
    } while (0)

/* ---- sw_shard_ops ---------------------------------------------------------- */

int op_setup(void* ctx, double* A, double* lb, double* top) {
    auto* S = (sw_shard_state*)ctx;
    hipStream_t st = S->h->stream;
    SH_TRY(zero_red(S, 4));
    SH_TRY(arm_pub(S, S->dv.red, 32));
    const bool fused = S->dv.pub.dst != nullptr; /* world 1: the all-reduce is the identity */
    LAUNCH(S, k_setup, dim3(nblk(S->NL)), dim3(kTB), 0, st, S->dv, S->jc.p, S->in_w, S->in_d, S->in_F,
           S->in_E, S->in_R, S->delta);
    disarm_pub(S);
    /* k_keys reads A from red[0]: at world 1 that is k_setup's own result, so the
     * key rows are enqueued before the host waits for the step result (their
     * 8 µs overlap its round trip; on invalid inputs they are computed and
     * discarded) */
    if (fused) LAUNCH(S, k_keys, dim3(nblk((int64_t)S->NL * 64)), dim3(kTB), 0, st, S->dv);
    uint64_t mx[4];
    SH_TRY(coll_reduce(S, S->dv.red, 4, 1, mx));
    if (mx[2]) return S->h->err = "invalid problem (per-job inputs)", SW_ERR_INVALID; /* every rank */
    if (S->host_comm && S->world > 1 && !S->peer) { /* kernels read A from red[0] */
        memcpy(S->hx.p, mx, 16);
        SH_HIP(S, hipMemcpyAsync(S->dv.red, S->hx.p, 16, hipMemcpyHostToDevice, st));
        SH_HIP(S, hipStreamSynchronize(st));
    }
    if (!fused) LAUNCH(S, k_keys, dim3(nblk((int64_t)S->NL * 64)), dim3(kTB), 0, st, S->dv);
    *A = sw_from_bits(mx[0]);
    *lb = sw_from_bits(mx[1]);
    *top = sw_from_bits(mx[3]);
    return SW_OK;
}

/* every job's width (the controller's width tail and fill, on first use) */
int op_widths(void* ctx, int32_t* w_all) {
    auto* S = (sw_shard_state*)ctx;
    hipStream_t st = S->h->stream;
    /* in place: this rank's block of the receive buffer is the send buffer
     * (no self-copy in the all-gather, none at all at world 1) */
    int32_t* wrecv = (int32_t*)S->xrecv.p;
    int32_t* wsend = wrecv + (size_t)S->rank * S->P;
    SH_HIP(S, hipMemsetAsync(wsend, 0, (size_t)S->P * 4, st));
    if (S->NL) SH_HIP(S, hipMemcpyAsync(wsend, S->in_w, (size_t)S->NL * 4, hipMemcpyDeviceToDevice, st));
    S->w_all.resize((size_t)S->P * S->world);
    SH_TRY(coll_gather(S, wsend, wrecv, (size_t)S->P * 4, S->w_all.data()));
    for (int64_t j = 0; j < S->N; ++j) w_all[j] = S->w_all[j]; /* rank r's block starts at job r·P */
    return SW_OK;
}

int op_force(void* ctx, double M, int32_t is_inf, int64_t out[2]) {
    auto* S = (sw_shard_state*)ctx;
    SH_TRY(zero_red(S, 2));
    SH_TRY(arm_pub(S, S->dv.red, 16));
    LAUNCH(S, k_force, dim3(nblk(S->NL)), dim3(kTB), 0, S->h->stream, S->dv, M, (int)is_inf);
    disarm_pub(S);
    return coll_reduce(S, S->dv.red, 2, 0, out);
}

template <bool LEVEL>
int probe(sw_shard_state* S, const uint64_t* v, int32_t K, uint64_t lo, int64_t* out) {
    Thresholds th;
    th.K = K;
    th.lo = lo;
    for (int i = 0; i < K; ++i) th.v[i] = v[i];
    SH_TRY(zero_red(S, K + 1));
    /* the price probe is bound by its block → global flush (K atomics per
     * block): a bounded grid; the level probe by its fp64 work: full grid */
    const unsigned pb = nblk((int64_t)S->NL * S->T);
    const unsigned grid = LEVEL ? pb : (unsigned)probe_blocks(pb);
    LAUNCH(S, k_probe<LEVEL>, dim3(grid), dim3(kTB), 0, S->h->stream, S->dv, th);
    int64_t bins[SW_SHARD_K + 1];
    SH_TRY(coll_reduce(S, S->dv.red, K + 1, 0, bins));
    int64_t suf = 0;
    for (int i = K - 1; i >= 0; --i) { suf += bins[i + 1]; out[i] = suf; }
    out[K] = suf + bins[0]; /* the items ≥ lo */
    return SW_OK;
}

int op_count_gt(void* ctx, const uint32_t* rho, int32_t K, uint64_t lo, int64_t* out) {
    uint64_t v[SW_SHARD_K];
    for (int i = 0; i < K; ++i) v[i] = rho[i];
    return probe<false>((sw_shard_state*)ctx, v, K, lo, out);
}

int op_feasible(void* ctx, const double* M, int32_t K, uint64_t lo, int64_t* out) {
    uint64_t v[SW_SHARD_K];
    for (int i = 0; i < K; ++i) v[i] = sw_bits(M[i]);
    return probe<true>((sw_shard_state*)ctx, v, K, lo, out);
}

/* The rounds of a device-chained search on the state at sb[0..kSt) (set in
 * stream order before), its item list gl (kGl words): nr rounds, each a
 * probe or a gather (by its state) → the collectives (above world 1: the
 * bins' all-reduce, and from round 1 on, when a round may be a gather, the
 * lists' all-gather) → the step applied in the next round, then the last
 * step in place.  *fin = the final state (lo = the answer, [3] = the rounds
 * taken).  Searches whose bracket closes early leave their last rounds empty. */
int enqueue_search(sw_shard_state* S, int32_t kind, int nr, unsigned long long* sb, unsigned long long* gl,
                   unsigned long long** fin, bool arm = false, SearchTail* tail = nullptr) {
    hipStream_t st = S->h->stream;
    const int W = S->world;
    /* round r reads round r − 1's slice: keep the nr slices inside one pass of
     * the ring (a wrap clears the whole ring) */
    if (S->ring_pos + nr > kRing) S->ring_pos = kRing;
    const unsigned pb = nblk((int64_t)S->NL * S->T);
    const long long* prev = nullptr;
    const unsigned long long* gview = gl; /* world 1: the rank's own list is every list */
    for (int r = 0; r < nr; ++r) {
        SH_TRY(zero_red(S, SW_SHARD_K + 1));
        const unsigned long long* xin = sb + kSt * ((r + 1) & 1); /* X_{r−1} (X_0 for r = 0) */
        unsigned long long* xout = sb + kSt * (r & 1);
        if (r == 0) xin = sb;
        if (kind == 0)
            LAUNCH(S, k_probe_dev<false>, dim3((unsigned)probe_blocks(pb)),
                   dim3(kTB), 0, st, S->dv, xin, xout, prev, gl, gview, W);
        else
            LAUNCH(S, k_probe_dev<true>, dim3(pb), dim3(kTB), 0, st, S->dv, xin, xout, prev, gl, gview, W);
        if (W > 1) {
            if (S->peer)
                SH_TRY(peer_xchg(S, S->dv.red, (size_t)(SW_SHARD_K + 1) * 8, 0, SW_SHARD_K + 1, S->dv.red));
            else if (S->comm)
                SH_NCCL(S, ncclAllReduce(S->dv.red, S->dv.red, (size_t)SW_SHARD_K + 1, ncclInt64, ncclSum,
                                         S->comm, st));
            if (r > 0) { /* round 0 probes: no bracket's ends are known before it */
                if (S->peer) {
                    SH_TRY(peer_xchg(S, gl, (size_t)kGl * 8, 3, 0, nullptr));
                    gview = (const unsigned long long*)peer_gathered(S);
                } else if (S->comm) {
                    SH_NCCL(S, ncclAllGather(gl, S->glall.p, (size_t)kGl * 8, ncclUint8, S->comm, st));
                    gview = S->glall.p;
                }
            }
        }
        prev = S->dv.red;
    }
    unsigned long long* sr = sb + kSt * ((nr - 1) & 1); /* X_{nr−1}, stepped in place */
    if (tail) { /* the consumer steps it: X_nr into the other half (X_{nr−2}'s, read by now) */
        tail->x = sr;
        tail->xo = sb + kSt * (nr & 1);
        tail->bins = prev;
        tail->lists = gview;
        tail->W = W;
        *fin = tail->xo;
        return SW_OK;
    }
    if (arm) SH_TRY(arm_pub(S, sr, 32)); /* world 1: the update publishes the state itself */
    LAUNCH(S, k_search_update, dim3(1), dim3(kTB), 0, st, sr, prev, gview, W, S->dv);
    disarm_pub(S);
    *fin = sr;
    return SW_OK;
}

/* swc_search with every round on the stream (enqueue_search): the bound on
 * the rounds enqueued (closed rounds are no-ops), one read-back at the end.
 * RCCL, the peer transport or a single rank: host collectives need the host
 * between rounds and use the controller's loop. */
int op_search(void* ctx, int32_t kind, uint64_t lo, uint64_t hi, int64_t bud, int64_t chi, uint64_t* out,
              int32_t* rounds) {
    auto* S = (sw_shard_state*)ctx;
    hipStream_t st = S->h->stream;
    /* a probe round leaves a span ≤ ⌊span / (K + 1)⌋ and a gather round
     * closes the bracket, so the rounds are at most the base-(K + 1) digits
     * of the initial span */
    int nr = 0;
    for (uint64_t sp = lo < hi ? hi - lo : 0; sp > 0; sp /= (uint64_t)(SW_SHARD_K + 1)) ++nr;
    *rounds = 0;
    *out = lo;
    if (nr == 0) return SW_OK;
    unsigned long long* sb = S->srch.p;
    LAUNCH(S, k_search_init, dim3(1), dim3(64), 0, st, sb, (unsigned long long)lo,
           (unsigned long long)hi, (long long)bud, (long long)chi);
    unsigned long long* sr = nullptr;
    SH_TRY(enqueue_search(S, kind, nr, sb, S->glist.p, &sr, true));
    unsigned long long v[4];
    SH_TRY(publish(S, sr, sizeof(v), v));
    *out = v[0];
    *rounds = (int32_t)v[3];
    return SW_OK;
}

/* the items of a search bracket (sw_shard_ops.gather; the host-driven
 * controller on host collectives): this rank's list, all-gathered */
int op_gather(void* ctx, int32_t kind, uint64_t lo, uint64_t hi, uint64_t* v, int64_t* w, int32_t* n) {
    auto* S = (sw_shard_state*)ctx;
    hipStream_t st = S->h->stream;
    unsigned long long* gl = S->glist.p;
    SH_HIP(S, hipMemsetAsync(gl, 0, 16, st));
    const unsigned pb = nblk((int64_t)S->NL * S->T);
    if (kind == 0)
        LAUNCH(S, k_gather<false>, dim3((unsigned)probe_blocks(pb)), dim3(kTB), 0, st, S->dv, lo, hi, gl);
    else
        LAUNCH(S, k_gather<true>, dim3(pb), dim3(kTB), 0, st, S->dv, lo, hi, gl);
    std::vector<unsigned long long> all((size_t)kGl * S->world);
    SH_TRY(coll_gather(S, gl, S->glall.p, (size_t)kGl * 8, all.data()));
    int32_t k = 0;
    for (int32_t r = 0; r < S->world; ++r) {
        const unsigned long long* L = all.data() + (size_t)r * kGl;
        if (L[0] > (unsigned long long)(SW_GATHER_CAP - k))
            return S->h->err = "search gather: more items than SW_GATHER_CAP", SW_ERR_CAPACITY;
        for (unsigned long long e = 0; e < L[0]; ++e, ++k) {
            v[k] = L[2 + 2 * e];
            w[k] = (int64_t)L[3 + 2 * e];
        }
    }
    *n = k;
    return SW_OK;
}

int op_between(void* ctx, double a, double b, int64_t* out) {
    auto* S = (sw_shard_state*)ctx;
    SH_TRY(zero_red(S, 1));
    SH_TRY(arm_pub(S, S->dv.red, 8));
    LAUNCH(S, k_between, dim3(nblk(S->NL)), dim3(kTB), 0, S->h->stream, S->dv, a, b);
    disarm_pub(S);
    return coll_reduce(S, S->dv.red, 1, 0, out);
}

int op_take_all(void* ctx) {
    auto* S = (sw_shard_state*)ctx;
    LAUNCH(S, k_take_all, dim3(nblk(S->NL)), dim3(kTB), 0, S->h->stream, S->dv);
    return SW_OK;
}

int op_take(void* ctx, uint32_t rho, int64_t* wt, int64_t* excl) {
    auto* S = (sw_shard_state*)ctx;
    SH_TRY(zero_red(S, 2));
    SH_TRY(arm_pub(S, S->dv.red, 16));
    LAUNCH(S, k_take, dim3(nblk(S->NL)), dim3(kTB), 0, S->h->stream, S->dv, rho);
    disarm_pub(S);
    std::vector<int64_t> all((size_t)2 * S->world);
    SH_TRY(coll_gather(S, S->dv.red, S->xrecv.p, 16, all.data()));
    *wt = 0;
    *excl = 0;
    for (int r = 0; r < S->world; ++r) {
        *wt += all[2 * r];
        if (r < S->rank) *excl += all[2 * r + 1];
    }
    return SW_OK;
}

int op_assign(void* ctx, uint32_t rho, int64_t rem, int64_t excl, int64_t* used) {
    auto* S = (sw_shard_state*)ctx;
    SH_TRY(zero_red(S, 1));
    (void)rho; /* k_take stored the tie counts at rho */
    SH_TRY(arm_pub(S, S->dv.red, 8));
    LAUNCH(S, k_assign, dim3(nblk(S->NL)), dim3(kTB), 0, S->h->stream, S->dv, (long long)rem,
           (long long)excl);
    disarm_pub(S);
    return coll_reduce(S, S->dv.red, 1, 0, used);
}

int op_tail_best(void* ctx, int64_t rem2, uint64_t* best) {
    auto* S = (sw_shard_state*)ctx;
    SH_TRY(zero_red(S, 1));
    LAUNCH(S, k_tail_best, dim3(nblk(S->NL)), dim3(kTB), 0, S->h->stream, S->dv, (long long)rem2);
    return coll_reduce(S, S->dv.red, 1, 1, best);
}

int op_tail_apply(void* ctx, int64_t jb) {
    auto* S = (sw_shard_state*)ctx;
    if (jb >= S->off && jb < S->off + S->NL)
        LAUNCH(S, k_tail_apply, dim3(1), dim3(1), 0, S->h->stream, S->dv, (int)(jb - S->off));
    return SW_OK;
}

int op_raise_stats(void* ctx, double M, int64_t out[3]) {
    auto* S = (sw_shard_state*)ctx;
    SH_TRY(zero_red(S, 5));
    SH_TRY(arm_pub(S, S->dv.red, 40));
    LAUNCH(S, k_raise_stats, dim3(nblk(S->NL)), dim3(kTB), 0, S->h->stream, S->dv, M);
    disarm_pub(S);
    /* per rank, gathered: the owner of the first job at M is the lowest rank
     * holding one (ranks hold ascending job ranges) */
    std::vector<unsigned long long> all((size_t)5 * S->world);
    SH_TRY(coll_gather(S, S->dv.red, S->xrecv.p, 40, all.data()));
    int owner = -1;
    out[0] = INT64_MAX;
    out[2] = 0;
    for (int r = 0; r < S->world; ++r) {
        const unsigned long long* b = all.data() + (size_t)5 * r;
        if (owner < 0 && b[0] != 0) { owner = r; out[0] = (int64_t)~b[0]; }
        out[2] += (int64_t)b[4];
    }
    double M2 = 0.0;
    for (int r = 0; r < S->world; ++r) {
        const unsigned long long* b = all.data() + (size_t)5 * r;
        const double v = r == owner ? (b[1] >= 2 ? M : sw_from_bits(b[2])) : sw_from_bits(b[3]);
        M2 = sw_max(M2, v);
    }
    out[1] = (int64_t)sw_bits(M2);
    return SW_OK;
}

int op_raise_best(void* ctx, double M, int64_t i1, double M2, const int64_t* tried, int32_t ntried,
                  uint64_t* best) {
    auto* S = (sw_shard_state*)ctx;
    RaiseTried rt;
    rt.n = ntried < SW_RAISE_TRIES ? ntried : SW_RAISE_TRIES;
    for (int q = 0; q < SW_RAISE_TRIES; ++q) rt.j[q] = q < rt.n ? (long long)tried[q] : -1;
    SH_TRY(zero_red(S, 1));
    SH_TRY(arm_pub(S, S->dv.red, 8));
    LAUNCH(S, k_raise_best, dim3(nblk(S->NL)), dim3(kTB), 0, S->h->stream, S->dv, M, (long long)i1, M2, rt);
    disarm_pub(S);
    return coll_reduce(S, S->dv.red, 1, 1, best);
}

int op_fill_best(void* ctx, const int64_t* load, uint64_t* best) {
    auto* S = (sw_shard_state*)ctx;
    FillLoad L;
    for (int t = 0; t < SW_TMAX; ++t) L.v[t] = t < S->dv.T ? (long long)load[t] : 0;
    SH_TRY(zero_red(S, 1));
    LAUNCH(S, k_fill_best, dim3(nblk(S->NL)), dim3(kTB), 0, S->h->stream, S->dv, L);
    return coll_reduce(S, S->dv.red, 1, 1, best);
}

int op_fill_apply(void* ctx, int64_t jb, int32_t t) {
    auto* S = (sw_shard_state*)ctx;
    if (jb >= S->off && jb < S->off + S->NL)
        LAUNCH(S, k_fill_apply, dim3(1), dim3(1), 0, S->h->stream, S->dv, (int)(jb - S->off), (int)t);
    return SW_OK;
}

/* A reduction step on the stream: k_eval into this rank's block of the
 * gather buffer, gathered in rank order (hout: also to the host).  *view =
 * where the gathered blocks are on the device (the peer transport's region
 * half: read it before the second exchange after this one). */
int eval_enqueue(sw_shard_state* S, int32_t sel, int32_t arg, const double** view, double* hout) {
    const int64_t LW = S->LW, blk = (sel == kEvSelUmax ? 3 : 2) * LW + 2;
    SH_TRY(zero_red(S, 2));
    const int32_t* arr = sel == SW_EV_GMAX || sel == SW_EV_PACKED ? S->arr[arg].p : nullptr;
    const uint64_t* ys = sel == SW_EV_FINAL ? S->y[arg].p : nullptr;
    /* lanes per block: a block's jobs (lpb lanes × q) fit its kTB threads */
    const int lpb = (int)std::max<int64_t>(1, kTB / S->q);
    double* xs = S->xrecv.p + (size_t)S->rank * blk; /* in-place all-gather */
    if (S->q > kTB) return S->h->err = "eval: more than 256 jobs per lane", SW_ERR_CAPACITY;
    if (hout) SH_TRY(arm_pub(S, xs, (size_t)blk * 8));
    LAUNCH(S, k_eval, dim3((unsigned)((LW + lpb - 1) / lpb)), dim3(kTB), 0, S->h->stream, S->dv,
           (int)sel, arr, ys, (int)(arg & 0xFF), (int)(arg >> 8), lpb, xs);
    disarm_pub(S);
    const void* v = S->xrecv.p;
    SH_TRY(coll_gather(S, xs, S->xrecv.p, (size_t)blk * 8, hout, &v));
    if (view) *view = (const double*)v;
    return SW_OK;
}

int op_eval(void* ctx, int32_t sel, int32_t arg, double* lanesA, double* lanesB, double* gm,
            int64_t* isum) {
    auto* S = (sw_shard_state*)ctx;
    const int64_t LW = S->LW, blk = 2 * LW + 2;
    std::vector<double> all((size_t)blk * S->world);
    SH_TRY(eval_enqueue(S, sel, arg, nullptr, all.data()));
    double g = 0.0;
    int64_t s = 0;
    for (int r = 0; r < S->world; ++r) {
        const double* b = all.data() + (size_t)r * blk;
        memcpy(lanesA + r * LW, b, (size_t)LW * 8);
        memcpy(lanesB + r * LW, b + LW, (size_t)LW * 8);
        g = sw_max(g, b[2 * LW]);
        int64_t v;
        memcpy(&v, b + 2 * LW + 1, 8);
        s += v;
    }
    *gm = g;
    *isum = s;
    return SW_OK;
}

/* the controller's array copies: a kernel launch (a D2D hipMemcpyAsync
 * costs the host several times a launch's enqueue, on the solve's critical
 * path between two host-synchronised steps) */
int op_copy(void* ctx, int32_t dst, int32_t src) {
    auto* S = (sw_shard_state*)ctx;
    if (S->NL)
        LAUNCH(S, k_copy_words, dim3(nblk(S->NL)), dim3(kTB), 0, S->h->stream,
               reinterpret_cast<uint32_t*>(S->arr[dst].p), reinterpret_cast<const uint32_t*>(S->arr[src].p),
               (int64_t)S->NL);
    return SW_OK;
}

int op_copy_y(void* ctx, int32_t dst, int32_t src) {
    auto* S = (sw_shard_state*)ctx;
    if (S->NL)
        LAUNCH(S, k_copy_words, dim3(nblk(2 * (int64_t)S->NL)), dim3(kTB), 0, S->h->stream,
               reinterpret_cast<uint32_t*>(S->y[dst].p), reinterpret_cast<const uint32_t*>(S->y[src].p),
               2 * (int64_t)S->NL);
    return SW_OK;
}

/* local: the share placement — only this rank's entries, no gather, caps is
 * this rank's share of every round (mode 4) or its class capacities (mode 5) */
/* local: this rank's entries only (no gather) — the share placement (shares:
 * its shares' device capacities, k_share_caps; one workgroup per share) or a
 * class-wise repack inside a share (jobs [jlo, jhi), caps = the class's
 * capacities) */
int pack_any(sw_shard_state* S, int32_t mode, int32_t src, double Mb, int32_t ydst, int32_t pdst,
             int32_t wc, const int32_t* caps, bool local = false, int32_t* shares = nullptr,
             int32_t jlo = 0, int32_t jhi = 0x7FFFFFFF, const long long* loads = nullptr,
             long long* dfc = nullptr) {
    hipStream_t st = S->h->stream;
    const int nsub = shares ? S->dv.nsub : 1;
    const int64_t Mg = shares ? S->dv.Pp : (local ? S->P : S->P * S->world); /* entries per workgroup */
    const int64_t M = Mg * nsub;
    CapsArg capsd;
    memset(&capsd, 0, sizeof(capsd));
    if (caps) {
        memcpy(capsd.v, caps, (size_t)S->T * 4);
        capsd.has = 1;
    }
    sw_pack_ent* mine = shares ? S->pall.p : S->pall.p + (size_t)S->rank * S->P;
    LAUNCH(S, k_pack_keys, dim3(nblk(shares ? M : S->P)), dim3(kTB), 0, st, S->dv, (int)mode, S->arr[src].p, Mb,
           (int)wc, mine, shares ? 1 : 0, (int)jlo, (int)jhi);
    const void* gv = mine;
    if (!local) /* in-place all-gather: the keys go straight to this rank's block */
        SH_TRY(coll_gather(S, S->pall.p + (size_t)S->rank * S->P, S->pall.p,
                           (size_t)S->P * sizeof(sw_pack_ent), nullptr, &gv));
    const sw_pack_ent* all = (const sw_pack_ent*)gv;
    const int nch = (int)((M + kSortChunk - 1) / kSortChunk);
    LAUNCH(S, k_pack_chunk_sort, dim3(nch), dim3(kSortThreads), 0, st, all, M, S->skeys.p,
           S->sidx.p);
    LAUNCH(S, k_pack_merge_rank, dim3(nblk((int64_t)nch * kSortChunk * kMergeG)), dim3(kTB), 0, st, S->skeys.p,
           S->sidx.p, nch, S->porder.p, (const int32_t*)nullptr, nsub > 1 ? (int)(Mg / kSortChunk) : 0);
    const ShardDev dv = S->dv;
    uint64_t* yd = S->y[ydst].p;
    int32_t* pd = S->arr[pdst].p;
    if (shares) { /* one workgroup per share: the one-wave loop, then the block loop for larger shares */
        const int wa = wave_pack_max();
        if (Mg > (nsub > 1 ? 20 : 64) * SW_BLOCK)
            return S->h->err = "share placement: a share holds more jobs than one workgroup's round loop",
                   SW_ERR_CAPACITY;
        if (loads) { /* both loop forms in one launch, the capacities computed there */
            LAUNCH(S, k_pack_rounds_share, dim3(nsub), dim3(SW_BLOCK), 0, st, dv, all, Mg, S->porder.p, yd, pd,
                   shares, wa, loads, nsub * S->world, (const int32_t*)S->arr[src].p, dfc);
            return SW_OK;
        }
        LAUNCH(S, k_pack_rounds_wave, dim3(nsub), dim3(64), 0, st, dv, all, Mg, S->porder.p, yd, pd, capsd, wa, 1,
               shares);
        if (Mg > wa) {
            if (Mg <= 8 * SW_BLOCK) {
                LAUNCH(S, (k_pack_rounds_sel<SW_BLOCK, 0>), dim3(nsub), dim3(SW_BLOCK), 0, st, dv, all, Mg, S->porder.p,
                       yd, pd, capsd, wa, 1, shares);
            } else if (Mg <= 20 * SW_BLOCK) {
                LAUNCH(S, (k_pack_rounds_sel<SW_BLOCK, 20>), dim3(nsub), dim3(SW_BLOCK), 0, st, dv, all, Mg,
                       S->porder.p, yd, pd, capsd, wa, 1, shares);
            } else { /* one share (nsub = 1) above 20·512 entries: the wide variants */
                LAUNCH(S, (k_pack_rounds_sel<SW_BLOCK, 0>), dim3(1), dim3(SW_BLOCK), 0, st, dv, all, Mg, S->porder.p,
                       yd, pd, capsd, wa, 1, shares);
                if (Mg > 32 * SW_BLOCK)
                    LAUNCH(S, (k_pack_rounds<64, SW_BLOCK>), dim3(1), dim3(SW_BLOCK), 0, st, dv, all, Mg, S->porder.p,
                           yd, pd, capsd, 8 * SW_BLOCK, 1, shares);
                else
                    LAUNCH(S, (k_pack_rounds<32, SW_BLOCK>), dim3(1), dim3(SW_BLOCK), 0, st, dv, all, Mg, S->porder.p,
                           yd, pd, capsd, 8 * SW_BLOCK, 1, shares);
            }
        }
        return SW_OK;
    }
    /* variants by entries M; above 8 positions per thread also the 8-position
     * variant, for instances whose active jobs fit it (k_pack_rounds) */
#define SW_LAUNCH_PACK(E, NT, ALO)                                                              \
    LAUNCH(S, (k_pack_rounds<E, NT>), dim3(1), dim3(NT), 0, st, dv, all, M, S->porder.p, yd, \
           pd, capsd, (int)(ALO), (int)(mode != 5))
    /* the one-wave loop for up to wa active entries, launched when the
     * entries are few enough that most placements fit it (all of them when
     * M ≤ wa: then no block variant is launched) */
    const int wa = wave_pack_max();
    const bool wave = wa > 0 && M <= 4 * (int64_t)wa;
    if (wave)
        LAUNCH(S, k_pack_rounds_wave, dim3(1), dim3(64), 0, st, dv, all, M, S->porder.p, yd, pd, capsd, wa,
               (int)(mode != 5));
    const int lo = wave ? wa : -1;
#define SW_LAUNCH_SEL(NT, EB, ALO)                                                                  \
    LAUNCH(S, (k_pack_rounds_sel<NT, EB>), dim3(1), dim3(NT), 0, st, dv, all, M, S->porder.p, yd, pd, \
           capsd, (int)(ALO), (int)(mode != 5))
    /* measured on C4's share placement (profiles/r7nt1_*): E by the active
     * entries in one launch against E by the entries, rank loop 148 → 125 µs
     * at W = 2 and 122 → 90 µs at W = 4; 256-thread loops (4 waves, twice the
     * positions per thread) were slower at W = 1 (0.729 against 0.706 ms) */
    if (wave && M <= wa) {
    } else if (M <= 64 * SW_BLOCK) {
        /* E by the active entries: one launch up to 8·512 of them */
        if (M <= 8 * SW_BLOCK) {
            SW_LAUNCH_SEL(SW_BLOCK, 0, lo);
        } else if (M <= 20 * SW_BLOCK) {
            SW_LAUNCH_SEL(SW_BLOCK, 20, lo);
        } else {
            SW_LAUNCH_SEL(SW_BLOCK, 0, lo);
            if (M > 32 * SW_BLOCK) SW_LAUNCH_PACK(64, SW_BLOCK, 8 * SW_BLOCK);
            else SW_LAUNCH_PACK(32, SW_BLOCK, 8 * SW_BLOCK);
        }
    } else {
        return S->h->err = "sharded placement holds at most 32768 jobs", SW_ERR_CAPACITY;
    }
#undef SW_LAUNCH_PACK
#undef SW_LAUNCH_SEL
    return SW_OK;
}

int op_pack(void* ctx, int32_t mode, int32_t src, double Mb, int32_t ydst, int32_t pdst) {
    return pack_any((sw_shard_state*)ctx, mode, src, Mb, ydst, pdst, 0, nullptr);
}

/* twin: e_pack_share (oracle/shard_twin.c) — the shares' loads all-gathered,
 * every share's capacities computed on the device (k_share_caps), this
 * rank's shares placed side by side, one workgroup each: no host round trip */
int pack_share_any(sw_shard_state* S, int32_t src, int32_t ydst, int32_t pdst, long long** dfc);

int op_pack_share(void* ctx, int32_t src, int32_t ydst, int32_t pdst) {
    return pack_share_any((sw_shard_state*)ctx, src, ydst, pdst, nullptr);
}

/* dfc (fast_solve): a zeroed step slot that receives Σ w·(src − placed) over
 * this rank's rows, summed by the loop kernel (one-launch shares only; else
 * nullptr comes back and the caller evaluates PACKED) */
int pack_share_any(sw_shard_state* S, int32_t src, int32_t ydst, int32_t pdst, long long** dfc) {
    hipStream_t st = S->h->stream;
    const int nsub = S->dv.nsub;
    SH_TRY(zero_red(S, nsub));
    LAUNCH(S, k_load, dim3(nblk(S->NL)), dim3(kTB), 0, st, S->dv, S->arr[src].p);
    const void* lv = S->dv.red; /* world 1: this rank's loads are every load */
    if (S->world > 1) {
        long long* lrecv = reinterpret_cast<long long*>(S->xrecv.p);
        SH_TRY(coll_gather(S, S->dv.red, lrecv, (size_t)nsub * 8, nullptr, &lv));
    }
    /* shares of at most 8·512 entries: k_pack_rounds_share computes its
     * capacities itself; larger ones take k_share_caps and the separate
     * loop variants */
    const bool one = S->dv.Pp <= 8 * SW_BLOCK;
    if (!one)
        LAUNCH(S, k_share_caps, dim3(1), dim3(64), 0, st, (const long long*)lv, nsub * S->world, S->rank, nsub,
               S->T, (long long)S->dv.G, S->scapsd.p);
    long long* slot = nullptr;
    if (dfc) {
        *dfc = nullptr;
        if (one) {
            SH_TRY(zero_red(S, 1));
            slot = S->dv.red;
            *dfc = slot;
        }
    }
    return pack_any(S, 4, src, 0.0, ydst, pdst, 0, nullptr, true, S->scapsd.p, 0, 0x7FFFFFFF,
                    one ? (const long long*)lv : nullptr, slot);
}

/* twin: e_share_repair — each of this rank's shares whose pack stranded
 * rounds has its width profile repaired inside the share (host:
 * sw_profile_repair), every changed class repacked alone (local, the share's
 * jobs only) */
int op_share_repair(void* ctx, int32_t src, int32_t ydst, int32_t pdst) {
    auto* S = (sw_shard_state*)ctx;
    if (S->NL <= 0) return SW_OK;
    const int32_t NL = S->NL, T = S->T, nsub = S->dv.nsub;
    std::vector<uint64_t> y((size_t)NL);
    std::vector<int32_t> n((size_t)NL), pl((size_t)NL), w((size_t)NL), caps((size_t)SW_VSHARES * 64 + 64);
    hipStream_t st = S->h->stream;
    SH_HIP(S, hipMemcpyAsync(caps.data(), S->scapsd.p, caps.size() * 4, hipMemcpyDeviceToHost, st));
    SH_HIP(S, hipMemcpyAsync(y.data(), S->y[ydst].p, (size_t)NL * 8, hipMemcpyDeviceToHost, st));
    SH_HIP(S, hipMemcpyAsync(n.data(), S->arr[src].p, (size_t)NL * 4, hipMemcpyDeviceToHost, st));
    SH_HIP(S, hipMemcpyAsync(pl.data(), S->arr[pdst].p, (size_t)NL * 4, hipMemcpyDeviceToHost, st));
    SH_HIP(S, hipMemcpyAsync(w.data(), S->in_w, (size_t)NL * 4, hipMemcpyDeviceToHost, st));
    SH_HIP(S, hipStreamSynchronize(st));
    if (caps[(size_t)SW_VSHARES * 64] == 0) return SW_OK; /* no shares */
    for (int32_t sh = 0; sh < nsub; ++sh) {
        const int32_t lo = (int32_t)std::min<int64_t>(NL, sh * S->dv.Ps),
                      hi = (int32_t)std::min<int64_t>(NL, (sh + 1) * S->dv.Ps);
        int64_t dfc = 0;
        for (int32_t i = lo; i < hi; ++i) dfc += (int64_t)w[i] * (n[i] - pl[i]);
        if (dfc == 0) continue;
        sw_repair_t R;
        memset(&R, 0, sizeof(R));
        bool over = false;
        for (int32_t i = lo; i < hi && !over; ++i)
            if (n[i] > 0 && sw_repair_add_class(&R, w[i]) < 0) over = true;
        if (over) continue;
        for (int32_t t = 0; t < T; ++t) R.L[t] = caps[(size_t)sh * 64 + t];
        for (int32_t i = lo; i < hi; ++i) {
            for (int32_t t = 0; t < T; ++t)
                if ((y[i] >> t) & 1u) R.L[t] -= w[i];
            if (n[i] <= 0) continue;
            const int32_t c = sw_repair_class(&R, w[i]);
            R.M[c] += 1;
            R.D[c] += n[i] - pl[i];
            for (int32_t t = 0; t < T; ++t) R.caps[c][t] += (int32_t)((y[i] >> t) & 1u);
        }
        if (sw_profile_repair(&R, T) != 0) continue;
        for (int32_t c = 0; c < R.ncls; ++c) {
            if (!R.changed[c]) continue;
            SH_TRY(pack_any(S, 5, src, 0.0, ydst, pdst, R.wc[c], R.caps[c], true, nullptr, lo, hi));
        }
    }
    return SW_OK;
}

int op_pack_class(void* ctx, int32_t src, int32_t wc, const int32_t* caps, int32_t ydst,
                  int32_t pdst) {
    return pack_any((sw_shard_state*)ctx, 5, src, 0.0, ydst, pdst, wc, caps);
}

int op_class_caps(void* ctx, int32_t src, int32_t ysrc, int32_t wc, int32_t psrc, int32_t* caps,
                  int32_t* next_w, int64_t* md) {
    auto* S = (sw_shard_state*)ctx;
    SH_TRY(zero_red(S, 67));
    LAUNCH(S, k_class_caps, dim3(nblk(S->NL)), dim3(kTB), 0, S->h->stream, S->dv, S->arr[src].p,
           S->y[ysrc].p, (int)wc, psrc >= 0 ? (const int32_t*)S->arr[psrc].p : nullptr,
           (int)(psrc == SW_CLASS_HIST));
    int64_t cnt[64];
    uint64_t nx = 0;
    SH_TRY(coll_reduce(S, S->dv.red, S->T, 0, cnt));
    SH_TRY(coll_reduce(S, S->dv.red + 64, 1, 1, &nx));
    SH_TRY(coll_reduce(S, S->dv.red + 65, 2, 0, md));
    for (int t = 0; t < S->T; ++t) caps[t] = (int32_t)cnt[t];
    *next_w = nx == 0 ? 0x7FFFFFFF : (int32_t)(0xFFFFFFFFull - nx);
    return SW_OK;
}

/* twin: e_p2x (oracle/shard_twin.c) — gather the P2 placement, run the
 * exchange step replicated, keep this rank's rows */
/* the exchange step on the stream; *res = the step slot whose [0] receives
 * the cycles cancelled (the same on every rank); arm: publish it (world 1) */
int p2x_enqueue(sw_shard_state* S, int32_t ysrc, int32_t nsrc, long long** res, bool arm,
                const long long* skip = nullptr) {
    hipStream_t st = S->h->stream;
    const int64_t M = S->P * S->world;
    p2x_ent* mine = reinterpret_cast<p2x_ent*>(S->pall.p + (size_t)S->rank * S->P);
    const int T = S->T;
    const bool prepared = M > SW_BLOCK && M <= SW_P2X_AMAX * 4;
    /* workspace after the X arrays (prepared set-up): hdr, ord, pc, bitsets, Wb, Wk, block counts,
     * width counts */
    const size_t xa = ((size_t)M * SW_P2X_ARR_BYTES + 15) & ~(size_t)15;
    const size_t words = (size_t)T * ((size_t)(M + 63) / 64 + SW_P2X_KMAX);
    const size_t need = xa + 256 + (size_t)M * 4 + (size_t)M * 8 + words * 8 +
                        (size_t)SW_P2X_KMAX * T * T * 9 + 64 + (size_t)nblk(M) * 4 + 16 + 257 * 4 + 16;
    if (S->p2ws.reserve(prepared ? need : (size_t)M * SW_P2X_ARR_BYTES) || (prepared && S->p2keys.reserve((size_t)M)))
        return host_fail(S, "P2 exchange workspace");
    unsigned char* base = S->p2ws.p + xa;
    int32_t* hdr = reinterpret_cast<int32_t*>(base);
    int32_t* ord = reinterpret_cast<int32_t*>(base + 256);
    double* pc = reinterpret_cast<double*>(base + 256 + (((size_t)M * 4 + 15) & ~(size_t)15));
    uint64_t* B = reinterpret_cast<uint64_t*>(pc + M);
    double* Wb = reinterpret_cast<double*>(B + words);
    int8_t* Wk = reinterpret_cast<int8_t*>(Wb + (size_t)SW_P2X_KMAX * T * T);
    int32_t* bcnt = reinterpret_cast<int32_t*>(Wk + (size_t)SW_P2X_KMAX * T * T);
    uint32_t* wmap = reinterpret_cast<uint32_t*>(hdr + SW_P2X_HDR_INTS);
    const int nb = nblk(M);
    int32_t* wcnt = bcnt + nb; /* 256 width counts + the finish counter */
    /* world 1: nothing to gather, so the entry kernel also counts (k_p2x_cnt) */
    const bool fold = prepared && S->world == 1 && nblk(S->P) == nb;
    LAUNCH(S, k_p2x_ent, dim3(nblk(S->P)), dim3(kTB), 0, st, S->dv, S->y[ysrc].p, S->arr[nsrc].p, mine,
           fold ? bcnt : nullptr, fold ? wmap : nullptr, fold ? wcnt : nullptr);
    const void* gv = nullptr;
    SH_TRY(coll_gather(S, mine, S->pall.p, (size_t)S->P * sizeof(p2x_ent), nullptr, &gv));
    SH_TRY(zero_red(S, 1));
    const int maxA = (int)std::min<int64_t>(M, SW_P2X_AMAX);
    const size_t lds = ((sizeof(sw_p2x_lds) + 15) & ~(size_t)15) + sw_p2x_var_bytes(maxA, S->T);
    /* the set-up by several workgroups (k_p2x_pre*) when the gathered entries
     * fill more than one workgroup's sort: the step's own workgroup then
     * starts from the prepared state */
    sw_p2x_pre pre;
    memset(&pre, 0, sizeof(pre));
    if (prepared) {
        if (!fold) LAUNCH(S, k_p2x_cnt, dim3(nb), dim3(kTB), 0, st, (const p2x_ent*)gv, M, bcnt, wmap, wcnt);
        LAUNCH(S, k_p2x_compact, dim3(nb), dim3(kTB), 0, st, (const p2x_ent*)gv, M, bcnt, S->p2ws.p, wmap,
               hdr, wcnt, T);
        LAUNCH(S, k_p2x_keys, dim3(nb), dim3(kTB), 0, st, S->p2ws.p, M, hdr, S->p2keys.p);
        /* the active keys only: chunks past A exit, the merge ranks against ⌈A / 1024⌉ chunks */
        const int nch = (int)((M + kSortChunk - 1) / kSortChunk);
        LAUNCH(S, k_pack_chunk_sort, dim3(nch), dim3(kSortThreads), 0, st, S->p2keys.p, M, S->skeys.p,
               S->sidx.p, (const int32_t*)(hdr + SW_P2X_HDR_A));
        LAUNCH(S, k_pack_merge_rank, dim3(nblk((int64_t)nch * kSortChunk * kMergeG)), dim3(kTB), 0, st, S->skeys.p,
               S->sidx.p, nch, S->porder.p, (const int32_t*)(hdr + SW_P2X_HDR_A));
        const int64_t slots = (M + 63) / 64 + SW_P2X_KMAX;
        LAUNCH(S, k_p2x_pre_bits, dim3(nblk(slots * 64)), dim3(kTB), 0, st, hdr, S->porder.p, S->p2ws.p,
               M, T, ord, pc, B);
        LAUNCH(S, k_p2x_pre_w, dim3(nblk((int64_t)SW_P2X_KMAX * T * T * 64)), dim3(kTB), 0, st, hdr, pc, B, T,
               Wb, Wk);
        pre.hdr = hdr;
        pre.ord = ord;
        pre.pc = pc;
        pre.B = B;
        pre.Wb = Wb;
        pre.Wk = Wk;
    }
    if (arm) SH_TRY(arm_pub(S, S->dv.red, 8));
    LAUNCH(S, k_p2x, dim3(1), dim3(SW_BLOCK), lds, st, S->dv, (const p2x_ent*)gv, M, S->p2ws.p,
           S->y[ysrc].p, pre, (int)prepared, skip);
    disarm_pub(S);
    *res = S->dv.red;
    return SW_OK;
}

int op_p2x(void* ctx, int32_t ysrc, int32_t nsrc, int32_t* cancels) {
    auto* S = (sw_shard_state*)ctx;
    long long* r = nullptr;
    SH_TRY(p2x_enqueue(S, ysrc, nsrc, &r, true));
    uint64_t nc = 0;
    SH_TRY(coll_reduce(S, S->dv.red, 1, 1, &nc)); /* every rank computed the same count */
    *cancels = (int32_t)nc;
    return SW_OK;
}

/* twin: e_reround (oracle/shard_twin.c) — gather the P1 plan and every job's
 * inputs, run the re-optimisation replicated, keep this rank's rows */
int op_reround(void* ctx, int32_t* moves) {
    auto* S = (sw_shard_state*)ctx;
    hipStream_t st = S->h->stream;
    const int64_t M = S->P * S->world;
    const size_t Mj = (size_t)std::max<int64_t>(S->N, 1);
    const size_t wsb = ((Mj * sizeof(sw_jobc) + 15) & ~(size_t)15) + 8 * Mj * 4 + 8 * SW_RR_WORDS +
                       4 * Mj + 4 * SW_RR_WORDS + 2 * Mj + 16;
    if (S->rrin.reserve((size_t)M * sizeof(rr_in)) || S->rrrow.reserve((size_t)M * sizeof(rr_row)) ||
        S->rrws.reserve(wsb))
        return host_fail(S, "re-optimisation workspace");
    rr_in* in_all = reinterpret_cast<rr_in*>(S->rrin.p);
    rr_row* row_all = reinterpret_cast<rr_row*>(S->rrrow.p);
    rr_in* in_mine = in_all + (size_t)S->rank * S->P;
    rr_row* row_mine = row_all + (size_t)S->rank * S->P;
    LAUNCH(S, k_rr_ent, dim3(nblk(S->P)), dim3(kTB), 0, st, S->dv, S->in_w, S->in_F, S->in_E,
           S->in_d, S->in_R, S->in_p, in_mine, row_mine);
    /* in place: each rank's block is already where the gather puts it */
    SH_TRY(coll_gather(S, in_mine, in_all, (size_t)S->P * sizeof(rr_in), nullptr));
    SH_TRY(coll_gather(S, row_mine, row_all, (size_t)S->P * sizeof(rr_row), nullptr));
    SH_TRY(zero_red(S, 1));
    const size_t lds = ((sizeof(sw_xchg) + 15) & ~(size_t)15) + 2 * 8 * (SW_RR_CAPMAX + 1) +
                       8 * SW_RR_WORDS;
    LAUNCH(S, k_rr, dim3(1), dim3(SW_BLOCK), lds, st, S->dv, S->delta, (const rr_in*)in_all,
           (const rr_row*)row_all, S->rrws.p);
    uint64_t mv = 0;
    SH_TRY(coll_reduce(S, S->dv.red, 1, 1, &mv)); /* every rank computed the same count */
    *moves = (int32_t)mv;
    return SW_OK;
}

/* Reserve the per-solve buffers and upload this rank's jobs. */
int prepare(sw_shard_state* S, const sw_problem* pr, int64_t off, int64_t N, bool dev,
            const sw_result* res) {
    hipStream_t st = S->h->stream;
    S->NL = pr->num_jobs;
    S->T = pr->future_rounds;
    S->N = N;
    S->off = off;
    S->q = (N + SW_DET_LANES - 1) / SW_DET_LANES;
    if (S->q == 0) S->q = 1;
    S->LW = SW_DET_LANES / S->world;
    S->P = S->LW * S->q;
    S->delta = pr->round_duration;
    const int32_t V = sw_share_count(N, pr->num_gpus, S->world);
    const int32_t nsub = V / S->world;
    const int64_t Ps = nsub > 1 ? (int64_t)(SW_DET_LANES / V) * S->q : S->P;
    const int64_t Pp = nsub > 1 ? (Ps + kSortChunk - 1) / kSortChunk * kSortChunk : S->P;
    const size_t NL = (size_t)std::max<int32_t>(S->NL, 1), T = (size_t)S->T;
    const size_t M = std::max<size_t>((size_t)S->P * S->world, (size_t)(nsub * Pp));
    const size_t Mpad = (M + kSortChunk - 1) / kSortChunk * kSortChunk;
    const size_t xbytes = std::max<size_t>({(size_t)(3 * S->LW + 2) * 8, (size_t)S->P * 4, 16});
    bool bad = S->w.reserve(NL) || S->F.reserve(NL) || S->E.reserve(NL) || S->d.reserve(NL) ||
               S->R.reserve(NL) || S->p.reserve(NL) || S->jc.reserve(NL) || S->keys.reserve(NL * T) ||
               S->l.reserve(NL) || S->taken.reserve(NL) || S->tie.reserve(NL) ||
               S->tieblk.reserve(nblk((int64_t)NL)) ||
               S->xa.reserve(2 * NL) || S->plan.reserve(NL * T) ||
               S->planned.reserve(NL) || S->red.reserve((size_t)kRed * kRing) ||
               S->xrecv.reserve((xbytes / 8 + 1) * S->world) || S->pall.reserve(M) ||
               S->porder.reserve(M) || 
               S->srch.reserve(4 * kSt) || S->glist.reserve(2 * (size_t)kGl) ||
               S->glall.reserve((size_t)kGl * S->world) || S->fctl.reserve(1) || S->scapsd.reserve((size_t)SW_VSHARES * 64 + 64) ||
               S->skeys.reserve(Mpad) || S->sidx.reserve(Mpad);
    for (int a = 0; a < SW_A_COUNT; ++a) bad = bad || S->arr[a].reserve(NL);
    for (int a = 0; a < SW_Y_COUNT; ++a) bad = bad || S->y[a].reserve(NL);
    if (bad || S->hx.reserve(std::max<size_t>(xbytes * S->world, kRed * 8)))
        return S->h->err = "shard allocation failed", SW_ERR_HIP;
    if (dev) {
        S->in_w = pr->nworkers; S->in_F = pr->completed_epochs; S->in_E = pr->total_epochs;
        S->in_d = pr->epoch_duration; S->in_R = pr->remaining_runtime; S->in_p = pr->priority;
        S->zero_pending = S->NL > 0;
    } else {
        S->in_w = S->w.p; S->in_F = S->F.p; S->in_E = S->E.p;
        S->in_d = S->d.p; S->in_R = S->R.p; S->in_p = S->p.p;
    }
    if (S->NL && !dev) {
        const size_t n = (size_t)S->NL;
        SH_HIP(S, hipMemcpyAsync(S->w.p, pr->nworkers, n * 4, hipMemcpyHostToDevice, st));
        SH_HIP(S, hipMemcpyAsync(S->F.p, pr->completed_epochs, n * 4, hipMemcpyHostToDevice, st));
        SH_HIP(S, hipMemcpyAsync(S->E.p, pr->total_epochs, n * 4, hipMemcpyHostToDevice, st));
        SH_HIP(S, hipMemcpyAsync(S->d.p, pr->epoch_duration, n * 8, hipMemcpyHostToDevice, st));
        SH_HIP(S, hipMemcpyAsync(S->R.p, pr->remaining_runtime, n * 8, hipMemcpyHostToDevice, st));
        SH_HIP(S, hipMemcpyAsync(S->p.p, pr->priority, n * 8, hipMemcpyHostToDevice, st));
        S->zero_pending = true; /* k_zero_state once the kernel view is built */
    }
    ShardDev& v = S->dv;
    memset(&v, 0, sizeof(v));
    v.NL = S->NL; v.T = S->T; v.G = pr->num_gpus; v.nb = pr->num_bases;
    v.LW = (int32_t)S->LW; v.rank = S->rank;
    v.off = off; v.N = N; v.q = S->q; v.P = S->P;
    v.nsub = nsub; v.Ps = Ps; v.Pp = Pp;
    v.k = pr->regularizer;
    for (int b = 0; b < SW_BMAX; ++b) {
        v.beta[b] = b < pr->num_bases ? pr->bases[b] : 0.0;
        v.ell[b] = b < pr->num_bases ? pr->log_bases[b] : 0.0;
    }
    sw_pwl_slopes(pr->num_bases, pr->bases, pr->log_bases, v.slope);
    v.jc = S->jc.p; v.keys = S->keys.p; v.p = S->in_p; v.l = S->l.p; v.taken = S->taken.p;
    v.tie = S->tie.p; v.tieblk = S->tieblk.p; v.xa = S->xa.p;
    for (int a = 0; a < SW_A_COUNT; ++a) v.arr[a] = S->arr[a].p;
    for (int a = 0; a < SW_Y_COUNT; ++a) v.y[a] = S->y[a].p;
    v.plan = S->plan.p; v.planned = S->planned.p; v.red = S->red.p;
    if (dev && res->plan) v.plan = res->plan; /* the final step writes the caller's HBM */
    if (dev && res->planned_rounds) v.planned = res->planned_rounds;
    S->ring_pos = kRing; /* the first step clears the ring */
    if (S->zero_pending) { /* the state, and the ring with it */
        LAUNCH(S, k_zero_state, dim3(nblk(std::max<int64_t>(S->NL, (int64_t)kRing * kRed))), dim3(kTB), 0, st,
               v);
        S->zero_pending = false;
        S->ring_pos = 0;
    }
    return SW_OK;
}

int shard_attach(sw_handle* h, int32_t rank, int32_t world) {
    if (!h) return SW_ERR_INVALID;
    int64_t lo, hi;
    if (sw_shard_range(0, world, rank, &lo, &hi) != 0)
        return h->err = "world must divide 512 and 0 <= rank < world", SW_ERR_INVALID;
    sw_shard_release(h);
    h->shard = new (std::nothrow) sw_shard_state();
    if (!h->shard) return h->err = "out of host memory", SW_ERR_HIP;
    h->shard->h = h;
    h->shard->rank = rank;
    h->shard->world = world;
    return SW_OK;
}

}  // namespace

void sw_shard_release(sw_handle* h) {
    if (!h || !h->shard) return;
    sw_shard_state* S = h->shard;
    if (S->comm) (void)ncclCommDestroy(S->comm);
    for (int p = 0; p < SW_PEER_MAX_WORLD; ++p)
        if (S->opened[p]) (void)hipIpcCloseMemHandle(S->opened[p]);
    if (S->xreg) (void)hipFree(S->xreg);
    if (S->xerr) (void)hipFree(S->xerr);
    S->w.release(); S->F.release(); S->E.release(); S->l.release(); S->taken.release();
    S->tie.release(); S->tieblk.release(); S->xa.release();
    S->planned.release(); S->porder.release(); S->d.release(); S->R.release();
    S->p.release(); S->xrecv.release(); S->jc.release(); S->keys.release();
    S->plan.release(); S->red.release(); S->pall.release(); S->p2ws.release(); S->rrin.release(); S->rrrow.release(); S->rrws.release(); S->hx.release();
    if (S->pub) (void)hipHostFree(S->pub);
    if (S->pub_flag) (void)hipHostFree(S->pub_flag);
    S->pub = nullptr; S->pub_flag = nullptr; S->pub_words = 0;
    S->p2keys.release();
    S->srch.release(); S->glist.release(); S->glall.release(); S->skeys.release(); S->sidx.release(); S->scapsd.release(); S->fctl.release();
    for (int a = 0; a < SW_A_COUNT; ++a) S->arr[a].release();
    for (int a = 0; a < SW_Y_COUNT; ++a) S->y[a].release();
    delete S;
    h->shard = nullptr;
}

extern "C" {

#ifdef SW_STAMPS
/* Diagnostic builds only (not part of include/shockwave_amd.h): round-loop
 * phase cycles and counters (24 words, sw_pack.h SWP_FLUSH) accumulated since
 * the last call (which also clears them). */
int sw_debug_pack_stamps(uint64_t* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sw_pack_stamps), 24 * sizeof(uint64_t)) != hipSuccess)
        return SW_ERR_HIP;
    uint64_t z[24] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_sw_pack_stamps), z, sizeof(z)) == hipSuccess ? SW_OK : SW_ERR_HIP;
}
#endif

int sw_dist_shard_range(int64_t total_jobs, int32_t world, int32_t rank, int64_t* lo, int64_t* hi) {
    if (!lo || !hi) return SW_ERR_INVALID;
    return sw_shard_range(total_jobs, world, rank, lo, hi) == 0 ? SW_OK : SW_ERR_INVALID;
}

int sw_dist_unique_id(void* out_bytes) {
    if (!out_bytes) return SW_ERR_INVALID;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return SW_ERR_RCCL;
    memcpy(out_bytes, id.internal, SW_NCCL_UNIQUE_ID_BYTES);
    return SW_OK;
}

int sw_dist_init(sw_handle* h, const void* unique_id, int32_t rank, int32_t world) {
    if (!h || !unique_id) return SW_ERR_INVALID;
    SH_TRY(shard_attach(h, rank, world));
    {
        /* world 1 too: the collectives then run through RCCL as at world > 1 */
        ncclUniqueId id;
        memcpy(id.internal, unique_id, SW_NCCL_UNIQUE_ID_BYTES);
        if (hipSetDevice(h->device) != hipSuccess) return h->err = "hipSetDevice", SW_ERR_HIP;
        ncclResult_t r = ncclCommInitRank(&h->shard->comm, world, id, rank);
        if (r != ncclSuccess) {
            h->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
            h->shard->comm = nullptr;
            sw_shard_release(h);
            return SW_ERR_RCCL;
        }
    }
    return SW_OK;
}

int sw_dist_init_host(sw_handle* h, const sw_host_comm* comm, int32_t rank, int32_t world) {
    if (!h || !comm || !comm->allreduce_sum_i64 || !comm->allreduce_max_u64 ||
        !comm->allreduce_max_f64 || !comm->allgather)
        return SW_ERR_INVALID;
    SH_TRY(shard_attach(h, rank, world));
    h->shard->host_comm = true;
    h->shard->hc = *comm;
    return SW_OK;
}

}  // extern "C"

/* Region slot bytes for instances up to `jobs` jobs at world W: the largest
 * step payload — the placement entries (P·24 B), the lane partials
 * ((3·LW + 2)·8 B with the fast path's third sum), the widths (P·4 B) or a
 * ≤ kRed-value all-reduce. */
static long long peer_slot_bytes(int64_t jobs, int32_t W) {
    const int64_t q = std::max<int64_t>(1, (jobs + SW_DET_LANES - 1) / SW_DET_LANES);
    const int64_t LW = SW_DET_LANES / W, P = LW * q;
    long long b = std::max<long long>({(long long)P * (long long)sizeof(sw_pack_ent), (3 * LW + 2) * 8,
                                       P * 4, (long long)kRed * 8, (long long)kGl * 8});
    return (b + 255) / 256 * 256;
}

int sw_dist_enable_peer(sw_handle* h, int64_t max_total_jobs) {
    if (!h || !h->shard || max_total_jobs < 0) return SW_ERR_INVALID;
    sw_shard_state* S = h->shard;
    const int32_t W = S->world;
    /* world 1: nothing to exchange, the init call's transport stays (an
     * exchange with itself measured 0.68-0.70 ms per C4 solve against 0.63 ms
     * on RCCL: its system-scope fences cost more than RCCL's identity call) */
    if (W == 1) return SW_OK;
    if (W > SW_PEER_MAX_WORLD) return h->err = "peer transport: world exceeds SW_PEER_MAX_WORLD", SW_ERR_INVALID;
    if (S->peer) return h->err = "peer transport already enabled", SW_ERR_INVALID;
    if (hipSetDevice(h->device) != hipSuccess) return h->err = "hipSetDevice", SW_ERR_HIP;
    if (!S->host_comm && !S->comm)
        return h->err = "peer transport: sw_dist_init or sw_dist_init_host first", SW_ERR_INVALID;
    /* an all-gather on the init call's collective (setup only) */
    auto gather = [&](const void* send, void* recv, size_t n) -> int {
        if (S->host_comm)
            return S->hc.allgather(S->hc.ctx, send, recv, (int64_t)n) ? host_fail(S, "peer setup all-gather")
                                                                       : SW_OK;
        DevBuf<unsigned char> ds, dr;
        if (ds.reserve(n) || dr.reserve(n * (size_t)W)) return h->err = "peer setup: allocation", SW_ERR_HIP;
        SH_HIP(S, hipMemcpy(ds.p, send, n, hipMemcpyHostToDevice));
        SH_NCCL(S, ncclAllGather(ds.p, dr.p, n, ncclUint8, S->comm, h->stream));
        SH_HIP(S, hipStreamSynchronize(h->stream));
        SH_HIP(S, hipMemcpy(recv, dr.p, n * (size_t)W, hipMemcpyDeviceToHost));
        return SW_OK;
    };
    auto undo = [&]() {
        for (int p = 0; p < SW_PEER_MAX_WORLD; ++p)
            if (S->opened[p]) { (void)hipIpcCloseMemHandle(S->opened[p]); S->opened[p] = nullptr; }
        if (S->xreg) (void)hipFree(S->xreg);
        if (S->xerr) (void)hipFree(S->xerr);
        S->xreg = nullptr;
        S->xerr = nullptr;
    };
    const long long slot = peer_slot_bytes(max_total_jobs, W);
    const long long half = slot * W;
    const size_t bytes = (size_t)kXHdr + 2 * (size_t)half;
    /* every rank: {ok, process identity, device, region pointer, IPC handle}.
     * A local failure is carried through both all-gathers instead of
     * returning early, so that every rank reaches them and all ranks keep the
     * init call's transport together when any rank could not set up its side.
     * Process identity = a per-process random nonce (drawn once) plus the
     * kernel's boot id: ranks in different containers can share a PID, never
     * both of these, so the raw-pointer path is taken only inside one process. */
    struct Rec {
        long long ok, device;
        unsigned long long nonce[2];
        char boot[40];
        unsigned long long ptr;
        hipIpcMemHandle_t ih;
    };
    Rec mine;
    memset(&mine, 0, sizeof(mine));
    process_identity(mine.nonce, mine.boot, sizeof(mine.boot));
    mine.device = h->device;
    if (const char* e = getenv("SW_PEER_TIMEOUT_MS")) {
        const long long ms = atoll(e);
        if (ms > 0) S->xtimeout = (unsigned long long)ms * 100000ull;
    }
    {
        /* fine-grained device memory: peers write it over xGMI, and this
         * GPU's L2 must not hold stale copies of those lines.  Coarse-grained
         * memory could serve stale lines, so without fine-grained memory the
         * setup fails and every rank keeps the init transport. */
        void* reg = nullptr;
        if (hipExtMallocWithFlags(&reg, bytes, hipDeviceMallocFinegrained) != hipSuccess) {
            (void)hipGetLastError();
            reg = nullptr;
        }
        S->xreg = (unsigned char*)reg;
        bool ok = reg != nullptr && hipMemset(reg, 0, bytes) == hipSuccess &&
                  hipMalloc((void**)&S->xerr, sizeof(int)) == hipSuccess &&
                  hipMemset(S->xerr, 0, sizeof(int)) == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
                  hipIpcGetMemHandle(&mine.ih, reg) == hipSuccess;
        mine.ok = ok ? 1 : 0;
        mine.ptr = (unsigned long long)(uintptr_t)reg;
        (void)hipGetLastError();
    }
    std::vector<Rec> all((size_t)W);
    {
        const int rc = gather(&mine, all.data(), sizeof(Rec));
        if (rc < 0) { undo(); return rc; }
    }
    long long ok = 1;
    for (int32_t p = 0; p < W; ++p) ok &= all[(size_t)p].ok;
    /* Ranks of this process on this device wait for each other INSIDE their
     * exchange kernels, so each needs a hardware queue of its own: a waiting
     * kernel queued in front of a peer's kernel blocks it until the timeout.
     * HIP maps a process's streams round robin onto GPU_MAX_HW_QUEUES queues
     * (4 by default), and the process holds other streams too (the handles'
     * copy streams, torch's, RCCL's), so at most half of them may carry
     * same-device ranks: more is refused up front, on every rank alike. */
    int32_t same = 0;
    for (int32_t p = 0; p < W; ++p)
        same += all[(size_t)p].nonce[0] == mine.nonce[0] && all[(size_t)p].nonce[1] == mine.nonce[1] &&
                memcmp(all[(size_t)p].boot, mine.boot, sizeof(mine.boot)) == 0 &&
                all[(size_t)p].device == mine.device;
    int32_t hwq = 4;
    if (const char* e = getenv("GPU_MAX_HW_QUEUES")) {
        const int v = atoi(e);
        if (v > 0) hwq = v;
    }
    const bool queues_short = same > 1 && same > hwq / 2;
    if (queues_short) ok = 0;
    for (int32_t p = 0; p < W && ok; ++p) {
        if (p == S->rank) {
            S->ps.base[p] = S->xreg;
        } else if (all[(size_t)p].nonce[0] == mine.nonce[0] && all[(size_t)p].nonce[1] == mine.nonce[1] &&
                   memcmp(all[(size_t)p].boot, mine.boot, sizeof(mine.boot)) == 0) {
            /* same process: the pointer itself; another device needs peer access */
            if (all[(size_t)p].device != mine.device) {
                const hipError_t pe = hipDeviceEnablePeerAccess((int)all[(size_t)p].device, 0);
                if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) {
                    (void)hipGetLastError();
                    ok = 0;
                    break;
                }
                (void)hipGetLastError();
            }
            S->ps.base[p] = (unsigned char*)(uintptr_t)all[(size_t)p].ptr;
        } else {
            void* q = nullptr;
            if (hipIpcOpenMemHandle(&q, all[(size_t)p].ih, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                (void)hipGetLastError();
                ok = 0;
                break;
            }
            S->opened[p] = q;
            S->ps.base[p] = (unsigned char*)q;
        }
    }
    /* 1 = mapped, 0 = could not map, -1 = refused for lack of hardware queues */
    long long st = queues_short ? -1 : ok;
    std::vector<long long> oks((size_t)W);
    {
        const int rc = gather(&st, oks.data(), sizeof(long long));
        if (rc < 0) { undo(); return rc; }
    }
    bool refused = false;
    for (int32_t p = 0; p < W; ++p) {
        refused |= oks[(size_t)p] < 0;
        ok &= oks[(size_t)p] > 0;
    }
    if (refused) {
        undo();
        return h->err = "peer transport: more same-device ranks in one process than half of "
                        "GPU_MAX_HW_QUEUES (init transport kept)",
               SW_ERR_INVALID;
    }
    if (!ok) {
        undo();
        return h->err = "peer transport: a rank could not map the exchange regions (init transport kept)",
               SW_ERR_HIP;
    }
    S->xslot = slot;
    S->xhalf = half;
    S->xseq = 0;
    S->xmax_jobs = max_total_jobs;
    S->peer = true;
    return SW_OK;
}

namespace {
int slow_solve(sw_shard_state* S, const sw_problem* local, int64_t total_jobs, sw_result* res, bool dirty);

/* An all-reduce of n step words in place, on the stream, without the host
 * (fast_solve): the identity at world 1, RCCL or the peer transport above. */
int coll_dev_reduce(sw_shard_state* S, void* dbuf, int n, int op) {
    if (S->world == 1) return SW_OK;
    if (S->peer) return peer_xchg(S, dbuf, (size_t)n * 8, op, n, dbuf);
    if (!S->comm) return S->h->err = "fast path: no device collective", SW_ERR_INVALID;
    const ncclDataType_t ty = op == 0 ? ncclInt64 : op == 1 ? ncclUint64 : ncclFloat64;
    SH_NCCL(S, ncclAllReduce(dbuf, dbuf, (size_t)n, ty, op == 0 ? ncclSum : ncclMax, S->comm, S->h->stream));
    return SW_OK;
}

/*
 * The solve's common path with the controller's decisions on the device
 * (DESIGN.md §7.2): setup, the level search, SELECT at M_lo (its price search,
 * take and assign), the SELECT / UMAX evaluations, the next level interval's
 * count, the share placement, the exchange step and the final evaluation are
 * all enqueued at once — every collective on the stream (RCCL or the peer
 * transport), every decision a one-wave kernel (k_fast_*) — and the host
 * reads one result.  The path is sw_shard_solve's whenever the level search
 * ends at M_lo (no other level can win), the tie group fills the budget (no
 * width tail) and every share places its counts: then the same kernels on
 * the same values give the same result bit for bit.  Otherwise the result
 * says escape and the host-driven controller solves the instance again
 * (returns 2); 1 = solved; 0 = not attempted; < 0 = error.  Host collectives
 * keep the host controller (every step needs the host there).
 */
int fast_solve(sw_shard_state* S, const sw_problem* pr, int64_t N, sw_result* res) {
    static const bool off = getenv("SW_SHARD_NOFAST") != nullptr; /* A/B: the host-driven controller */
    static const bool trace = getenv("SW_FAST_TRACE") != nullptr; /* diagnostics: sync after each stage */
#define FAST_TRACE(what)                                                                      \
    do {                                                                                      \
        if (trace) {                                                                          \
            hipError_t e_ = hipStreamSynchronize(S->h->stream);                              \
            fprintf(stderr, "fast_solve: %s: %s\n", what, hipGetErrorString(e_));           \
        }                                                                                     \
    } while (0)
    if (off || (S->host_comm && !S->peer) || !(N > 0 && pr->regularizer > 0.0)) return 0;
    hipStream_t st = S->h->stream;
    const int W = S->world, LW = (int)S->LW;
    const long long C = (long long)pr->num_gpus * pr->future_rounds;
    FastCtl* fc = S->fctl.p;
    unsigned long long* sbL = S->srch.p;           /* the level search's states */
    unsigned long long* sbP = S->srch.p + 2 * kSt; /* the price search's */
    unsigned long long* glL = S->glist.p;          /* their item lists */
    unsigned long long* glP = S->glist.p + kGl;
    disarm_pub(S);
    /* setup (op_setup): constants, key rows, the maxima */
    SH_TRY(zero_red(S, 4));
    long long* R0 = S->dv.red;
    LAUNCH(S, k_setup, dim3(nblk(S->NL)), dim3(kTB), 0, st, S->dv, S->jc.p, S->in_w, S->in_d, S->in_F, S->in_E,
           S->in_R, S->delta);
    SH_TRY(coll_dev_reduce(S, R0, 4, 1));
    LAUNCH(S, k_keys, dim3(nblk((int64_t)S->NL * 64)), dim3(kTB), 0, st, S->dv, fc, sbL, C, pr->regularizer);
    FAST_TRACE("setup");
    /* the level search M_lo: kFastRounds rounds (a probe, then typically the
     * gather of a small bracket; a search that needs more leaves the path) */
    unsigned long long *srl = nullptr, *spf = nullptr;
    SearchTail tl{}, tp{}; /* their last steps, taken by k_force and k_take */
    SH_TRY(enqueue_search(S, 1, kFastRounds, sbL, glL, &srl, false, &tl));
    FAST_TRACE("level search");
    /* SELECT(M_lo) (swc_select): force, the price search, take, assign */
    SH_TRY(zero_red(S, 2));
    long long* R1 = S->dv.red;
    if (W == 1) { /* the force's last block sets up the price search */
        LAUNCH(S, k_force, dim3(nblk(S->NL)), dim3(kTB), 0, st, S->dv, 0.0, 0, (const unsigned long long*)srl, tl,
               fc, sbP);
    } else {
        LAUNCH(S, k_force, dim3(nblk(S->NL)), dim3(kTB), 0, st, S->dv, 0.0, 0, (const unsigned long long*)srl, tl);
        SH_TRY(coll_dev_reduce(S, R1, 2, 0));
        LAUNCH(S, k_fast_price_init, dim3(1), dim3(64), 0, st, fc, (const long long*)R1,
               (const unsigned long long*)srl, sbP);
    }
    SH_TRY(enqueue_search(S, 0, kFastRounds, sbP, glP, &spf, false, &tp));
    FAST_TRACE("price search");
    SH_TRY(zero_red(S, 2));
    long long* R2 = S->dv.red;
    LAUNCH(S, k_take, dim3(nblk(S->NL)), dim3(kTB), 0, st, S->dv, 0u, (const unsigned long long*)spf,
           (const FastCtl*)fc, tp);
    const void* gv = R2;
    if (W > 1) SH_TRY(coll_gather(S, R2, S->xrecv.p, 16, nullptr, &gv));
    SH_TRY(zero_red(S, 1));
    long long* R3 = S->dv.red;
    LAUNCH(S, k_assign, dim3(nblk(S->NL)), dim3(kTB), 0, st, S->dv, 0ll, 0ll, fc, (const long long*)gv, W);
    SH_TRY(coll_dev_reduce(S, R3, 1, 0));
    /* world 1: the width tail on the device (above it the tail's collectives
     * are host steps: k_fast_sel_ctl sends the solve to the host path) */
    if (W == 1) LAUNCH(S, k_fast_tail, dim3(1), dim3(kTailTB), 0, st, S->dv, fc, (const long long*)R3);
    FAST_TRACE("take/assign");
    /* the SELECT evaluation and swc_level_search's utility optimum in one
     * pass, then the level values in (M_lo, M_lo + wmax] (none: M_lo wins) */
    const double* v = nullptr;
    SH_TRY(eval_enqueue(S, kEvSelUmax, 0, &v, nullptr));
    LAUNCH(S, k_fast_sel_ctl, dim3(1), dim3(64), 0, st, fc, (const long long*)R3, v,
           (const unsigned long long*)spf, W, LW);
    SH_TRY(zero_red(S, 1));
    long long* R4 = S->dv.red;
    LAUNCH(S, k_between, dim3(nblk(S->NL)), dim3(kTB), 0, st, S->dv, 0.0, 0.0, (const FastCtl*)fc);
    SH_TRY(coll_dev_reduce(S, R4, 1, 0));
    /* (k_between also copied the counts arr[SW_A_N] into arr[SW_A_NB]) */
    FAST_TRACE("between");
    /* the share placement (P1's and, in density order, P2's), then the
     * exchange step and the final evaluation on it (sw_shard_solve) */
    long long* Rd = nullptr; /* the stranded rounds, summed by the loop kernel (else PACKED below) */
    SH_TRY(pack_share_any(S, SW_A_NB, SW_Y_CUR, SW_A_PL, &Rd));
    if (Rd) {
        SH_TRY(coll_dev_reduce(S, Rd, 1, 0));
    } else {
        SH_TRY(eval_enqueue(S, SW_EV_PACKED, SW_A_PL, &v, nullptr));
        LAUNCH(S, k_fast_packed, dim3(1), dim3(64), 0, st, fc, v, W, LW);
    }
    FAST_TRACE("pack");
    /* the exchange step, the final evaluation and the result (twice when the
     * share placement stranded rounds: again after the host's share repair) */
    auto finish = [&](const long long* R4f, const long long* Rdf, int extra_iters, int extra_status,
                      FastOut& o) -> int {
        long long* R5 = nullptr;
        SH_TRY(p2x_enqueue(S, SW_Y_CUR, SW_A_PL, &R5, false, Rdf));
        FAST_TRACE("p2x");
        SH_TRY(eval_enqueue(S, SW_EV_FINAL, SW_Y_CUR, &v, nullptr));
        SH_TRY(publish_reserve(S, sizeof(FastOut) / 4 + 1));
        const unsigned long long seq = ++S->pub_seq;
        LAUNCH(S, k_fast_final, dim3(1), dim3(64), 0, st, (const FastCtl*)fc, R4f, (const long long*)R5, v,
               (const unsigned long long*)srl, (const unsigned long long*)spf, W, LW,
               reinterpret_cast<FastOut*>(S->pub_dev), S->pub_flag_dev, seq, (const int*)S->xerr, Rdf,
               extra_iters, extra_status);
        FAST_TRACE("final");
        /* one wait for the whole solve */
        auto t0 = std::chrono::steady_clock::now();
        uint32_t spins = 0;
        while (__atomic_load_n(S->pub_flag, __ATOMIC_ACQUIRE) < seq) {
            __builtin_ia32_pause();
            if (((++spins) & 0xFFFFu) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
                SH_HIP(S, hipStreamSynchronize(st));
                if (__atomic_load_n(S->pub_flag, __ATOMIC_ACQUIRE) < seq)
                    return S->h->err = "fast path: the result never arrived", SW_ERR_HIP;
                break;
            }
        }
        memcpy(&o, S->pub, sizeof(o));
        if (trace)
            fprintf(stderr, "fast_solve: escape %d objective %.17g iters %d status %d\n", o.escape, o.objective,
                    o.iters, o.status);
        if (o.xerr) {
            S->xfailed = true; /* sticky: the ranks stopped at different exchanges */
            return S->h->err = "peer exchange: a rank's flag never arrived (timed out)", SW_ERR_RCCL;
        }
        return SW_OK;
    };
    FastOut o;
    SH_TRY(finish((const long long*)R4, (const long long*)Rd, 0, 0, o));
    if (o.escape == 2) {
        /* only the share placement stranded rounds (sw_shard_solve): the
         * shares' repair (host: sw_profile_repair, then class repacks on the
         * device), its PACKED evaluation — one more collective step — and,
         * when it places every count, the rest of the path on this state (the
         * exchange left the placement as it was); P2 is the repaired density
         * placement (SW_STATUS_P2_REPAIRED) */
        SH_TRY(op_share_repair(S, SW_A_NB, SW_Y_CUR, SW_A_PL));
        double gmr;
        int64_t dfc = 0;
        std::vector<double> la((size_t)SW_DET_LANES), lb((size_t)SW_DET_LANES);
        SH_TRY(op_eval(S, SW_EV_PACKED, SW_A_PL, la.data(), lb.data(), &gmr, &dfc));
        if (dfc != 0) return 2; /* the gathered orders: the host-driven controller */
        SH_TRY(finish(nullptr, nullptr, 1, SW_STATUS_P2_REPAIRED, o));
    }
#undef FAST_TRACE
    if (o.escape) return 2;
    res->objective = o.objective;
    res->utility = o.utility;
    res->makespan = o.makespan;
    res->p2_objective = o.p2;
    res->bound = o.bound;
    res->iters = o.iters;
    res->status = o.status;
    return 1;
}

int dist_solve(sw_handle* h, const sw_problem* local, int64_t job_offset, int64_t total_jobs,
               sw_result* res, bool dev) {
    if (!h || !res || !local) return SW_ERR_INVALID;
    if (!h->shard) return h->err = "sw_dist_init / sw_dist_init_host first", SW_ERR_INVALID;
    sw_shard_state* S = h->shard;
    if (dev) { /* scalars here; the per-job checks run in k_setup */
        sw_problem sc = *local;
        sc.num_jobs = 0;
        if (sw_validate_problem(&sc) != 0 || local->num_jobs < 0 ||
            (local->num_jobs > 0 && (!local->nworkers || !local->epoch_duration ||
                                     !local->completed_epochs || !local->total_epochs ||
                                     !local->remaining_runtime || !local->priority)))
            return h->err = "invalid problem", SW_ERR_INVALID;
    } else if (sw_validate_problem(local) != 0) {
        return h->err = "invalid problem", SW_ERR_INVALID;
    }
    int64_t lo, hi;
    if (sw_shard_range(total_jobs, S->world, S->rank, &lo, &hi) != 0 || lo != job_offset ||
        hi - lo != local->num_jobs)
        return h->err = "slice does not match sw_dist_shard_range", SW_ERR_INVALID;
    if (hipSetDevice(h->device) != hipSuccess) return h->err = "hipSetDevice", SW_ERR_HIP;
    if (S->peer && total_jobs > S->xmax_jobs)
        return h->err = "total_jobs exceeds sw_dist_enable_peer's max_total_jobs", SW_ERR_CAPACITY;
    if (S->peer && S->xfailed)
        return h->err = "peer exchange timed out earlier: the ranks' sequence numbers diverged, "
                        "rebuild the handle", SW_ERR_RCCL;
    SH_TRY(prepare(S, local, job_offset, total_jobs, dev, res));
    int rc = fast_solve(S, local, total_jobs, res);
    if (rc < 0) return rc;
    if (rc == 1) {
        rc = SW_OK;
    } else {
        rc = slow_solve(S, local, total_jobs, res, rc == 2);
        if (rc < 0) return rc;
    }
    const size_t n = (size_t)S->NL;
    if (n && !dev) {
        if (res->plan)
            SH_HIP(S, hipMemcpyAsync(res->plan, S->plan.p, n * S->T, hipMemcpyDeviceToHost, h->stream));
        if (res->planned_rounds)
            SH_HIP(S, hipMemcpyAsync(res->planned_rounds, S->planned.p, n * 4, hipMemcpyDeviceToHost,
                                     h->stream));
    }
    SH_HIP(S, hipStreamSynchronize(h->stream));
    if (S->peer) { /* a timed-out exchange after the last publish */
        int e = 0;
        SH_HIP(S, hipMemcpy(&e, S->xerr, sizeof(int), hipMemcpyDeviceToHost));
        if (e) {
            S->xfailed = true; /* sticky: the handle is unusable from here on */
            return h->err = "peer exchange: a rank's flag never arrived (timed out)", SW_ERR_RCCL;
        }
    }
    return rc;
}

/* The host-driven controller (sw_shard_ctl.h) over this engine's ops: every
 * solve that leaves fast_solve's common path, and every solve on host
 * collectives.  A fast path that escaped left its state behind: cleared first. */
int slow_solve(sw_shard_state* S, const sw_problem* local, int64_t total_jobs, sw_result* res, bool dirty) {
    sw_handle* h = S->h;
    if (dirty) { /* the state and the ring, as prepare() leaves them (k_zero_state clears the
                  * ring from S.red: its base, not the last step's slice) */
        S->dv.red = S->red.p;
        LAUNCH(S, k_zero_state, dim3(nblk(std::max<int64_t>(S->NL, (int64_t)kRing * kRed))), dim3(kTB), 0,
               h->stream, S->dv);
        S->ring_pos = 0;
    }
    sw_shard_ops ops;
    ops.ctx = S;
    ops.setup = op_setup;
    ops.widths = op_widths;
    ops.force = op_force;
    ops.count_gt = op_count_gt;
    ops.feasible = op_feasible;
    ops.gather = op_gather;
    ops.between = op_between;
    ops.take_all = op_take_all;
    ops.take = op_take;
    ops.assign = op_assign;
    ops.tail_best = op_tail_best;
    ops.tail_apply = op_tail_apply;
    ops.fill_best = op_fill_best;
    ops.fill_apply = op_fill_apply;
    ops.eval = op_eval;
    ops.copy = op_copy;
    ops.copy_y = op_copy_y;
    ops.pack = op_pack;
    ops.class_caps = op_class_caps;
    ops.pack_class = op_pack_class;
    ops.p2x = op_p2x;
    ops.reround = op_reround;
    ops.search = (S->host_comm && !S->peer) ? nullptr : op_search; /* host collectives need the host per round */
    ops.pack_share = op_pack_share;
    ops.share_repair = op_share_repair;
    ops.raise_stats = op_raise_stats;
    ops.raise_best = op_raise_best;
    static const bool trace = getenv("SW_FAST_TRACE") != nullptr;
    if (trace) fprintf(stderr, "slow_solve: start (dirty %d)\n", (int)dirty);
    int rc = sw_shard_solve(&ops, total_jobs, local->future_rounds, local->num_gpus,
                            local->regularizer, &res->objective, &res->utility, &res->makespan,
                            &res->p2_objective, &res->bound, &res->iters, &res->status);
    if (trace) fprintf(stderr, "slow_solve: rc %d objective %.17g iters %d\n", rc, res->objective, res->iters);
    if (rc < 0) return rc == -1 ? (h->err = "out of host memory", SW_ERR_HIP) : rc;
    return rc;
}
}  // namespace

extern "C" {

int sw_dist_plan_solve(sw_handle* h, const sw_problem* local, int64_t job_offset, int64_t total_jobs,
                       sw_result* res) {
    if (h && res && res->plan_masks) return h->err = "plan_masks: batch entry points only", SW_ERR_INVALID;
    return dist_solve(h, local, job_offset, total_jobs, res, false);
}

int sw_dist_plan_solve_dev(sw_handle* h, const sw_problem* local, int64_t job_offset,
                           int64_t total_jobs, sw_result* res) {
    if (h && res && res->plan_masks) return h->err = "plan_masks: batch entry points only", SW_ERR_INVALID;
    return dist_solve(h, local, job_offset, total_jobs, res, true);
}

}  // extern "C"
