/*
 * sw_api.hip — host side of the C-ABI declared in include/shockwave_amd.h.
 *
 * Owns one HIP stream (or borrows the caller's) and the device SoA of one
 * batch.  Upload packs the caller's per-job arrays into pinned staging and
 * copies them to HBM in one transfer per array; run launches the plan kernel
 * (one workgroup per instance) on the stream; download copies plans and
 * per-instance results back.  No exception crosses the ABI.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/shockwave_amd.h"
#include "sw_arith.h"
#include "sw_device.h"
#include "sw_handle.h"
#include "sw_p2x.h"
#include "sw_validate.h"

/* on-chip batches up to this many instances (one per CU) fuse the exchange
 * step into the full kernel (SW_FUSE_MAX overrides) */
static int fuse_max_count() {
    static const int v = [] {
        const char* e = getenv("SW_FUSE_MAX");
        return e ? atoi(e) : 256;
    }();
    return v;
}

/* On-chip batches above this many instances take the split kernels
 * (SW_SPLIT_MIN overrides).  The split buys several instances per CU in the
 * light phases, but an instance its pack kernel leaves is solved again from
 * the start by the full kernel, and each of the four kernels waits for its
 * slowest instance: with few instances per CU (a single solve, the 512-
 * instance C5 sweep with its slow small-cluster instances) one full kernel
 * is faster. */
static int split_min_count() {
    static const int v = [] {
        const char* e = getenv("SW_SPLIT_MIN");
        return e ? atoi(e) : 256;
    }();
    return v;
}


extern "C" size_t sw_plan_kernel_lds_bytes(int one);
extern "C" hipError_t sw_launch_plan(const sw_batch_dev* B, int KT, int one, size_t lds,
                                     hipStream_t stream);
extern "C" hipError_t sw_launch_split(sw_batch_dev* B, size_t p2x_lds, hipStream_t stream);
extern "C" hipError_t sw_launch_p2x(const sw_batch_dev* B, int maxN, int maxT, hipStream_t stream);
extern "C" size_t sw_p2x_kernel_lds_bytes(int maxN, int maxT);

namespace {

thread_local std::string g_create_error;

}  // namespace

namespace {

int fail(sw_handle* h, int code, const std::string& msg) {
    if (h) h->err = msg;
    return code;
}

int hip_fail(sw_handle* h, hipError_t e, const char* what) {
    return fail(h, SW_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define SW_HIP(h, call)                                        \
    do {                                                       \
        hipError_t _e = (call);                                \
        if (_e != hipSuccess) return hip_fail((h), _e, #call); \
    } while (0)

int collect_timing(sw_handle* h) {
    for (size_t i = 0; i < h->ev_used; ++i) {
        SW_HIP(h, hipEventSynchronize(h->ev_pool[2 * i + 1]));
        float ms = 0.f;
        SW_HIP(h, hipEventElapsedTime(&ms, h->ev_pool[2 * i], h->ev_pool[2 * i + 1]));
        h->ms_plan += ms;
        SW_HIP(h, hipEventSynchronize(h->ev_p2x[2 * i + 1]));
        SW_HIP(h, hipEventElapsedTime(&ms, h->ev_p2x[2 * i], h->ev_p2x[2 * i + 1]));
        h->ms_p2x += ms;
        h->runs += 1;
    }
    h->ev_used = 0;
    return SW_OK;
}

constexpr size_t kEventPairs = 256;
constexpr int kMaxChunks = 16; /* host-boundary pipeline */

size_t a16(size_t b) { return (b + 15) & ~(size_t)15; }

/* The input block of count instances and J jobs: the descriptors, then w,
 * F, E (int32) and d, R, p (f64). */
size_t in_block_bytes(int32_t count, int64_t J) {
    return a16((size_t)count * sizeof(sw_inst_dev)) + 3 * a16((size_t)J * 4) + 3 * a16((size_t)J * 8);
}

/* The output block: count results, J counts, P plan bytes. */
size_t res_block_bytes(int32_t count, int64_t J, int64_t P) {
    return a16((size_t)count * sizeof(sw_out_dev)) + a16((size_t)J * 4) + a16((size_t)P);
}

/* Views of both blocks (device and pinned) for a batch of count instances,
 * J jobs and P plan bytes; the blocks are reserved for at least these. */
void set_views(sw_handle* h, int32_t count, int64_t J, int64_t P) {
    const size_t i4 = a16((size_t)J * 4), i8 = a16((size_t)J * 8);
    const size_t id = a16((size_t)count * sizeof(sw_inst_dev));
    h->d_inst = (sw_inst_dev*)h->d_in.p;
    h->h_inst = (sw_inst_dev*)h->h_in.p;
    unsigned char* d = h->d_in.p + id;
    unsigned char* x = h->h_in.p + id;
    h->d_w = (int32_t*)d;            h->h_w = (int32_t*)x;
    h->d_F = (int32_t*)(d + i4);     h->h_F = (int32_t*)(x + i4);
    h->d_E = (int32_t*)(d + 2 * i4); h->h_E = (int32_t*)(x + 2 * i4);
    h->d_d = (double*)(d + 3 * i4);  h->h_d = (double*)(x + 3 * i4);
    h->d_R = (double*)(d + 3 * i4 + i8);     h->h_R = (double*)(x + 3 * i4 + i8);
    h->d_p = (double*)(d + 3 * i4 + 2 * i8); h->h_p = (double*)(x + 3 * i4 + 2 * i8);
    h->in_bytes = in_block_bytes(count, J);
    const size_t o = a16((size_t)count * sizeof(sw_out_dev)), c = a16((size_t)J * 4);
    h->d_out = (sw_out_dev*)h->d_res.p;          h->h_out = (sw_out_dev*)h->h_res.p;
    h->d_planned = (int32_t*)(h->d_res.p + o);   h->h_planned = (int32_t*)(h->h_res.p + o);
    h->d_plan = h->d_res.p + o + c;              h->h_plan = h->h_res.p + o + c;
    h->res_bytes = res_block_bytes(count, J, P);
}


}  // namespace

extern "C" {

int sw_abi_version(void) { return SW_ABI_VERSION; }

const char* sw_create_error(void) { return g_create_error.c_str(); }

sw_handle* sw_create(const sw_config* cfg) {
    g_create_error.clear();
    sw_handle* h = new (std::nothrow) sw_handle();
    if (!h) {
        g_create_error = "out of host memory";
        return nullptr;
    }
    h->device = cfg ? cfg->device : 0;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) {
        g_create_error = std::string("no HIP device: ") + hipGetErrorString(e);
        delete h;
        return nullptr;
    }
    if (h->device < 0 || h->device >= ndev) {
        g_create_error = "device ordinal out of range";
        delete h;
        return nullptr;
    }
    e = hipSetDevice(h->device);
    if (e == hipSuccess) {
        if (cfg && cfg->stream) {
            h->stream = (hipStream_t)cfg->stream;
        } else {
            e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
            h->own_stream = (e == hipSuccess);
        }
    }
    h->ev_pool.assign(2 * kEventPairs, nullptr);
    h->ev_p2x.assign(2 * kEventPairs, nullptr);
    for (size_t i = 0; e == hipSuccess && i < h->ev_pool.size(); ++i) e = hipEventCreate(&h->ev_pool[i]);
    for (size_t i = 0; e == hipSuccess && i < h->ev_p2x.size(); ++i) e = hipEventCreate(&h->ev_p2x[i]);
    if (e != hipSuccess) {
        g_create_error = std::string("HIP init failed: ") + hipGetErrorString(e);
        sw_destroy(h);
        return nullptr;
    }
    /* optional up-front reservation */
    if (cfg && cfg->max_instances > 0 && cfg->max_total_jobs > 0) {
        size_t J = (size_t)cfg->max_total_jobs, I = (size_t)cfg->max_instances;
        if (h->d_in.reserve(in_block_bytes((int32_t)I, (int64_t)J)) ||
            h->d_res.reserve(res_block_bytes((int32_t)I, (int64_t)J, (int64_t)J * SW_MAX_ROUNDS)) ||
            h->d_masks.reserve(J) || h->d_nb.reserve(J) || h->d_lvl.reserve(I) ||
            h->d_p2ws.reserve(J * SW_P2X_ARR_BYTES) ||
            h->h_in.reserve(in_block_bytes((int32_t)I, (int64_t)J)) ||
            h->h_res.reserve(res_block_bytes((int32_t)I, (int64_t)J, (int64_t)J * SW_MAX_ROUNDS)) ||
            h->h_masks.reserve(J)) {
            g_create_error = "device reservation failed";
            sw_destroy(h);
            return nullptr;
        }
    }
    return h;
}

void sw_destroy(sw_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->up) (void)hipStreamSynchronize(h->up);
    if (h->dn) (void)hipStreamSynchronize(h->dn);
    sw_shard_release(h);
    sw_mmf_release(h);
    h->d_in.release(); h->d_res.release();
    h->d_ws_u8.release(); h->d_ws_u64.release(); h->d_ws_sort.release();
    h->d_ws_keys.release(); h->d_ws_jc.release(); h->d_stamps.release();
    h->d_masks.release(); h->d_p2ws.release(); h->d_nb.release(); h->d_lvl.release();
    h->h_in.release(); h->h_res.release();
    h->h_masks.release();
    for (hipEvent_t ev : h->ev_chunk)
        if (ev) (void)hipEventDestroy(ev);
    if (h->up) (void)hipStreamDestroy(h->up);
    if (h->dn) (void)hipStreamDestroy(h->dn);
    for (hipEvent_t ev : h->ev_xs)
        if (ev) (void)hipEventDestroy(ev);
    for (hipStream_t x : h->xs)
        if (x) (void)hipStreamDestroy(x);
    for (hipEvent_t ev : h->ev_pool)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : h->ev_p2x)
        if (ev) (void)hipEventDestroy(ev);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

const char* sw_last_error(const sw_handle* h) { return h ? h->err.c_str() : "null handle"; }

void* sw_stream(sw_handle* h) { return h ? (void*)h->stream : nullptr; }

}  // extern "C"

namespace {

/* Host threads for validation, staging and unpacking: one per ~64k jobs, at
 * most 16 (a GPU's CPU share on the MI355X box; SW_HOST_THREADS overrides). */
int host_threads(int64_t jobs) {
    static const int cap = [] {
        const char* e = getenv("SW_HOST_THREADS");
        const int v = e ? atoi(e) : 0;
        if (v > 0) return std::min(v, 256);
        const unsigned hw = std::thread::hardware_concurrency();
        return (int)std::max(1u, std::min(hw ? hw : 1u, 16u));
    }();
    return (int)std::max<int64_t>(1, std::min<int64_t>(cap, jobs / 65536));
}

int64_t jobs_of(const sw_handle* h, int32_t lo, int32_t hi) {
    return hi > lo ? h->inst[hi - 1].job_off + h->inst[hi - 1].N - h->inst[lo].job_off : 0;
}

/* f(a, b) over nt contiguous sub-ranges of instances [lo, hi) holding about
 * equal numbers of jobs; the calling thread takes the first.  A thread that
 * cannot be started runs its range inline (no exception crosses the ABI). */
template <class F>
void par_instances(const sw_handle* h, int32_t lo, int32_t hi, F&& f) {
    const int nt = std::min<int64_t>(host_threads(jobs_of(h, lo, hi)), hi - lo);
    if (nt <= 1) {
        if (hi > lo) f(lo, hi);
        return;
    }
    const int64_t J0 = h->inst[lo].job_off, J = jobs_of(h, lo, hi);
    std::vector<int32_t> cut(nt + 1);
    cut[0] = lo;
    cut[nt] = hi;
    for (int t = 1; t < nt; ++t) {
        const int64_t target = J0 + J * t / nt;
        auto it = std::lower_bound(h->inst.begin() + lo, h->inst.begin() + hi, target,
                                   [](const sw_inst_dev& d, int64_t v) { return d.job_off < v; });
        cut[t] = std::max(cut[t - 1], (int32_t)(it - h->inst.begin()));
    }
    std::vector<std::thread> th;
    th.reserve(nt - 1);
    for (int t = 1; t < nt; ++t) {
        if (cut[t] >= cut[t + 1]) continue;
        try {
            th.emplace_back([&f, &cut, t] { f(cut[t], cut[t + 1]); });
        } catch (...) {
            f(cut[t], cut[t + 1]);
        }
    }
    if (cut[0] < cut[1]) f(cut[0], cut[1]);
    for (auto& x : th) x.join();
}

/* Sizes and offsets of a batch from the problems' headers, capacity for it,
 * and no batch described until its upload completes. */
int prepare_batch(sw_handle* h, int32_t count, const sw_problem* probs) {
    if (count < 0 || (count > 0 && !probs)) return fail(h, SW_ERR_INVALID, "bad batch");
    SW_HIP(h, hipSetDevice(h->device));
    int64_t J = 0, P = 0;
    int32_t maxN = 0, maxT = 1;
    for (int32_t i = 0; i < count; ++i) {
        const sw_problem& pr = probs[i];
        if (pr.num_jobs < 0 || pr.future_rounds < 1 || pr.future_rounds > SW_MAX_ROUNDS)
            return fail(h, SW_ERR_INVALID, "invalid problem at index " + std::to_string(i));
        J += pr.num_jobs;
        P += (int64_t)pr.num_jobs * pr.future_rounds;
        maxN = std::max(maxN, pr.num_jobs);
        maxT = std::max(maxT, pr.future_rounds);
    }
    /* wait for any run still using the buffers */
    SW_HIP(h, hipStreamSynchronize(h->stream));
    if (h->up) SW_HIP(h, hipStreamSynchronize(h->up));
    if (h->dn) SW_HIP(h, hipStreamSynchronize(h->dn));
    if (collect_timing(h) != SW_OK) return SW_ERR_HIP;
    /* the previous batch is gone from here on: a reserve below frees the
     * old buffers before it allocates, so a failure must leave no batch
     * described that run / download could touch */
    h->loaded = false;
    h->count = 0;
    h->total_jobs = 0;
    h->total_plan = 0;
    const size_t Jz = (size_t)std::max<int64_t>(J, 1);
    const size_t inb = in_block_bytes(std::max(count, 1), (int64_t)Jz), resb = res_block_bytes(std::max(count, 1), (int64_t)Jz, std::max<int64_t>(P, 1));
    if (h->d_in.reserve(inb) || h->d_res.reserve(resb) ||
        h->d_masks.reserve(Jz) || h->d_nb.reserve(Jz) || h->d_lvl.reserve(std::max(count, 1)))
        return fail(h, SW_ERR_HIP, "device allocation failed");
    if (maxN > SW_LDS_JOBS || maxT > 32) {
        const int KT = maxT <= 32 ? 32 : 64;
        if (h->d_ws_u8.reserve(Jz * SW_WS_U8) || h->d_ws_u64.reserve(Jz * SW_WS_U64 + (size_t)SW_WS_PAD_U64 * std::max(count, 1)) ||
            h->d_ws_sort.reserve(Jz * 4) || h->d_ws_keys.reserve(Jz * KT) ||
            h->d_ws_jc.reserve(Jz))
            return fail(h, SW_ERR_HIP, "workspace allocation failed");
    }
    if (h->d_p2ws.reserve(Jz * SW_P2X_ARR_BYTES))
        return fail(h, SW_ERR_HIP, "P2 exchange workspace allocation failed");
    if (h->h_in.reserve(inb) || h->h_res.reserve(resb) || h->h_masks.reserve(Jz))
        return fail(h, SW_ERR_HIP, "pinned allocation failed");
    set_views(h, std::max(count, 1), (int64_t)Jz, std::max<int64_t>(P, 1));
    h->inst.resize(count);
    h->Ns.resize(count);
    h->Ts.resize(count);
    int64_t jo = 0, po = 0;
    for (int32_t i = 0; i < count; ++i) {
        sw_inst_dev& d = h->inst[i];
        d.N = probs[i].num_jobs;
        d.T = probs[i].future_rounds;
        d.job_off = jo;
        d.plan_off = po;
        h->Ns[i] = d.N;
        h->Ts[i] = d.T;
        jo += d.N;
        po += (int64_t)d.N * d.T;
    }
    h->maxN = maxN;
    h->maxT = maxT;
    h->pend_count = count;
    h->pend_jobs = J;
    h->pend_plan = P;
    return SW_OK;
}

/* Every problem of [0, count) validated (sw_validate.h) before the handle's
 * current batch is touched, in parallel over equal instance ranges; the
 * error names the first invalid index. */
int validate_all(sw_handle* h, const sw_problem* probs, int32_t count) {
    if (count < 0 || (count > 0 && !probs)) return fail(h, SW_ERR_INVALID, "bad batch");
    std::atomic<int32_t> bad{INT32_MAX};
    auto check = [&](int32_t a, int32_t b) {
        for (int32_t i = a; i < b; ++i)
            if (sw_validate_problem(&probs[i]) != 0) {
                int32_t cur = bad.load();
                while (i < cur && !bad.compare_exchange_weak(cur, i)) {
                }
                return;
            }
    };
    /* the thread count from the first problem's size (headers unchecked yet) */
    const int64_t n0 = count > 0 && probs[0].num_jobs > 0 ? probs[0].num_jobs : 1;
    const int nt = (int)std::min<int64_t>(host_threads(n0 * count), count);
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) {
        const int32_t a = (int32_t)((int64_t)count * t / nt), b = (int32_t)((int64_t)count * (t + 1) / nt);
        try {
            th.emplace_back([&check, a, b] { check(a, b); });
        } catch (...) {
            check(a, b);
        }
    }
    check(0, nt > 1 ? (int32_t)((int64_t)count / nt) : count);
    for (auto& x : th) x.join();
    if (bad.load() != INT32_MAX)
        return fail(h, SW_ERR_INVALID, "invalid problem at index " + std::to_string(bad.load()));
    return SW_OK;
}

/* Instances [lo, hi) into the pinned staging (validated problems). */
void stage(sw_handle* h, const sw_problem* probs, int32_t lo, int32_t hi) {
    par_instances(h, lo, hi, [&](int32_t a, int32_t b) {
        for (int32_t i = a; i < b; ++i) {
            const sw_problem& pr = probs[i];
            sw_inst_dev& d = h->inst[i];
            const int64_t jo = d.job_off, po = d.plan_off;
            memset(&d, 0, sizeof(d));
            d.N = pr.num_jobs;
            d.T = pr.future_rounds;
            d.G = pr.num_gpus;
            d.nb = pr.num_bases;
            d.job_off = jo;
            d.plan_off = po;
            d.delta = pr.round_duration;
            d.k = pr.regularizer;
            for (int b = 0; b < SW_BMAX; ++b) {
                d.beta[b] = b < pr.num_bases ? pr.bases[b] : 0.0;
                d.ell[b] = b < pr.num_bases ? pr.log_bases[b] : 0.0;
            }
            h->h_inst[i] = d;
            const size_t n = (size_t)pr.num_jobs;
            if (n) {
                memcpy(h->h_w + jo, pr.nworkers, n * sizeof(int32_t));
                memcpy(h->h_F + jo, pr.completed_epochs, n * sizeof(int32_t));
                memcpy(h->h_E + jo, pr.total_epochs, n * sizeof(int32_t));
                memcpy(h->h_d + jo, pr.epoch_duration, n * sizeof(double));
                memcpy(h->h_R + jo, pr.remaining_runtime, n * sizeof(double));
                memcpy(h->h_p + jo, pr.priority, n * sizeof(double));
            }
        }
    });
}

/* H2D of instances [lo, hi) (their descriptors and job arrays) on s. */
int h2d(sw_handle* h, int32_t lo, int32_t hi, hipStream_t s) {
    if (hi <= lo) return SW_OK;
    const int64_t j0 = h->inst[lo].job_off, nj = jobs_of(h, lo, hi);
    if (lo == 0 && hi == h->pend_count) { /* the whole batch: one copy of the block */
        SW_HIP(h, hipMemcpyAsync(h->d_in.p, h->h_in.p, h->in_bytes, hipMemcpyHostToDevice, s));
        return SW_OK;
    }
    SW_HIP(h, hipMemcpyAsync(h->d_inst + lo, h->h_inst + lo, (size_t)(hi - lo) * sizeof(sw_inst_dev),
                             hipMemcpyHostToDevice, s));
    if (nj > 0) {
        SW_HIP(h, hipMemcpyAsync(h->d_w + j0, h->h_w + j0, nj * 4, hipMemcpyHostToDevice, s));
        SW_HIP(h, hipMemcpyAsync(h->d_F + j0, h->h_F + j0, nj * 4, hipMemcpyHostToDevice, s));
        SW_HIP(h, hipMemcpyAsync(h->d_E + j0, h->h_E + j0, nj * 4, hipMemcpyHostToDevice, s));
        SW_HIP(h, hipMemcpyAsync(h->d_d + j0, h->h_d + j0, nj * 8, hipMemcpyHostToDevice, s));
        SW_HIP(h, hipMemcpyAsync(h->d_R + j0, h->h_R + j0, nj * 8, hipMemcpyHostToDevice, s));
        SW_HIP(h, hipMemcpyAsync(h->d_p + j0, h->h_p + j0, nj * 8, hipMemcpyHostToDevice, s));
    }
    return SW_OK;
}

/* The solve kernels for instances [lo, hi) of the loaded batch on s: the
 * per-instance arrays offset to lo, the per-job ones global (each
 * descriptor holds its global job and plan offsets). */
int launch(sw_handle* h, int32_t lo, int32_t hi, hipStream_t s, bool timed, bool want_masks,
           int force_split = -1) {
    sw_batch_dev B;
    memset(&B, 0, sizeof(B));
    B.want_masks = want_masks ? 1 : 0;
    B.inst = h->d_inst + lo;
    B.count = hi - lo;
    B.KT = h->maxT <= 32 ? 32 : 64;
    B.w = h->d_w;
    B.d = h->d_d;
    B.F = h->d_F;
    B.E = h->d_E;
    B.R = h->d_R;
    B.p = h->d_p;
    B.plan = h->d_plan;
    B.planned = h->d_planned;
    B.masks = h->d_masks.p;
    B.out = h->d_out + lo;
    B.nb = h->d_nb.p;
    B.lvl = h->d_lvl.p + lo;
#ifdef SW_STAMPS
    B.stamps = h->d_stamps.p + (size_t)lo * SW_STAMP_SLOTS;
#endif
    const int one = h->maxN <= SW_LDS_JOBS && h->maxT <= 32;
    if (!one) {
        B.ws.u8 = h->d_ws_u8.p;
        B.ws.u64 = h->d_ws_u64.p;
        B.ws.sort = h->d_ws_sort.p;
        B.ws.keys = h->d_ws_keys.p;
        B.ws.jc = h->d_ws_jc.p;
    }
    B.p2ws = h->d_p2ws.p;
    size_t lds = sw_plan_kernel_lds_bytes(one);
    if (timed) {
        if (h->ev_used == kEventPairs && collect_timing(h) != SW_OK) return SW_ERR_HIP;
        SW_HIP(h, hipEventRecord(h->ev_pool[2 * h->ev_used], s));
    }
    /* Dispatch.  On-chip batches (every N ≤ SW_LDS_JOBS, T ≤ 32) above
     * split_min_count() instances: the level-search kernel, then the pack
     * kernel — each instance's P2 exchange step runs at its end, in the same
     * workgroup — then the full kernel for the instances the pack kernel
     * marked, with their exchange steps fused at its end too
     * (sw_launch_split).  Smaller on-chip batches of at most fuse_max_count()
     * instances: the full kernel with the exchange fused at its end.  The
     * rest (larger on-chip batches below the split size, and every batch with
     * an instance above SW_LDS_JOBS jobs or 32 rounds): the full kernel, then
     * the exchange kernel (sw_p2x_kernel.hip).  Timing: with the exchange
     * fused, the plan events bracket both stages and the exchange events an
     * empty interval, so sw_kernel_times reports the exchange inside the plan
     * time (include/shockwave_amd.h sw_set_timing). */
#ifdef SW_STAMPS
    const bool split = false; /* diagnostic builds time the phases inside the full kernel */
#else
    const bool split = one && (force_split >= 0 ? force_split != 0 : B.count > split_min_count());
#endif
    B.fuse_p2x = one && (split || B.count <= fuse_max_count()); /* split: always fused */
    if (B.fuse_p2x) lds = std::max(lds, sw_p2x_kernel_lds_bytes(h->maxN, h->maxT));
    hipError_t e = split ? sw_launch_split(&B, sw_p2x_kernel_lds_bytes(h->maxN, h->maxT), s)
                         : sw_launch_plan(&B, B.KT, one, lds, s);
    if (e != hipSuccess) return hip_fail(h, e, "plan kernel launch");
    if (timed) {
        SW_HIP(h, hipEventRecord(h->ev_pool[2 * h->ev_used + 1], s));
        SW_HIP(h, hipEventRecord(h->ev_p2x[2 * h->ev_used], s));
    }
    /* the P2 exchange step (sw_p2x_kernel.hip) on the plan kernels' masks */
    if (!B.fuse_p2x) {
        e = sw_launch_p2x(&B, h->maxN, h->maxT, s);
        if (e != hipSuccess) return hip_fail(h, e, "sw_p2x_kernel launch");
    }
    if (timed) {
        SW_HIP(h, hipEventRecord(h->ev_p2x[2 * h->ev_used + 1], s));
        h->ev_used++;
    }
    return SW_OK;
}

/* Which outputs the caller asked for (any result of the batch). */
struct Wants {
    bool plan = false, masks = false, planned = false;
};

Wants wants_of(const sw_result* res, int32_t count) {
    Wants w;
    for (int32_t i = 0; i < count; ++i) {
        w.plan |= res[i].plan != nullptr;
        w.masks |= res[i].plan_masks != nullptr;
        w.planned |= res[i].planned_rounds != nullptr;
    }
    return w;
}

/* D2H of instances [lo, hi)'s outputs on s. */
int d2h(sw_handle* h, int32_t lo, int32_t hi, hipStream_t s, const Wants& w) {
    if (hi <= lo) return SW_OK;
    const int64_t j0 = h->inst[lo].job_off, nj = jobs_of(h, lo, hi);
    const int64_t p0 = h->inst[lo].plan_off,
                  np = h->inst[hi - 1].plan_off + (int64_t)h->inst[hi - 1].N * h->inst[hi - 1].T - p0;
    if (w.masks && nj > 0)
        SW_HIP(h, hipMemcpyAsync(h->h_masks.p + j0, h->d_masks.p + j0, nj * 8, hipMemcpyDeviceToHost, s));
    if (lo == 0 && hi == h->pend_count && w.plan && w.planned) { /* results, counts, plans: one copy */
        SW_HIP(h, hipMemcpyAsync(h->h_res.p, h->d_res.p, h->res_bytes, hipMemcpyDeviceToHost, s));
        return SW_OK;
    }
    if (w.plan && np > 0)
        SW_HIP(h, hipMemcpyAsync(h->h_plan + p0, h->d_plan + p0, np, hipMemcpyDeviceToHost, s));
    if (w.planned && nj > 0)
        SW_HIP(h, hipMemcpyAsync(h->h_planned + j0, h->d_planned + j0, nj * 4, hipMemcpyDeviceToHost, s));
    SW_HIP(h, hipMemcpyAsync(h->h_out + lo, h->d_out + lo, (size_t)(hi - lo) * sizeof(sw_out_dev),
                             hipMemcpyDeviceToHost, s));
    return SW_OK;
}

/* Staged outputs of instances [lo, hi) into the caller's results, in
 * parallel; SW_FALLBACK when any kept P1's placement. */
int unpack(sw_handle* h, sw_result* res, int32_t lo, int32_t hi) {
    std::atomic<int> fb{0};
    par_instances(h, lo, hi, [&](int32_t a, int32_t b) {
        int f = 0;
        for (int32_t i = a; i < b; ++i) {
            const sw_inst_dev& d = h->inst[i];
            const sw_out_dev& o = h->h_out[i];
            sw_result& r = res[i];
            if (r.plan && d.N > 0) memcpy(r.plan, h->h_plan + d.plan_off, (size_t)d.N * d.T);
            if (r.plan_masks && d.N > 0) memcpy(r.plan_masks, h->h_masks.p + d.job_off, (size_t)d.N * 8);
            if (r.planned_rounds && d.N > 0)
                memcpy(r.planned_rounds, h->h_planned + d.job_off, (size_t)d.N * 4);
            r.objective = o.objective;
            r.utility = o.utility;
            r.makespan = o.makespan;
            r.p2_objective = o.p2_objective;
            r.bound = o.bound;
            r.iters = o.iters;
            r.status = o.status;
            f |= (o.status & SW_STATUS_P2_FALLBACK) != 0;
        }
        if (f) fb.store(1);
    });
    return fb.load() ? SW_FALLBACK : SW_OK;
}

void mark_loaded(sw_handle* h) {
    h->count = h->pend_count;
    h->total_jobs = h->pend_jobs;
    h->total_plan = h->pend_plan;
    h->loaded = true;
}

/* Chunks of a host-boundary solve (SW_PIPELINE_CHUNKS overrides; 1 = none). */
int pipeline_chunks(int32_t count) {
    static const int req = [] {
        const char* e = getenv("SW_PIPELINE_CHUNKS");
        const int v = e ? atoi(e) : 0;
        return v > 0 ? std::min(v, kMaxChunks) : 4;
    }();
    /* chunks of at least 2048 instances: each launch keeps every CU busy */
    return std::max(1, std::min<int>(req, count / 2048));
}

/*
 * sw_plan_solve_batch over host buffers as a pipeline of chunks of
 * instances: the host stages chunk c+1 while chunk c crosses PCIe, and
 * unpacks chunk c while later chunks are on the GPU; each chunk's H2D
 * (stream up), kernels (the handle's stream) and D2H (stream dn) are ordered
 * by events, so one chunk's copies overlap the neighbouring chunks' kernels.  Every problem is validated before any is
 * solved (the unchunked call's contract).
 */
int solve_pipelined(sw_handle* h, int32_t count, const sw_problem* probs, sw_result* res, int nch) {
    if (!h->up) SW_HIP(h, hipStreamCreateWithFlags(&h->up, hipStreamNonBlocking));
    if (!h->dn) SW_HIP(h, hipStreamCreateWithFlags(&h->dn, hipStreamNonBlocking));
    if (h->ev_chunk.empty()) {
        h->ev_chunk.assign(3 * kMaxChunks, nullptr);
        for (auto& ev : h->ev_chunk) SW_HIP(h, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    const Wants w = wants_of(res, count);
    std::vector<int32_t> cut(nch + 1);
    for (int c = 0; c <= nch; ++c) cut[c] = (int32_t)((int64_t)count * c / nch);
    int rc = SW_OK, err = SW_OK;
    for (int c = 0; c < nch && err == SW_OK; ++c) {
        hipEvent_t e_up = h->ev_chunk[3 * c], e_k = h->ev_chunk[3 * c + 1], e_dn = h->ev_chunk[3 * c + 2];
        stage(h, probs, cut[c], cut[c + 1]);
        if ((err = h2d(h, cut[c], cut[c + 1], h->up)) != SW_OK) break;
        SW_HIP(h, hipEventRecord(e_up, h->up));
        SW_HIP(h, hipStreamWaitEvent(h->stream, e_up, 0));
        if ((err = launch(h, cut[c], cut[c + 1], h->stream, false, w.masks)) != SW_OK) break;
        SW_HIP(h, hipEventRecord(e_k, h->stream));
        SW_HIP(h, hipStreamWaitEvent(h->dn, e_k, 0));
        if ((err = d2h(h, cut[c], cut[c + 1], h->dn, w)) != SW_OK) break;
        SW_HIP(h, hipEventRecord(e_dn, h->dn));
    }
    if (err != SW_OK) { /* nothing may still use the buffers */
        (void)hipStreamSynchronize(h->up);
        (void)hipStreamSynchronize(h->stream);
        (void)hipStreamSynchronize(h->dn);
        return err;
    }
    /* every chunk is staged and queued before the first unpack, so the
     * copy engine streams the H2D of all chunks back to back and no chunk's
     * kernels wait for the host */
    for (int c = 0; c < nch; ++c) {
        SW_HIP(h, hipEventSynchronize(h->ev_chunk[3 * c + 2]));
        rc |= unpack(h, res, cut[c], cut[c + 1]);
    }
    mark_loaded(h);
    return rc ? SW_FALLBACK : SW_OK;
}

/* Streams for sw_batch_run (SW_RUN_STREAMS overrides).  A split batch is
 * three launches, each waiting for its slowest instance, so a split batch
 * that does not fill the chip many times over (the 512-instance C5 sweep:
 * two instances per CU) ends with the slowest level search followed by the
 * slowest pack + exchange — of different instances.  Cut into contiguous
 * chunks on their own streams, a chunk's pack kernel starts when that
 * chunk's level searches are done, and the batch ends with the slowest
 * chunk's own chain.  Results are per instance, so the cut changes none. */
constexpr int kMaxRunStreams = 4; /* GPU_MAX_HW_QUEUES is 4 on the box */

int run_streams(const sw_handle* h) {
    static const int req = [] {
        const char* e = getenv("SW_RUN_STREAMS");
        return e ? atoi(e) : -1;
    }();
#ifdef SW_STAMPS
    return 1; /* diagnostic builds time the phases inside the full kernel */
#endif
    const bool one = h->maxN <= SW_LDS_JOBS && h->maxT <= 32;
    if (!one || h->count <= split_min_count()) return 1; /* not a split batch */
    int ns = req >= 0 ? req : (h->count <= 2048 ? 2 : 1);
    ns = std::max(1, std::min(ns, kMaxRunStreams));
    return std::min(ns, std::max(1, h->count / 64)); /* chunks of at least 64 */
}

int launch_streams(sw_handle* h, int ns) {
    if (h->xs.empty()) {
        h->xs.assign(kMaxRunStreams - 1, nullptr);
        h->ev_xs.assign(kMaxRunStreams, nullptr);
        for (auto& x : h->xs) SW_HIP(h, hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        for (auto& ev : h->ev_xs) SW_HIP(h, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    const bool timed = h->timing;
    if (timed) {
        if (h->ev_used == kEventPairs && collect_timing(h) != SW_OK) return SW_ERR_HIP;
        SW_HIP(h, hipEventRecord(h->ev_pool[2 * h->ev_used], h->stream));
    }
    SW_HIP(h, hipEventRecord(h->ev_xs[0], h->stream)); /* fork: the upload is done */
    for (int c = 1; c < ns; ++c) SW_HIP(h, hipStreamWaitEvent(h->xs[c - 1], h->ev_xs[0], 0));
    int err = SW_OK;
    for (int c = 0; c < ns && err == SW_OK; ++c) {
        const int32_t lo = (int32_t)((int64_t)h->count * c / ns), hi = (int32_t)((int64_t)h->count * (c + 1) / ns);
        err = launch(h, lo, hi, c == 0 ? h->stream : h->xs[c - 1], false, h->keep_masks, 1);
    }
    for (int c = 1; c < ns; ++c) { /* join (also after a failed launch: nothing may still run) */
        SW_HIP(h, hipEventRecord(h->ev_xs[c], h->xs[c - 1]));
        SW_HIP(h, hipStreamWaitEvent(h->stream, h->ev_xs[c], 0));
    }
    if (err != SW_OK) return err;
    if (timed) { /* the exchange runs inside the plan launches: an empty p2x interval */
        SW_HIP(h, hipEventRecord(h->ev_pool[2 * h->ev_used + 1], h->stream));
        SW_HIP(h, hipEventRecord(h->ev_p2x[2 * h->ev_used], h->stream));
        SW_HIP(h, hipEventRecord(h->ev_p2x[2 * h->ev_used + 1], h->stream));
        h->ev_used++;
    }
    return SW_OK;
}

}  // namespace

extern "C" {

int sw_batch_upload(sw_handle* h, int32_t count, const sw_problem* probs) {
    if (!h) return SW_ERR_INVALID;
    int rc = validate_all(h, probs, count);
    if (rc != SW_OK) return rc;
    if ((rc = prepare_batch(h, count, probs)) != SW_OK) return rc;
    stage(h, probs, 0, count);
    if ((rc = h2d(h, 0, count, h->stream)) != SW_OK) return rc;
    SW_HIP(h, hipStreamSynchronize(h->stream));
    mark_loaded(h);
#ifdef SW_STAMPS
    if (h->d_stamps.reserve((size_t)std::max(count, 1) * SW_STAMP_SLOTS))
        return fail(h, SW_ERR_HIP, "stamp buffer allocation failed");
    SW_HIP(h, hipMemset(h->d_stamps.p, 0, (size_t)std::max(count, 1) * SW_STAMP_SLOTS * sizeof(uint64_t)));
#endif
    return SW_OK;
}

#ifdef SW_STAMPS
/* Diagnostic builds only (not part of include/shockwave_amd.h). */
int sw_debug_stamps(sw_handle* h, uint64_t* out) {
    SW_HIP(h, hipStreamSynchronize(h->stream));
    SW_HIP(h, hipMemcpy(out, h->d_stamps.p, (size_t)h->count * SW_STAMP_SLOTS * sizeof(uint64_t),
                        hipMemcpyDeviceToHost));
    return SW_OK;
}
#endif

int sw_batch_run(sw_handle* h) {
    if (!h) return SW_ERR_INVALID;
    if (!h->loaded) return fail(h, SW_ERR_INVALID, "no batch uploaded");
    if (h->count <= 0) return SW_OK;
    SW_HIP(h, hipSetDevice(h->device));
    h->masks_valid = h->keep_masks;
    const int ns = run_streams(h);
    if (ns <= 1) return launch(h, 0, h->count, h->stream, h->timing, h->keep_masks);
    return launch_streams(h, ns);
}

int sw_batch_keep_masks(sw_handle* h, int32_t keep) {
    if (!h) return SW_ERR_INVALID;
    h->keep_masks = keep != 0;
    return SW_OK;
}

int sw_batch_download(sw_handle* h, sw_result* res) {
    if (!h) return SW_ERR_INVALID;
    if (!h->loaded) return fail(h, SW_ERR_INVALID, "no batch uploaded");
    if (h->count > 0 && !res) return fail(h, SW_ERR_INVALID, "null result array");
    SW_HIP(h, hipSetDevice(h->device));
    const Wants w = wants_of(res, h->count);
    if (w.masks && !h->masks_valid)
        return fail(h, SW_ERR_INVALID, "plan_masks: the last sw_batch_run did not keep them (sw_batch_keep_masks)");
    int rc = d2h(h, 0, h->count, h->stream, w);
    if (rc != SW_OK) return rc;
    SW_HIP(h, hipStreamSynchronize(h->stream));
    if (collect_timing(h) != SW_OK) return SW_ERR_HIP;
    return unpack(h, res, 0, h->count);
}

int sw_plan_solve_batch(sw_handle* h, int32_t count, const sw_problem* probs, sw_result* res) {
    if (!h) return SW_ERR_INVALID;
    if (count > 0 && !res) return fail(h, SW_ERR_INVALID, "null result array");
#ifndef SW_STAMPS
    /* the chunk pipeline for large on-chip batches on the handle's own
     * stream (a borrowed stream keeps every step on it) */
    const int nch = h->own_stream && !h->timing ? pipeline_chunks(count) : 1;
    if (nch > 1) {
        int32_t maxN = 0, maxT = 0;
        for (int32_t i = 0; i < count && probs; ++i) {
            maxN = std::max(maxN, probs[i].num_jobs);
            maxT = std::max(maxT, probs[i].future_rounds);
        }
        if (maxN <= SW_LDS_JOBS && maxT <= 32) {
            int rc = validate_all(h, probs, count);
            if (rc != SW_OK) return rc;
            if ((rc = prepare_batch(h, count, probs)) != SW_OK) return rc;
            return solve_pipelined(h, count, probs, res, nch);
        }
    }
#endif
    int rc = sw_batch_upload(h, count, probs);
    if (rc < 0) return rc;
    if (count > 0) { /* sw_batch_run, keeping the masks only if asked for */
        const bool km = wants_of(res, count).masks;
        SW_HIP(h, hipSetDevice(h->device));
        h->masks_valid = km;
        if ((rc = launch(h, 0, h->count, h->stream, h->timing, km)) < 0) return rc;
    }
    return sw_batch_download(h, res);
}

int sw_plan_solve(sw_handle* h, const sw_problem* prob, sw_result* res) {
    return sw_plan_solve_batch(h, 1, prob, res);
}

int sw_set_timing(sw_handle* h, int32_t enable) {
    if (!h) return SW_ERR_INVALID;
    if (collect_timing(h) != SW_OK) return SW_ERR_HIP;
    h->timing = enable != 0;
    h->ms_plan = 0.0;
    h->ms_p2x = 0.0;
    h->runs = 0;
    return SW_OK;
}

int sw_kernel_times(sw_handle* h, double* ms_p2x, double* ms_plan, int32_t* runs) {
    if (!h) return SW_ERR_INVALID;
    SW_HIP(h, hipSetDevice(h->device));
    if (collect_timing(h) != SW_OK) return SW_ERR_HIP;
    if (ms_p2x) *ms_p2x = h->ms_p2x;
    if (ms_plan) *ms_plan = h->ms_plan;
    if (runs) *runs = h->runs;
    return SW_OK;
}

}  // extern "C"
