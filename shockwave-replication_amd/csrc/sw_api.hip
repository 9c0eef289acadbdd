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

#include <algorithm>
#include <new>
#include <string>
#include <vector>

#include "../../include/shockwave_amd.h"
#include "sw_arith.h"
#include "sw_device.h"
#include "sw_handle.h"
#include "sw_validate.h"

/* batches above this many instances take the split kernels (MI355X: 256 CUs) */
constexpr int kSplitMinCount = 256;

#define SW_P2X_ARR_BYTES 24 /* sw_p2x_dev.h: exchange workspace bytes per job */

extern "C" size_t sw_plan_kernel_lds_bytes(int one);
extern "C" hipError_t sw_launch_plan(const sw_batch_dev* B, int KT, int one, size_t lds,
                                     hipStream_t stream);
extern "C" hipError_t sw_launch_split(sw_batch_dev* B, hipStream_t stream);
extern "C" hipError_t sw_launch_p2x(const sw_batch_dev* B, int maxN, int maxT, unsigned char* ws,
                                    hipStream_t stream);

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
        if (h->d_inst.reserve(I) || h->d_out.reserve(I) || h->d_w.reserve(J) ||
            h->d_F.reserve(J) || h->d_E.reserve(J) || h->d_planned.reserve(J) || h->d_masks.reserve(J) ||
            h->d_d.reserve(J) || h->d_R.reserve(J) || h->d_p.reserve(J) ||
            h->d_plan.reserve(J * SW_MAX_ROUNDS)) {
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
    sw_shard_release(h);
    sw_mmf_release(h);
    h->d_inst.release(); h->d_w.release(); h->d_F.release(); h->d_E.release();
    h->d_planned.release(); h->d_d.release(); h->d_R.release(); h->d_p.release();
    h->d_plan.release(); h->d_ws_u8.release(); h->d_ws_u64.release(); h->d_ws_sort.release();
    h->d_ws_keys.release(); h->d_ws_jc.release(); h->d_out.release(); h->d_stamps.release();
    h->d_masks.release(); h->d_p2ws.release(); h->d_nb.release(); h->d_lvl.release();
    h->h_w.release(); h->h_F.release(); h->h_E.release(); h->h_planned.release();
    h->h_d.release(); h->h_R.release(); h->h_p.release(); h->h_plan.release(); h->h_out.release();
    for (hipEvent_t ev : h->ev_pool)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : h->ev_p2x)
        if (ev) (void)hipEventDestroy(ev);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

const char* sw_last_error(const sw_handle* h) { return h ? h->err.c_str() : "null handle"; }

void* sw_stream(sw_handle* h) { return h ? (void*)h->stream : nullptr; }

int sw_batch_upload(sw_handle* h, int32_t count, const sw_problem* probs) {
    if (!h) return SW_ERR_INVALID;
    if (count < 0 || (count > 0 && !probs)) return fail(h, SW_ERR_INVALID, "bad batch");
    SW_HIP(h, hipSetDevice(h->device));
    int64_t J = 0, P = 0;
    int32_t maxN = 0, maxT = 1;
    for (int32_t i = 0; i < count; ++i) {
        if (sw_validate_problem(&probs[i]) != 0)
            return fail(h, SW_ERR_INVALID, "invalid problem at index " + std::to_string(i));
        J += probs[i].num_jobs;
        P += (int64_t)probs[i].num_jobs * probs[i].future_rounds;
        maxN = std::max(maxN, probs[i].num_jobs);
        maxT = std::max(maxT, probs[i].future_rounds);
    }
    /* wait for any run still using the buffers */
    SW_HIP(h, hipStreamSynchronize(h->stream));
    if (collect_timing(h) != SW_OK) return SW_ERR_HIP;
    /* the previous batch is gone from here on: a reserve below frees the
     * old buffers before it allocates, so a failure must leave no batch
     * described that run / download could touch */
    h->loaded = false;
    h->count = 0;
    h->total_jobs = 0;
    h->total_plan = 0;
    const size_t Jz = (size_t)std::max<int64_t>(J, 1);
    if (h->d_inst.reserve(std::max(count, 1)) || h->d_out.reserve(std::max(count, 1)) ||
        h->d_w.reserve(Jz) || h->d_F.reserve(Jz) || h->d_E.reserve(Jz) ||
        h->d_planned.reserve(Jz) || h->d_d.reserve(Jz) || h->d_R.reserve(Jz) ||
        h->d_p.reserve(Jz) || h->d_masks.reserve(Jz) || h->d_nb.reserve(Jz) ||
        h->d_lvl.reserve(std::max(count, 1)) || h->d_plan.reserve((size_t)std::max<int64_t>(P, 1)))
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
    if (h->h_w.reserve(Jz) || h->h_F.reserve(Jz) || h->h_E.reserve(Jz) || h->h_d.reserve(Jz) ||
        h->h_R.reserve(Jz) || h->h_p.reserve(Jz) || h->h_planned.reserve(Jz) ||
        h->h_plan.reserve((size_t)std::max<int64_t>(P, 1)) ||
        h->h_out.reserve(std::max(count, 1)))
        return fail(h, SW_ERR_HIP, "pinned allocation failed");
    h->inst.resize(count);
    h->Ns.resize(count);
    h->Ts.resize(count);
    int64_t jo = 0, po = 0;
    for (int32_t i = 0; i < count; ++i) {
        const sw_problem& pr = probs[i];
        sw_inst_dev& d = h->inst[i];
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
        const size_t n = (size_t)pr.num_jobs;
        if (n) {
            memcpy(h->h_w.p + jo, pr.nworkers, n * sizeof(int32_t));
            memcpy(h->h_F.p + jo, pr.completed_epochs, n * sizeof(int32_t));
            memcpy(h->h_E.p + jo, pr.total_epochs, n * sizeof(int32_t));
            memcpy(h->h_d.p + jo, pr.epoch_duration, n * sizeof(double));
            memcpy(h->h_R.p + jo, pr.remaining_runtime, n * sizeof(double));
            memcpy(h->h_p.p + jo, pr.priority, n * sizeof(double));
        }
        h->Ns[i] = pr.num_jobs;
        h->Ts[i] = pr.future_rounds;
        jo += pr.num_jobs;
        po += (int64_t)pr.num_jobs * pr.future_rounds;
    }
    h->maxN = maxN;
    h->maxT = maxT;
    if (count > 0) {
        hipStream_t s = h->stream;
        SW_HIP(h, hipMemcpyAsync(h->d_inst.p, h->inst.data(), count * sizeof(sw_inst_dev),
                                 hipMemcpyHostToDevice, s));
        if (J > 0) {
            SW_HIP(h, hipMemcpyAsync(h->d_w.p, h->h_w.p, J * 4, hipMemcpyHostToDevice, s));
            SW_HIP(h, hipMemcpyAsync(h->d_F.p, h->h_F.p, J * 4, hipMemcpyHostToDevice, s));
            SW_HIP(h, hipMemcpyAsync(h->d_E.p, h->h_E.p, J * 4, hipMemcpyHostToDevice, s));
            SW_HIP(h, hipMemcpyAsync(h->d_d.p, h->h_d.p, J * 8, hipMemcpyHostToDevice, s));
            SW_HIP(h, hipMemcpyAsync(h->d_R.p, h->h_R.p, J * 8, hipMemcpyHostToDevice, s));
            SW_HIP(h, hipMemcpyAsync(h->d_p.p, h->h_p.p, J * 8, hipMemcpyHostToDevice, s));
        }
        SW_HIP(h, hipStreamSynchronize(s));
    }
    h->count = count;
    h->total_jobs = J;
    h->total_plan = P;
    h->loaded = true;
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
    sw_batch_dev B;
    memset(&B, 0, sizeof(B));
    B.inst = h->d_inst.p;
    B.count = h->count;
    B.KT = h->maxT <= 32 ? 32 : 64;
    B.w = h->d_w.p;
    B.d = h->d_d.p;
    B.F = h->d_F.p;
    B.E = h->d_E.p;
    B.R = h->d_R.p;
    B.p = h->d_p.p;
    B.plan = h->d_plan.p;
    B.planned = h->d_planned.p;
    B.masks = h->d_masks.p;
    B.out = h->d_out.p;
    B.nb = h->d_nb.p;
    B.lvl = h->d_lvl.p;
#ifdef SW_STAMPS
    B.stamps = h->d_stamps.p;
#endif
    const int one = h->maxN <= SW_LDS_JOBS && h->maxT <= 32;
    if (!one) {
        B.ws.u8 = h->d_ws_u8.p;
        B.ws.u64 = h->d_ws_u64.p;
        B.ws.sort = h->d_ws_sort.p;
        B.ws.keys = h->d_ws_keys.p;
        B.ws.jc = h->d_ws_jc.p;
    }
    const size_t lds = sw_plan_kernel_lds_bytes(one);
    if (h->timing) {
        if (h->ev_used == kEventPairs && collect_timing(h) != SW_OK) return SW_ERR_HIP;
        SW_HIP(h, hipEventRecord(h->ev_pool[2 * h->ev_used], h->stream));
    }
    /* on-chip batches of more instances than CUs: level-search kernel, pack
     * kernel, full kernel for the instances the pack kernel leaves
     * (sw_kernels.hip) — the split buys several instances per CU; up to one
     * instance per CU (a scheduler's single solve) the full kernel alone is
     * one launch instead of three, and otherwise the full kernel for every
     * instance */
#ifdef SW_STAMPS
    const bool split = false; /* diagnostic builds time the phases inside the full kernel */
#else
    const bool split = one && B.count > kSplitMinCount;
#endif
    hipError_t e = split ? sw_launch_split(&B, h->stream) : sw_launch_plan(&B, B.KT, one, lds, h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "plan kernel launch");
    if (h->timing) {
        SW_HIP(h, hipEventRecord(h->ev_pool[2 * h->ev_used + 1], h->stream));
        SW_HIP(h, hipEventRecord(h->ev_p2x[2 * h->ev_used], h->stream));
    }
    /* the P2 exchange step (sw_p2x_kernel.hip) on the plan kernel's masks */
    e = sw_launch_p2x(&B, h->maxN, h->maxT, h->d_p2ws.p, h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "sw_p2x_kernel launch");
    if (h->timing) {
        SW_HIP(h, hipEventRecord(h->ev_p2x[2 * h->ev_used + 1], h->stream));
        h->ev_used++;
    }
    return SW_OK;
}

int sw_batch_download(sw_handle* h, sw_result* res) {
    if (!h) return SW_ERR_INVALID;
    if (!h->loaded) return fail(h, SW_ERR_INVALID, "no batch uploaded");
    if (h->count > 0 && !res) return fail(h, SW_ERR_INVALID, "null result array");
    SW_HIP(h, hipSetDevice(h->device));
    hipStream_t s = h->stream;
    if (h->count > 0) {
        if (h->total_plan > 0)
            SW_HIP(h, hipMemcpyAsync(h->h_plan.p, h->d_plan.p, h->total_plan,
                                     hipMemcpyDeviceToHost, s));
        if (h->total_jobs > 0)
            SW_HIP(h, hipMemcpyAsync(h->h_planned.p, h->d_planned.p, h->total_jobs * 4,
                                     hipMemcpyDeviceToHost, s));
        SW_HIP(h, hipMemcpyAsync(h->h_out.p, h->d_out.p, h->count * sizeof(sw_out_dev),
                                 hipMemcpyDeviceToHost, s));
    }
    SW_HIP(h, hipStreamSynchronize(s));
    if (collect_timing(h) != SW_OK) return SW_ERR_HIP;
    int rc = SW_OK;
    for (int32_t i = 0; i < h->count; ++i) {
        const sw_inst_dev& d = h->inst[i];
        const sw_out_dev& o = h->h_out.p[i];
        sw_result& r = res[i];
        if (r.plan && d.N > 0) memcpy(r.plan, h->h_plan.p + d.plan_off, (size_t)d.N * d.T);
        if (r.planned_rounds && d.N > 0)
            memcpy(r.planned_rounds, h->h_planned.p + d.job_off, (size_t)d.N * 4);
        r.objective = o.objective;
        r.utility = o.utility;
        r.makespan = o.makespan;
        r.p2_objective = o.p2_objective;
        r.bound = o.bound;
        r.iters = o.iters;
        r.status = o.status;
        if (o.status & SW_STATUS_P2_FALLBACK) rc = SW_FALLBACK;
    }
    return rc;
}

int sw_plan_solve_batch(sw_handle* h, int32_t count, const sw_problem* probs, sw_result* res) {
    int rc = sw_batch_upload(h, count, probs);
    if (rc < 0) return rc;
    rc = sw_batch_run(h);
    if (rc < 0) return rc;
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
