/*
 * sw_handle.h — the opaque sw_handle of include/shockwave_amd.h (private to
 * the library: sw_api.hip, sw_shard.hip) and small RAII-free buffer helpers.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/shockwave_amd.h"
#include "sw_device.h"

struct sw_shard_state;

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;  // elements
    hipError_t reserve(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 1);
        hipError_t e = hipMalloc((void**)&p, want * sizeof(T));
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

template <typename T>
struct HostBuf {
    T* p = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 1);
        hipError_t e = hipHostMalloc((void**)&p, want * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct sw_handle {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    /* batch description (host) */
    bool loaded = false; /* a batch upload completed (run / download need one) */
    bool keep_masks = true;   /* sw_batch_run stores plan_masks (sw_batch_keep_masks) */
    bool masks_valid = false; /* the last run stored them */
    int32_t count = 0;
    int64_t total_jobs = 0;
    int64_t total_plan = 0;
    int32_t maxN = 0, maxT = 0;
    std::vector<sw_inst_dev> inst;
    std::vector<int32_t> Ns, Ts;
    /* device */
    sw_inst_dev* d_inst = nullptr; /* view: the head of d_in */
    /* the per-job inputs of a batch as one block (one H2D for a whole
     * batch), and its outputs as another (one D2H): views set per batch by
     * sw_api.hip set_views() */
    DevBuf<unsigned char> d_in, d_res;
    int32_t *d_w = nullptr, *d_F = nullptr, *d_E = nullptr, *d_planned = nullptr;
    double *d_d = nullptr, *d_R = nullptr, *d_p = nullptr;
    uint8_t* d_plan = nullptr;
    sw_out_dev* d_out = nullptr;
    size_t in_bytes = 0, res_bytes = 0; /* the current batch's block sizes */
    DevBuf<uint8_t> d_ws_u8;
    DevBuf<uint64_t> d_ws_u64, d_ws_sort;
    DevBuf<float> d_ws_keys;
    DevBuf<sw_jobc> d_ws_jc;
    DevBuf<uint64_t> d_masks;     /* final round masks (plan kernel → P2 exchange) */
    DevBuf<uint8_t> d_nb;         /* level-search counts (level kernel → pack kernel) */
    DevBuf<sw_lvl_dev> d_lvl;     /* level-search results per instance                */
    DevBuf<unsigned char> d_p2ws; /* P2 exchange arrays of instances > SW_LDS_JOBS jobs */
    DevBuf<uint64_t> d_stamps; /* SW_STAMPS diagnostic builds */
    /* pinned staging */
    HostBuf<unsigned char> h_in, h_res; /* the blocks' pinned mirrors */
    int32_t *h_w = nullptr, *h_F = nullptr, *h_E = nullptr, *h_planned = nullptr;
    double *h_d = nullptr, *h_R = nullptr, *h_p = nullptr;
    uint8_t* h_plan = nullptr;
    sw_out_dev* h_out = nullptr;
    HostBuf<uint64_t> h_masks;    /* bit-packed plans (sw_result.plan_masks) */
    sw_inst_dev* h_inst = nullptr; /* view: the head of h_in */
    /* host-boundary chunk pipeline (sw_plan_solve_batch): copy streams and
     * per-chunk events, created on first use */
    hipStream_t up = nullptr, dn = nullptr;
    std::vector<hipEvent_t> ev_chunk;
    /* sw_batch_run over several streams (run_streams in sw_api.hip): the
     * extra streams and their fork / join events, created on first use */
    std::vector<hipStream_t> xs;
    std::vector<hipEvent_t> ev_xs;
    /* the batch being uploaded (described once its upload completes) */
    int32_t pend_count = 0;
    int64_t pend_jobs = 0, pend_plan = 0;
    /* timing: one event pair per timed launch, collected lazily */
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0; /* pairs recorded and not yet collected */
    std::vector<hipEvent_t> ev_p2x; /* one pair per timed launch of sw_p2x_kernel */
    double ms_plan = 0.0, ms_p2x = 0.0;
    int32_t runs = 0;
    /* sharded mode (sw_shard.hip) */
    sw_shard_state* shard = nullptr;
    /* MaxMinFairness allocation buffers (sw_mmf.hip) */
    void* mmf = nullptr;
};

/* sw_shard.hip: frees the sharded-mode state and communicator */
void sw_shard_release(sw_handle* h);
/* sw_mmf.hip: frees the MaxMinFairness buffers */
void sw_mmf_release(sw_handle* h);

