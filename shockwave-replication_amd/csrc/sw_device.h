/*
 * sw_device.h — device-side batch layout shared by sw_kernels.hip and the
 * host API (sw_api.hip).
 *
 * HBM layout (structure of arrays, one batch of independent instances):
 *   per-job inputs      w[int32] d[f64] F[int32] E[int32] R[f64] p[f64]
 *                       concatenated over instances (instance i starts at
 *                       inst[i].job_off)
 *   plan bytes          [Σ_i N_i·T_i] row-major per instance ([N_i][T_i])
 *   planned rounds      [Σ_i N_i] int32
 *   round masks         [Σ_i N_i] u64 (bit t: round t), the plan kernel's
 *                       final placement, read by the P2 exchange kernel
 *   per-instance out    sw_out_dev
 *   workspace (only for instances with N > SW_LDS_JOBS): per-job state,
 *                       fp32 key rows [job][KT], masks, sort keys.
 */
#pragma once
#include <stdint.h>

#include "sw_arith.h"

#define SW_STAMP_SLOTS 64 /* per-instance u64 slots of the SW_STAMPS diagnostic build (32…42: sw_p2x_kernel, 48…52: pack sub-phases) */
#define SW_LDS_JOBS 1024 /* instances up to this many jobs keep all state on chip (2 per thread) */

struct sw_inst_dev {
    int32_t N, T, G, nb;
    int64_t job_off;
    int64_t plan_off;
    double delta, k;
    double beta[SW_BMAX];
    double ell[SW_BMAX];
};

struct sw_out_dev {
    double objective, utility, makespan, p2_objective, bound;
    int32_t iters, status;
};

/* Global workspace, per job (used only when N > SW_LDS_JOBS). */
struct sw_ws_dev {
    uint8_t* u8;    /* [total_jobs][SW_WS_U8]      */
    uint64_t* u64;  /* [total_jobs][SW_WS_U64]     */
    uint64_t* sort; /* [2·total_jobs][2] sort keys  */
    float* keys;    /* [total_jobs][KT]             */
    sw_jobc* jc;    /* [total_jobs]                 */
};
#define SW_WS_U8 8   /* per-job u8 state arrays   */
#define SW_WS_U64 6  /* per-job u64 arrays        */
/* per-instance u64 padding of the u64 workspace: the round loop's position
 * slots (pmask, pst, pord; slot = (p mod PPL)·64 + p div PPL with
 * PPL = ⌈A/64⌉) reach up to A + 62, so each slot array holds N + 64 entries */
#define SW_WS_PAD_U64 192

/* Per-instance result of the level-search kernel (sw_level_kernel), read by
 * the pack kernel (sw_pack_kernel). */
struct sw_lvl_dev {
    double U, M, bound; /* utility and makespan of the best level's counts, P1 bound */
    int64_t passes;
};
/* out.status of an instance the pack kernel left to the full plan kernel */
#define SW_STATUS_SLOW_MARK 0x40000000

struct sw_batch_dev {
    const sw_inst_dev* inst;
    int32_t count;
    int32_t KT;
    const int32_t* w;
    const double* d;
    const int32_t* F;
    const int32_t* E;
    const double* R;
    const double* p;
    uint8_t* plan;
    int32_t* planned;
    uint64_t* masks;
    sw_out_dev* out;
    uint8_t* nb;      /* level-search counts per job (sw_level_kernel → sw_pack_kernel) */
    sw_lvl_dev* lvl;  /* per instance                                              */
    int32_t only_slow; /* sw_plan_kernel: solve only instances marked SW_STATUS_SLOW_MARK */
    sw_ws_dev ws;
    unsigned char* p2ws; /* P2 exchange arrays, SW_P2X_ARR_BYTES per job (sw_p2x_inst.h) */
    int32_t fuse_p2x;    /* sw_plan_kernel: run the exchange step after the solve (sw_p2x_inst.h) */
    int32_t want_masks;  /* sw_pack_kernel: store the final masks (a caller asked for plan_masks) */
    int32_t lds_bytes;   /* sw_pack_kernel: its dynamic LDS allocation (the exchange arrays' room) */
    uint64_t* stamps; /* diagnostic builds only (SW_STAMPS): [count][SW_STAMP_SLOTS] cycles (8…13: pack round-loop phases, 16…: level search, 32…: exchange) */
};
