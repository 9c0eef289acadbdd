/*
 * shockwave_amd.h — C-ABI of the MI355X-native Shockwave plan solver.
 *
 * Drop-in boundary.  The reference has no FFI: its boundary is the Python
 * method ShockwaveScheduler.current_round_schedule()
 * (reference scheduler/shockwave.py:77-91), which builds P1
 * (_eisenberg_gale_program, shockwave.py:330-388) and P2
 * (_prioritize_unfair_jobs, shockwave.py:281-328) in CVXPY and hands both to
 * Gurobi (_solve_gurobi, shockwave.py:400-411).  The native crossing in the
 * reference is problem.solve() (shockwave.py:401-408).  This header replaces
 * exactly that crossing: the host mirror (shockwave-replication_amd/shockwave.py)
 * runs the estimators as the reference does (shockwave.py:111-134, :255-278),
 * packs the per-job numbers into the SoA arrays below, and calls
 * sw_plan_solve() in place of the two problem.solve() calls.  The result is the
 * 0/1 plan that _generate_schedule (shockwave.py:390-398) reads back.
 *
 * Conventions
 *   - Plain C types only.  No C++ exceptions cross this boundary.
 *   - Caller owns every array passed in or out; the library copies what it
 *     needs.  The library owns its device buffers (one set per handle).
 *   - A handle is not thread-safe; the reference calls the solve under
 *     _scheduler_lock (scheduler.py:1729), so one handle per thread suffices.
 *   - Return codes: SW_OK (0) = solved; SW_FALLBACK (1) = solved, but P2
 *     could not place every P1 round and the P1 placement was kept (the
 *     reference's "P2 has no solution → return P1 schedule", shockwave.py:
 *     325-326); negative = error, message in sw_last_error().
 */
#ifndef SHOCKWAVE_AMD_H
#define SHOCKWAVE_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SW_ABI_VERSION 2

/* Limits of this build. */
#define SW_MAX_ROUNDS 64 /* future_rounds T (reference configs use 20 and 30) */
#define SW_MAX_BASES 8   /* len(log_approximation_bases) (reference: 6)        */
#define SW_MAX_WIDTH 255 /* nworkers of a job that fits the cluster (traces: 1-8) */

/* Return / status codes. */
#define SW_OK 0
#define SW_FALLBACK 1          /* P2 failed to place all rounds; P1 plan kept   */
#define SW_ERR_INVALID (-1)    /* bad sizes or non-finite / out-of-range input */
#define SW_ERR_HIP (-2)        /* HIP runtime error                             */
#define SW_ERR_CAPACITY (-3)   /* problem exceeds the handle's reserved sizes  */
#define SW_ERR_RCCL (-4)       /* RCCL error (sharded mode)                     */
#define SW_ERR_NOT_BUILT (-5)  /* feature not compiled into this library        */

/* Result status bits (sw_result.status). */
#define SW_STATUS_P1_REPACKED 0x1 /* aggregate P1 counts needed repair to pack
                                     (re-solved on a smaller budget, then single
                                     rounds added into stranded capacity) */
#define SW_STATUS_P2_FALLBACK 0x2 /* P2 placement fell back to the P1 plan    */
#define SW_STATUS_NO_PLANNED 0x4  /* no job has planned rounds (shockwave.py:319-320) */
/* Which P2 placement was kept: none of these bits = the
 * density order p_j/(n_j·w_j) placed every round. */
#define SW_STATUS_P2_WEIGHT_ORDER 0x8 /* the weight order p_j/n_j placed every round   */
#define SW_STATUS_P2_CLASSWISE 0x10   /* width classes repacked inside the P1 profile  */
#define SW_STATUS_P2_REPAIRED 0x20    /* density order with its width profile repaired */
/* The exchange step (negative-cycle cancelling over round moves, DESIGN.md
 * §3.6) improved the kept P2 placement. */
#define SW_STATUS_P2_EXCHANGED 0x40
/* The P1 objective is not certified within 1e-3 of `bound` (an upper bound
 * on the reference MILP's P1 optimum): bound − objective > 1e-3·|objective|.
 * Set where fragmenting widths or a lumpy level structure leave the greedy
 * rounding short of the relaxation, so a caller can tell a certified plan
 * from a best effort. */
#define SW_STATUS_P1_UNCERTIFIED 0x80

/*
 * One plan solve.  Field ↔ reference:
 *   num_jobs        len(self.job_metadata)                     shockwave.py:27-28
 *   future_rounds   self.future_rounds (T)                     shockwave.py:17
 *   num_gpus        self.num_gpus (G)                          shockwave.py:15
 *   round_duration  self.round_duration (Δ)                    shockwave.py:16
 *   regularizer     self.regularizer (k)                       shockwave.py:19
 *   bases           config["log_approximation_bases"] (β)      shockwave.py:100
 *   log_bases       log(β_b), log(0) → log(1e-6)               shockwave.py:101-105
 *   nworkers        job.nworkers (w_j)                         shockwave.py:66
 *   epoch_duration  np.mean(epoch_durations[:F+1]) (d_j)       shockwave.py:118-120
 *   completed_epochs job.completed_epochs (F_j)                shockwave.py:133
 *   total_epochs    job.total_epochs (E_j)                     shockwave.py:134
 *   remaining_runtime compute_remaining_runtime() call #2 (R_j) shockwave.py:261
 *   priority        FTF_j ** lambda (p_j)                      shockwave.py:368
 * All per-job arrays have num_jobs entries, in job_metadata insertion order.
 */
typedef struct sw_problem {
    int32_t num_jobs;
    int32_t future_rounds;
    int32_t num_gpus;
    int32_t num_bases;
    double round_duration;
    double regularizer;
    const double* bases;
    const double* log_bases;
    const int32_t* nworkers;
    const double* epoch_duration;
    const int32_t* completed_epochs;
    const int32_t* total_epochs;
    const double* remaining_runtime;
    const double* priority;
} sw_problem;

/*
 * Outputs.  plan is row-major [num_jobs][future_rounds], 1 = job j runs in
 * future round t (the round_schedule_vars[j][t] that _generate_schedule reads,
 * shockwave.py:394-396).  planned_rounds[j] = Σ_t plan[j][t].
 *   objective     P1 objective  (1/(N·T)) Σ p_j·L_j − k·max_j makespan_j   shockwave.py:373-379
 *   utility       the first term alone
 *   makespan      max_j max(0, R_j − d_j·e_j)                              shockwave.py:260-263, :363
 *   p2_objective  Σ_{n_j>0} p_j·(Σ_t t·y_jt)/n_j                           shockwave.py:309-322
 *   bound         an upper bound on the aggregate P1 optimum (and so on the
 *                 reference MILP's): the largest Lagrangian bound the level
 *                 search's branch and bound leaves (sw_bnb.h)
 *   iters         number of level/price evaluations the solver made
 * plan_masks (optional, ABI 2) is the same plan bit-packed: one word per job,
 * bit t = plan[j][t] — 8 bytes per job across the host boundary instead of
 * future_rounds.  Any of plan / plan_masks / planned_rounds may be NULL; the
 * batch entry points copy back only what some result of the batch asks for.
 * The sharded entry points (sw_dist_*) write plan and planned_rounds only and
 * reject a non-NULL plan_masks.
 */
typedef struct sw_result {
    uint8_t* plan;
    int32_t* planned_rounds;
    double objective;
    double utility;
    double makespan;
    double p2_objective;
    double bound;
    int32_t iters;
    int32_t status;
    uint64_t* plan_masks;
} sw_result;

/* Handle creation.  max_* reserve device capacity; 0 picks defaults. */
typedef struct sw_config {
    int32_t device;          /* HIP device ordinal                              */
    int32_t max_instances;   /* instances per batched call                      */
    int64_t max_total_jobs;  /* Σ num_jobs over a batch                         */
    int32_t max_jobs_per_instance;
    void* stream;            /* hipStream_t to launch on; NULL = own stream     */
} sw_config;

typedef struct sw_handle sw_handle;

int sw_abi_version(void);
sw_handle* sw_create(const sw_config* cfg);
void sw_destroy(sw_handle* h);
const char* sw_last_error(const sw_handle* h);
/* Message of the last sw_create() failure (no handle exists then). */
const char* sw_create_error(void);

/*
 * Single solve, host pointers in and out (synchronous).  Replaces the two
 * problem.solve() calls of shockwave.py:381 and :323 plus the read-back at
 * :390-398.
 */
int sw_plan_solve(sw_handle* h, const sw_problem* prob, sw_result* res);

/*
 * Batched solve of `count` independent problems (seed × cluster-size sweeps).
 * Host pointers; synchronous.  results[i] must point to caller buffers sized
 * for problems[i].
 */
int sw_plan_solve_batch(sw_handle* h, int32_t count, const sw_problem* problems,
                        sw_result* results);

/*
 * Device-resident batch (inputs already in HBM, for benchmarking and for
 * callers that keep the SoA on the GPU):
 *   sw_batch_upload   copies `count` problems into the handle's device SoA;
 *   sw_batch_run      enqueues the solve kernels on the handle's stream
 *                     (asynchronous, no host sync, graph-capturable); a
 *                     split batch of at most 2048 instances runs as two
 *                     chunks on the handle's stream and one internal stream
 *                     forked from and joined back into it by events, so the
 *                     call stays ordered on the handle's stream
 *                     (SW_RUN_STREAMS overrides the count, 1..4);
 *   sw_batch_download synchronises and copies plans/results back.
 */
int sw_batch_upload(sw_handle* h, int32_t count, const sw_problem* problems);
int sw_batch_run(sw_handle* h);
int sw_batch_download(sw_handle* h, sw_result* results);

/*
 * Whether sw_batch_run also stores the bit-packed plans (plan_masks, 8 bytes
 * per job in HBM) besides the plan bytes: keep = 1 (the default) or 0.  With
 * 0 the kernels skip those stores, and sw_batch_download of a run made so
 * refuses a result that asks for plan_masks (SW_ERR_INVALID).  The
 * host-buffer entry points (sw_plan_solve, sw_plan_solve_batch) decide from
 * their own results' plan_masks and ignore this setting.
 */
int sw_batch_keep_masks(sw_handle* h, int32_t keep);

/* The HIP stream the handle launches on (hipStream_t as void*). */
void* sw_stream(sw_handle* h);

/*
 * Per-kernel timing with HIP events recorded on the handle's stream around
 * each launch of sw_batch_run.  enable=1 turns it on (adds two event records
 * per kernel).  sw_kernel_times() synchronises and returns accumulated ms for
 * [0] the P2 exchange kernel (sw_p2x_kernel) and [1] the plan kernels
 * (sw_plan_kernel, or the split level / pack / slow-path kernels of large
 * on-chip batches), plus the number of runs.  Wherever the exchange step runs
 * fused inside the plan kernels — every on-chip batch of at most 256
 * instances (every single solve) and every split batch — [0] reads 0 and [1]
 * holds both stages, which are then not separable.
 */
int sw_set_timing(sw_handle* h, int32_t enable);
int sw_kernel_times(sw_handle* h, double* ms_p2x, double* ms_plan, int32_t* runs);

/*
 * Sharded single instance (jobs split across ranks, one process per GPU;
 * SURVEY.md §8(e), the 10k-job C4 shape).  Replaces the same problem.solve()
 * crossing as sw_plan_solve, for instances sharded by job.
 *
 * Every step of the solve is a pass over the rank's jobs plus one collective:
 * per-round demand / price-step counts and the makespan are all-reduced, the
 * deterministic-sum lane partials are all-gathered.  On RCCL
 * or the peer transport the whole common path is enqueued at once, with the
 * controller's decisions taken on the device, and the host reads one result.
 * Collectives run on RCCL over xGMI (sw_dist_init), peer memory
 * (sw_dist_enable_peer) or caller-supplied host collectives
 * (sw_dist_init_host, e.g. gloo).
 *
 * Sharding rule: world must divide 512 (1, 2, 4, … 512) and rank r must hold
 * exactly the jobs sw_dist_shard_range(total_jobs, world, r) returns.
 *
 * The result contract.  The plan is placed in V shares —
 * V = 8 for instances of 4,096 … 65,536 jobs on at least 512 GPUs at every
 * world ≤ 8, else V = world — each share's jobs alone in the share's part of
 * every round.  So:
 *   - P1 (planned_rounds, objective, utility, makespan, bound, the P1 status
 *     bits) is sw_plan_solve's on the whole instance, bit for bit, at every
 *     world size (or better, when only the shares place the level search's
 *     counts);
 *   - the plan rows and p2_objective are sw_plan_solve's when V = 1, and
 *     otherwise depend on V only, not on the world size: a large instance
 *     gives one result at worlds 1, 2, 4 and 8; P2 stays within 1.002 of the
 *     single instance's (tests/test_shard.py SHARE_P2_RATIO);
 *   - at every world the result equals the CPU shard engine
 *     (oracle/shard_twin.c) bit for bit.
 *
 * unique_id points to SW_NCCL_UNIQUE_ID_BYTES bytes produced by
 * sw_dist_unique_id() on rank 0 and broadcast by the caller.  local describes
 * this rank's slice of jobs (num_jobs = local count, scalars global);
 * job_offset/total_jobs place the slice.  res->plan / planned_rounds receive
 * this rank's rows; scalar results are global and identical on every rank;
 * res->iters counts collective steps.
 */
#define SW_NCCL_UNIQUE_ID_BYTES 128
int sw_dist_unique_id(void* out_bytes);
int sw_dist_init(sw_handle* h, const void* unique_id, int32_t rank, int32_t world);
int sw_dist_plan_solve(sw_handle* h, const sw_problem* local, int64_t job_offset,
                       int64_t total_jobs, sw_result* res);
int sw_dist_shard_range(int64_t total_jobs, int32_t world, int32_t rank, int64_t* lo,
                        int64_t* hi);
/*
 * Device-resident variant ("host (or device) pointers"):
 * local's per-job arrays are device pointers on the handle's device, and
 * res->plan / res->planned_rounds are device pointers (or NULL), written on
 * the handle's stream — nothing crosses PCIe but the step scalars.  The
 * per-job checks of the host path run on the device; a bad input on any rank
 * returns SW_ERR_INVALID on every rank.  Synchronous like sw_dist_plan_solve.
 */
int sw_dist_plan_solve_dev(sw_handle* h, const sw_problem* local, int64_t job_offset,
                           int64_t total_jobs, sw_result* res);

/*
 * Host collectives (blocking, in rank order, same call sequence on every
 * rank).  allgather: recv holds world × bytes, rank r's block at r·bytes.
 * Each returns 0 on success.
 */
typedef struct sw_host_comm {
    void* ctx;
    int (*allreduce_sum_i64)(void* ctx, int64_t* buf, int32_t n);
    int (*allreduce_max_u64)(void* ctx, uint64_t* buf, int32_t n);
    int (*allreduce_max_f64)(void* ctx, double* buf, int32_t n);
    int (*allgather)(void* ctx, const void* send, void* recv, int64_t bytes);
} sw_host_comm;
/* Sharded mode with host collectives instead of RCCL (the struct is copied;
 * comm->ctx must outlive the handle's solves). */
int sw_dist_init_host(sw_handle* h, const sw_host_comm* comm, int32_t rank, int32_t world);

/*
 * Peer-memory step transport (call after sw_dist_init / sw_dist_init_host,
 * on every rank, world ≤ SW_PEER_MAX_WORLD): every rank's exchange region is
 * mapped into every other rank (hipIpcOpenMemHandle; directly for ranks in
 * the same process), and from then on each step's all-reduce / all-gather is
 * one kernel on the handle's stream that stores this rank's partial into
 * every peer's region over xGMI and releases a sequence flag there, waits
 * (bounded: 10 s, or SW_PEER_TIMEOUT_MS from the environment at this call)
 * for every peer's flag in its own region, and combines in rank order —
 * instead of an RCCL call per step.  A timed-out wait returns SW_ERR_RCCL
 * and leaves the handle unusable (the ranks stopped at different exchanges):
 * every later solve on it returns SW_ERR_RCCL, rebuild the handle.  The
 * communicator set up by the init call is used once, to exchange the region
 * handles.  max_total_jobs bounds the instances (total_jobs) later solves
 * may pass (the regions are sized from it; larger ones return
 * SW_ERR_CAPACITY).  World 1 keeps the init call's transport.  If any rank
 * cannot allocate (fine-grained device memory is required) or map its side,
 * every rank returns an error and keeps the init call's transport.  Results are the same bits as with RCCL or host
 * collectives.  Each rank's exchange kernel waits on the GPU for its peers,
 * so ranks that share one device must run on distinct hardware queues: more
 * than GPU_MAX_HW_QUEUES / 2 ranks of one process on ONE device (the other
 * half is left to the process's other streams) return SW_ERR_INVALID on
 * every rank up front, and the init call's transport stays.
 */
#define SW_PEER_MAX_WORLD 64
int sw_dist_enable_peer(sw_handle* h, int64_t max_total_jobs);

/*
 * Gavel MaxMinFairness allocation for one worker type — the Fig-9 baseline
 * policy of the Shockwave comparison.  Replaces the ECOS solve of
 * policies/max_min_fairness.py:68-93 (MaxMinFairnessPolicy →
 * MaxMinFairnessPolicyWithPerf with unit throughputs, proportional.py:27-44),
 * which the simulator calls from _compute_allocation (scheduler.py:2386-2466):
 *
 *     maximise min_j c_j·x_j   s.t.  Σ_j sf_j·x_j ≤ num_workers,  0 ≤ x_j ≤ 1
 *
 * scale_factors[j] = job.scale_factor, coefficients[j] = scale_factor /
 * priority_weight, in sorted job-id order (policy.py:14-33).  allocation[j]
 * receives x_j: the unique optimum when capacity binds, otherwise the
 * analytic centre of the optimal face (the point an interior-point solver
 * such as ECOS converges to).  level (optional, 2 doubles) receives the
 * optimal min share t* and the capacity multiplier μ (0 when capacity binds).
 * Synchronous; num_jobs = 0 is a no-op (policy.flatten returns None).
 */
int sw_mmf_allocate(sw_handle* h, int32_t num_jobs, int32_t num_workers,
                    const int32_t* scale_factors, const double* coefficients, double* allocation,
                    double* level);

/*
 * The heterogeneity-aware allocation over several worker types:
 * MaxMinFairnessPolicyWithPerf.get_allocation (policies/max_min_fairness.py:
 * 44-100) with the base constraints of policy.py:57-63,
 *
 *     maximise min_j Σ_k coefficients[j][k]·x[j][k]
 *     s.t.  Σ_j scale_factors[j]·x[j][k] ≤ workers[k]  (every type k),
 *           Σ_k x[j][k] ≤ 1,  x ≥ 0,
 *
 * coefficients row-major [num_jobs][num_types] = throughput · priority weight
 * · scale factor (the caller's normalisation, max_min_fairness.py:57-73; the
 * Fig-9 policy, MaxMinFairnessPolicy, passes unit throughputs), jobs in sorted
 * id order, types in sorted name order (policy.py:28-44).  Solved exactly by
 * the simplex method (Bland's rule) on the GPU: allocation receives an
 * optimal vertex (row-major, unclipped), level[0] the optimal min share t*,
 * level[1] the pivots taken.  ECOS, the reference's solver, returns an
 * interior point of the same optimal face: the level is the LP's, the
 * allocation is one of its optima (the same one only where it is unique).
 * Limits: num_jobs ≤ 2048, 1 ≤ num_types ≤ 16, tableau ≤ 256 MB
 * (SW_ERR_CAPACITY).  Synchronous; num_jobs = 0 is a no-op.  Added in
 * round 5; reference interface: the WithPerf policy's get_allocation.
 */
int sw_mmf_allocate_types(sw_handle* h, int32_t num_jobs, int32_t num_types, const int32_t* workers,
                          const int32_t* scale_factors, const double* coefficients, double* allocation,
                          double* level);

#ifdef __cplusplus
}
#endif

#endif /* SHOCKWAVE_AMD_H */
