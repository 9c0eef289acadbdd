/*
 * sw_dist.hip — sharded single-instance solve (placeholder until the RCCL
 * path lands).
 */
#include <hip/hip_runtime.h>

#include "../../include/shockwave_amd.h"

extern "C" {

int sw_dist_unique_id(void* out_bytes) {
    (void)out_bytes;
    return SW_ERR_NOT_BUILT;
}

int sw_dist_init(sw_handle* h, const void* unique_id, int32_t rank, int32_t world) {
    (void)h; (void)unique_id; (void)rank; (void)world;
    return SW_ERR_NOT_BUILT;
}

int sw_dist_plan_solve(sw_handle* h, const sw_problem* local, int64_t job_offset,
                       int64_t total_jobs, sw_result* res) {
    (void)h; (void)local; (void)job_offset; (void)total_jobs; (void)res;
    return SW_ERR_NOT_BUILT;
}

}
