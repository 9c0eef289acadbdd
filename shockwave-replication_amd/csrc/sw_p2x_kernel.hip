/*
 * sw_p2x_kernel.hip — the P2 exchange step on the GPU (sw_p2x.h; DESIGN.md
 * §3.6): negative-cycle cancelling over round moves, bit-identical to the
 * sequential specification oracle/p2x_twin.c.  Reference: the P2 MILP,
 * shockwave.py:281-328 (Gurobi at MIPGap 1e-3).
 *
 * One 512-thread workgroup per instance, launched after the plan stage on
 * the same stream: the plan kernels leave every job's final round mask in
 * HBM (batch.masks); this kernel improves the masks of the instances whose
 * P2 placement placed every round, rewrites the plan bytes of the jobs that
 * moved and the P2 objective (sw_p2x_inst.h).  A batch solved by the full
 * plan kernel alone runs the same step at the end of that kernel instead.
 * The step itself is sw_p2x_block (sw_p2x_dev.h), which the sharded engine
 * runs on its gathered placement.
 * The step is latency-bound (a chain of small block phases), so the kernel is
 * lean (few VGPRs, ~50 KB LDS at 900 jobs × 30 rounds) and several instances
 * share a CU.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shockwave_amd.h"
#include "sw_arith.h"
#include "sw_block.h"
#include "sw_device.h"
#include "sw_p2x.h"
#include "sw_p2x_dev.h"
#include "sw_p2x_inst.h"

/* The batch kernel: instance blockIdx.x.  At ≤ 64 VGPRs and ~34 KB of LDS
 * four 512-thread workgroups share a CU. */
__global__ __launch_bounds__(SW_BLOCK, 8) void sw_p2x_kernel(sw_batch_dev B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    sw_p2x_instance(B, B.p2ws, smem, blockIdx.x);
}

/* LDS bytes of the batch kernel for instances up to maxN jobs, maxT rounds. */
extern "C" size_t sw_p2x_kernel_lds_bytes(int maxN, int maxT) {
    return ((sizeof(sw_p2x_lds) + 15) & ~(size_t)15) + sw_p2x_var_bytes(maxN, maxT);
}

extern "C" hipError_t sw_launch_p2x(const sw_batch_dev* B, int maxN, int maxT, hipStream_t stream) {
    const size_t lds = sw_p2x_kernel_lds_bytes(maxN, maxT);
    dim3 grid(B->count), block(SW_BLOCK);
    hipLaunchKernelGGL(sw_p2x_kernel, grid, block, lds, stream, *B);
    return hipGetLastError();
}

