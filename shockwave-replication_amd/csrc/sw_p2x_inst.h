/*
 * sw_p2x_inst.h — one instance's P2 exchange step on a workgroup, from the
 * plan kernel's HBM outputs to the rewritten plan rows and P2 objective
 * (DESIGN.md §3.6).  Shared by sw_p2x_kernel (sw_p2x_kernel.hip) and the
 * full plan kernel's fused form (sw_kernels.hip).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shockwave_amd.h"
#include "sw_arith.h"
#include "sw_block.h"
#include "sw_device.h"
#include "sw_p2x.h"
#include "sw_p2x_dev.h"

/*
 * The exchange step of instance inst on its workgroup, after the plan
 * kernel's emit (batch.masks, out[inst].status) — in sw_p2x_kernel, or at
 * the end of the full plan kernel when one launch solves the batch
 * (sw_kernels.hip).  Every early return is uniform over the workgroup.
 * The per-job arrays live in the workspace ws (SW_P2X_ARR_BYTES per job,
 * L2-resident while the instance runs) so that the LDS holds only the step's
 * own state (~30 KB at 900 jobs × 30 rounds).
 */
/* thread tid's jobs [j0, j1) of an N-job instance (the plan kernel's split).
 * The thread index goes through an empty asm so every call recomputes the
 * bound (one multiply) instead of the compiler keeping one copy live across
 * the exchange step: at the pack kernel's 64-VGPR cap that copy was spilled. */
__device__ __forceinline__ int sw_tid_opaque() {
    int x = (int)threadIdx.x;
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ int j0r(int N) { return sw_tid_opaque() * ((N + SW_BLOCK - 1) / SW_BLOCK); }
__device__ __forceinline__ int j1r(int N) {
    const int q = (N + SW_BLOCK - 1) / SW_BLOCK;
    return min(sw_tid_opaque() * q + q, N);
}

__device__ __forceinline__ void sw_p2x_instance(const sw_batch_dev& B, unsigned char* ws,
                                                unsigned char* smem, int inst) {
    const sw_inst_dev* I = &B.inst[inst];
    sw_out_dev* out = &B.out[inst];
    const int N = I->N, T = I->T, G = I->G;
    if (out->status & SW_STATUS_P2_FALLBACK) return; /* P1's x is kept as is (:325-326) */
    const int64_t jo = I->job_off;
    sw_p2x_lds* L = reinterpret_cast<sw_p2x_lds*>(smem);
    unsigned char* var = smem + ((sizeof(sw_p2x_lds) + 15) & ~(size_t)15);
    sw_blk blk;
    blk.X = &L->X;
    blk.par = 0;
    sw_p2x_arrays X;
    {
        unsigned char* base = ws + (size_t)SW_P2X_ARR_BYTES * jo;
        const size_t n = (size_t)N;
        X.cc = reinterpret_cast<double*>(base);
        X.cm = reinterpret_cast<uint64_t*>(X.cc + n);
        X.cw = reinterpret_cast<int32_t*>(X.cm + n);
        X.cj = X.cw + n;
    }
    /* compaction in job order: thread l takes jobs [l·q, (l+1)·q) (the
     * plan kernel's job split, so the P2 sum below has its lanes) */
    const int q = (N + SW_BLOCK - 1) / SW_BLOCK;
    const int j0 = threadIdx.x * q, j1 = min(j0 + q, N);
    int act = 0;
    for (int j = j0; j < j1; ++j) act += B.masks[jo + j] != 0ull;
    int A;
    const int a0 = blk.exscan(act, A);
    if (A > SW_P2X_AMAX) return;
    for (int j = j0, a = a0; j < j1; ++j) {
        const uint64_t m = B.masks[jo + j];
        if (!m) continue;
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
    if (nc == 0) return;
    /* rewrite the moved jobs' plan bytes; the P2 objective of the final
     * masks, summed like the plan kernel's emit.  The compaction offsets are
     * counted again (one scan; B.masks is unchanged until this loop) rather
     * than kept live through the step, where the 64-VGPR kernel spilled them */
    /* N read again through a volatile load, so the compiler recomputes the
     * job range and its addresses here instead of keeping the first ones */
    const int N2 = *(volatile const int*)&I->N;
    const int64_t jo2 = *(volatile const int64_t*)&I->job_off;
    int act2 = 0;
    for (int j = j0r(N2); j < j1r(N2); ++j) act2 += B.masks[jo2 + j] != 0ull;
    int A2;
    const int a0r = blk.exscan(act2, A2);
    uint8_t* plan = B.plan + I->plan_off;
    double acc = 0.0;
    for (int j = j0r(N2), a = a0r; j < j1r(N2); ++j) {
        const uint64_t m0 = B.masks[jo2 + j];
        if (!m0) {
            acc = acc + 0.0;
            continue;
        }
        const uint64_t m = X.cm[a++];
        if (m != m0) {
            B.masks[jo2 + j] = m;
            for (int t = 0; t < T; ++t) plan[(size_t)j * T + t] = (uint8_t)((m >> t) & 1ull);
        }
        const int cnt = __popcll(m);
        const int64_t Ssum = (int64_t)__popcll(m & 0xAAAAAAAAAAAAAAAAull) +
                             2 * (int64_t)__popcll(m & 0xCCCCCCCCCCCCCCCCull) +
                             4 * (int64_t)__popcll(m & 0xF0F0F0F0F0F0F0F0ull) +
                             8 * (int64_t)__popcll(m & 0xFF00FF00FF00FF00ull) +
                             16 * (int64_t)__popcll(m & 0xFFFF0000FFFF0000ull) +
                             32 * (int64_t)__popcll(m & 0xFFFFFFFF00000000ull);
        acc = acc + ((double)Ssum / (double)cnt) * B.p[jo2 + j];
    }
    const double P2 = blk.detsum(acc);
    if (threadIdx.x == 0) {
        out->p2_objective = P2;
        out->status |= SW_STATUS_P2_EXCHANGED;
    }
}

