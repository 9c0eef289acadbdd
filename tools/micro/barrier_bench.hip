// Microbenchmark: cost of one block reduction (DPP wave sum, LDS slot per
// wave, one barrier, read all slots) as in sw_block.h, vs workgroup size.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/barrier_bench barrier_bench.hip && ./barrier_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ int32_t dpp_incscan_i32(int32_t x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);
    return x;
}

template <int BLOCK, int MODE>
__global__ __launch_bounds__(BLOCK) void k(int iters, int32_t* out, uint64_t* cyc) {
    __shared__ int32_t slot[2][16];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int32_t v = threadIdx.x & 7;
    int par = 0;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        int32_t s;
        if (MODE == 0) { /* block sum, one barrier */
            s = __builtin_amdgcn_readlane(dpp_incscan_i32(v), 63);
            if (lane == 0) slot[par][w] = s;
            __syncthreads();
            int32_t t = 0;
#pragma unroll
            for (int q = 0; q < BLOCK / 64; ++q) t += slot[par][q];
            par ^= 1;
            v = (v + t) & 15;
        } else { /* wave-only scan (no barrier) */
            s = __builtin_amdgcn_readlane(dpp_incscan_i32(v), 63);
            v = (v + s) & 15;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[blockIdx.x] = v; cyc[blockIdx.x] = t1 - t0; }
}

template <int BLOCK, int MODE>
void run(const char* name, int grid) {
    int32_t* out; uint64_t* cyc;
    hipMalloc(&out, grid * 4); hipMalloc(&cyc, grid * 8);
    const int iters = 4096;
    hipLaunchKernelGGL((k<BLOCK, MODE>), dim3(grid), dim3(BLOCK), 0, 0, iters, out, cyc);
    hipDeviceSynchronize();
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL((k<BLOCK, MODE>), dim3(grid), dim3(BLOCK), 0, 0, iters, out, cyc);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    uint64_t* h = (uint64_t*)malloc(grid * 8);
    hipMemcpy(h, cyc, grid * 8, hipMemcpyDeviceToHost);
    double avg = 0; for (int i = 0; i < grid; ++i) avg += h[i]; avg /= grid;
    printf("%-28s block %4d grid %5d: %.1f memtime-ticks/iter, %.3f ms, %.1f ns/iter\n", name, BLOCK, grid,
           avg / iters, ms, ms * 1e6 / iters);
    hipFree(out); hipFree(cyc); free(h);
}

int main() {
    for (int g : {256, 512, 1024}) {
        run<512, 0>("block-reduce 1 barrier", g);
        run<256, 0>("block-reduce 1 barrier", g);
        run<1024, 0>("block-reduce 1 barrier", g);
        run<64, 0>("block-reduce 1 barrier", g);
        run<512, 1>("wave scan, no barrier", g);
    }
    return 0;
}
