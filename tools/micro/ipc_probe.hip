// Probe: can two processes on ONE GPU map each other's device memory through
// hipIpcGetMemHandle / hipIpcOpenMemHandle (dmabuf IPC), and does a kernel
// see a peer kernel's flag release within a bounded spin?  The exchange path
// of the sharded engine depends on both.
//   hipcc --offload-arch=gfx950 -O2 -o tools/micro/ipc_probe tools/micro/ipc_probe.hip
//   timeout -k 5 60 tools/micro/ipc_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/wait.h>
#include <unistd.h>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "[%d] %s: %s\n", (int)getpid(), #x, hipGetErrorString(e_)); \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

// rank r writes value v into peer's slot[r], then releases flag[r] = seq;
// then waits (bounded) for its own flag[1 - r] == seq and reads slot[1 - r].
__global__ void k_xchg(unsigned long long* mine, unsigned long long* peer, int r,
                       unsigned long long v, unsigned long long seq, unsigned long long* out) {
    if (threadIdx.x != 0) return;
    peer[r] = v;                 // slot r of the peer
    __threadfence_system();
    __hip_atomic_store(&peer[8 + r], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t t0 = wall_clock64();
    unsigned long long f = 0;
    while (true) {
        f = __hip_atomic_load(&mine[8 + (1 - r)], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (f == seq) break;
        if (wall_clock64() - t0 > 100ull * 1000 * 1000 * 2) break; // ~2 s at 100 MHz
        __builtin_amdgcn_s_sleep(2);
    }
    out[0] = f;
    out[1] = mine[1 - r];
    out[2] = wall_clock64() - t0;
}

static int run(int r, int wfd, int rfd) {
    CK(hipSetDevice(0));
    unsigned long long* buf;
    CK(hipMalloc(&buf, 4096));
    CK(hipMemset(buf, 0, 4096));
    CK(hipDeviceSynchronize());
    hipIpcMemHandle_t h;
    CK(hipIpcGetMemHandle(&h, buf));
    if (write(wfd, &h, sizeof(h)) != (ssize_t)sizeof(h)) return 3;
    hipIpcMemHandle_t ph;
    if (read(rfd, &ph, sizeof(ph)) != (ssize_t)sizeof(ph)) return 3;
    void* peer = nullptr;
    CK(hipIpcOpenMemHandle(&peer, ph, hipIpcMemLazyEnablePeerAccess));
    unsigned long long* out;
    CK(hipHostMalloc((void**)&out, 64, hipHostMallocDefault));
    double tot_us = 0.0;
    const int reps = 200;
    for (int s = 1; s <= reps; ++s) {
        hipLaunchKernelGGL(k_xchg, dim3(1), dim3(64), 0, 0, buf, (unsigned long long*)peer, r,
                           1000ull * s + r, (unsigned long long)s, out);
        CK(hipDeviceSynchronize());
        if (out[0] != (unsigned long long)s || out[1] != 1000ull * s + (1 - r)) {
            fprintf(stderr, "[rank %d] step %d: flag %llu value %llu\n", r, s, out[0], out[1]);
            return 4;
        }
        tot_us += out[2] / 100.0;
    }
    printf("rank %d: %d exchanges ok, mean in-kernel wait %.2f us\n", r, reps, tot_us / reps);
    CK(hipIpcCloseMemHandle(peer));
    return 0;
}

int main() {
    int a[2], b[2];
    if (pipe(a) || pipe(b)) return 1;
    pid_t p = fork();
    if (p == 0) return run(1, b[1], a[0]);
    int rc = run(0, a[1], b[0]);
    int st = 0;
    waitpid(p, &st, 0);
    const int crc = WIFEXITED(st) ? WEXITSTATUS(st) : 99;
    printf("parent rc %d child rc %d\n", rc, crc);
    return rc || crc;
}
