// Poseidon2 one-thread permutation throughput on MI355X (zkmips_amd/csrc/p2.cuh).  Each thread
// permutes its own state ITER times (no memory traffic inside the loop), so the rate is the
// VALU-issue-bound permutation rate.  (The A/B against the pre-optimisation form is recorded in
// profiles/r01_p2_ab.txt; that form is gone.)
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 p2_probe.hip -o p2_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#include "../../zkmips_amd/csrc/p2.cuh"

#define ITER 64

__global__ __launch_bounds__(256) void k_new(uint32_t *out) {
    uint32_t s[16];
    for (int k = 0; k < 16; k++) s[k] = (threadIdx.x * 16 + k) % kb::P;
    for (int i = 0; i < ITER; i++) p2::permute(s);
    uint32_t x = 0;
    for (int k = 0; k < 16; k++) x ^= s[k];
    out[blockIdx.x * 256 + threadIdx.x] = x;
}
int main() {
    const int blocks = 256 * 64;
    uint32_t *out;
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_new, dim3(blocks), dim3(256), 0, 0, out);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k_new, dim3(blocks), dim3(256), 0, 0, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double perms = 3.0 * blocks * 256 * ITER;
    printf("p2: %.3f ms  %.3e perms/s\n", ms / 3, perms / (ms * 1e-3));
    return 0;
}
