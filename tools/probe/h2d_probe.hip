// H2D probe: how fast can a 1.1 GB row-major trace in page-locked host memory reach HBM?
//   memcpy    : one hipMemcpyAsync
//   chunks/S  : 16 chunks round-robin over S streams
//   zerocopy  : a kernel reading the host buffer directly (16 B per lane) and writing HBM
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <chrono>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_pull(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += st) dst[i] = src[i];
}

int main() {
    const size_t bytes = (size_t)67 * 4 * (1 << 22);
    void *h, *d;
    CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    CK(hipMalloc(&d, bytes));
    memset(h, 1, bytes);
    hipStream_t ss[8];
    for (auto &s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto fn) {
        for (int w = 0; w < 2; w++) { fn(); CK(hipDeviceSynchronize()); }
        CK(hipDeviceSynchronize());
        auto t0 = std::chrono::high_resolution_clock::now();
        const int it = 5;
        for (int r = 0; r < it; r++) fn();
        CK(hipDeviceSynchronize());
        double ms = std::chrono::duration<double, std::milli>(std::chrono::high_resolution_clock::now() - t0).count() / it;
        printf("%-14s %8.2f ms  %6.1f GB/s\n", name, ms, bytes / ms / 1e6);
    };
    timeit("memcpy", [&] { CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, ss[0])); });
    for (int S : {1, 2, 4, 8}) {
        char nm[32]; snprintf(nm, 32, "chunks16/%d", S);
        timeit(nm, [&] {
            const size_t c = bytes / 16;
            for (int k = 0; k < 16; k++)
                CK(hipMemcpyAsync((char *)d + k * c, (char *)h + k * c, c, hipMemcpyHostToDevice, ss[k % S]));
        });
    }
    for (int g : {256, 1024, 4096}) {
        char nm[32]; snprintf(nm, 32, "zerocopy/%d", g);
        timeit(nm, [&] { hipLaunchKernelGGL(k_pull, dim3(g), dim3(256), 0, ss[0], (const uint4 *)h, (uint4 *)d, bytes / 16); });
    }
    return 0;
}
