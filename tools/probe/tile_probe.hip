// Access-pattern probe for the LDE's strided passes (k_ntt_s9b): is a 512-row x 32-column tile of 128-B row
// segments at a 32 KB stride (a 2^22-point column viewed as 512 x 8192) slower to move than contiguous
// memory, with the same 1024-thread workgroups and 16 words per thread and no arithmetic?
//   contig      : read and write 64 KB contiguous blocks
//   strided_rd  : read the tile's 512 segments (stride S), write a contiguous 64 KB block (tile-major)
//   strided_wr  : read a contiguous block, write the tile's segments
//   strided_rw  : both sides strided (k_ntt_s9b's pattern, minus the butterflies and the LDS exchanges)
// 67 columns of 2^22 words each (the FibCpu main trace), one launch per pattern; GB/s = 2 x bytes / time.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tile_probe.hip -o tile_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); }   \
    } while (0)

constexpr int LOGN = 22, LOGS = 13, ROWS = 512, COLS = 32, NTH = 1024;
constexpr uint64_t N = 1ull << LOGN, S = 1ull << LOGS;

// workgroup -> (column, tile); thread -> (u = tid >> 5 row group, t = tid & 31 column in the tile)
template <bool SRD, bool SWR>
__global__ __launch_bounds__(NTH) void k_tile(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                             uint32_t tiles_per_col) {
    const uint32_t col = blockIdx.x / tiles_per_col, tile = blockIdx.x % tiles_per_col;
    const uint32_t t = threadIdx.x & 31, u = threadIdx.x >> 5;
    const uint64_t cbase = (uint64_t)col * N;
    const uint64_t tbase = cbase + (uint64_t)tile * ROWS * COLS;  // tile-major: 64 KB per tile
    const uint32_t c0 = tile * COLS;                               // strided: the tile's first column
    uint32_t v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t r = u + 32 * k;  // 512 rows
        v[k] = SRD ? src[cbase + (uint64_t)r * S + c0 + t] : src[tbase + (uint64_t)r * COLS + t];
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t r = u + 32 * k;
        const uint32_t x = v[k] + 1;
        if (SWR) dst[cbase + (uint64_t)r * S + c0 + t] = x;
        else dst[tbase + (uint64_t)r * COLS + t] = x;
    }
}

int main() {
    const uint64_t W = 67, words = W * N;
    uint32_t *a, *b;
    CK(hipMalloc(&a, words * 4));
    CK(hipMalloc(&b, words * 4));
    CK(hipMemset(a, 1, words * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t tpc = (uint32_t)(N / (ROWS * COLS));
    const dim3 grid((uint32_t)(W * tpc)), block(NTH);
    auto run = [&](const char *name, auto kernel) {
        for (int w = 0; w < 2; w++) hipLaunchKernelGGL(kernel, grid, block, 0, 0, a, b, tpc);
        CK(hipDeviceSynchronize());
        const int it = 10;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; i++) hipLaunchKernelGGL(kernel, grid, block, 0, 0, a, b, tpc);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= it;
        printf("%-11s %7.3f ms  %6.2f TB/s (read + write)\n", name, ms, 2.0 * words * 4 / (ms * 1e-3) / 1e12);
    };
    for (int rep = 0; rep < 2; rep++) {
        run("contig", k_tile<false, false>);
        run("strided_rd", k_tile<true, false>);
        run("strided_wr", k_tile<false, true>);
        run("strided_rw", k_tile<true, true>);
    }
    return 0;
}
