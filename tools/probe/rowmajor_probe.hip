// Access-pattern probe for VERDICT r05's "read the row-major upload in the first inverse strided pass": is reading
// k_ntt_s9b's 512-row x 32-column tiles (rows r S + c0 + t, S = 8192) straight out of a row-major 2^22 x 67 trace
// cheaper than transposing it first?  No arithmetic, the s9b thread layout (1024 threads, 16 words each), every
// tile written tile-major (64 KB contiguous) as the LDE's inverse pass writes it.
//   transpose   : row-major -> column-major (the product's k_to_col_major_rows scheme: 64 whole rows per
//                 256-thread block, an LDS tile of w x 65 words, 256-B column segments out)
//   cm_tiles    : the tiles read from the column-major copy (128-B row segments)
//   rm_tiles    : the tiles read from the row-major trace itself: each lane's word sits in its own 268-B row
//   rm_tiles_x  : rm_tiles with the 67 columns of one tile on consecutive workgroups of one XCD (L2 reuse of the
//                 rows the 67 column tiles share), as k_ntt_s9b orders its workgroups
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 rowmajor_probe.hip -o rowmajor_probe
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
constexpr uint32_t W = 67;

__global__ __launch_bounds__(256) void k_transpose(const uint32_t *__restrict__ in, uint32_t *__restrict__ out) {
    extern __shared__ uint32_t tile[];  // [c][r], pitch 65
    const uint64_t r0 = (uint64_t)blockIdx.x * 64;
    const uint32_t n = 64 * W;
    const uint32_t *src = in + r0 * W;
    for (uint32_t i = threadIdx.x; i < n; i += 256) {
        const uint32_t r = i / W, c = i - r * W;
        tile[c * 65 + r] = src[i];
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < W * 64; i += 256) {
        const uint32_t c = i / 64, r = i % 64;
        out[(uint64_t)c * N + r0 + r] = tile[c * 65 + r];
    }
}

// RM: source row-major (element (row, col) at row W + col) or column-major (col N + row); XCD: the workgroups of one
// tile's 67 columns consecutive on one XCD
template <bool RM, bool XCD>
__global__ __launch_bounds__(NTH) void k_tiles(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                              uint32_t tiles_per_col) {
    const uint32_t total = gridDim.x, lin = blockIdx.x;
    const uint32_t vid = XCD ? (lin & 7) * (total >> 3) + (lin >> 3) : lin;
    const uint32_t col = XCD ? vid % W : vid / tiles_per_col, tile = XCD ? vid / W : vid % tiles_per_col;
    const uint32_t t = threadIdx.x & 31, u = threadIdx.x >> 5;
    const uint32_t c0 = tile * COLS;
    uint32_t v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint64_t row = (uint64_t)(u + 32 * k) * S + c0 + t;
        v[k] = RM ? src[row * W + col] : src[(uint64_t)col * N + row];
    }
    const uint64_t tbase = (uint64_t)col * N + (uint64_t)tile * ROWS * COLS;
#pragma unroll
    for (int k = 0; k < 16; k++) dst[tbase + (uint64_t)(u + 32 * k) * COLS + t] = v[k] + 1;
}

int main() {
    const uint64_t words = W * N;
    uint32_t *rm, *cm, *out;
    CK(hipMalloc(&rm, words * 4));
    CK(hipMalloc(&cm, words * 4));
    CK(hipMalloc(&out, words * 4));
    CK(hipMemset(rm, 1, words * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t tpc = (uint32_t)(N / (ROWS * COLS));
    const dim3 grid((uint32_t)(W * tpc)), block(NTH);
    auto time = [&](const char *name, double bytes, auto launch) {
        for (int w = 0; w < 2; w++) launch();
        CK(hipEventRecord(e0));
        const int it = 10;
        for (int i = 0; i < it; i++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= it;
        printf("%-12s %8.3f ms  %7.0f GB/s (read + write of the 2^22 x 67 trace)\n", name, ms, bytes / ms / 1e6);
        return ms;
    };
    const double b2 = 2.0 * words * 4;
    const float tr = time("transpose", b2, [&] {
        hipLaunchKernelGGL(k_transpose, dim3((unsigned)(N / 64)), dim3(256), W * 65 * 4, 0, rm, cm);
    });
    const float cmt = time("cm_tiles", b2, [&] { hipLaunchKernelGGL((k_tiles<false, true>), grid, block, 0, 0, cm, out, tpc); });
    const float rmt = time("rm_tiles", b2, [&] { hipLaunchKernelGGL((k_tiles<true, false>), grid, block, 0, 0, rm, out, tpc); });
    const float rmx = time("rm_tiles_x", b2, [&] { hipLaunchKernelGGL((k_tiles<true, true>), grid, block, 0, 0, rm, out, tpc); });
    CK(hipGetLastError());
    printf("transpose + cm_tiles %.3f ms vs rm_tiles %.3f / rm_tiles_x %.3f ms\n", tr + cmt, rmt, rmx);
    return 0;
}
