// Device trace generation for the recursion machine's Poseidon2WideDeg3 chip: the reference's
// poseidon2_wide_event_to_row_koalabear(input, row, sbox_state = true) (crates/recursion/core/src/
// sys.rs:102-106, include/poseidon2_wide.hpp) as one whole-trace kernel.  See include/zkm_tracegen.h.
//
// Each thread owns one row: the permutation of its event's input, every round state, s0 column and
// s-box cube written as it is produced (columns/permutation.rs:20-72 layout: external states [8][16],
// internal state [16], s0 [12], output [16], external s-boxes [8][16], internal s-boxes [13]).  The
// arithmetic stays in Montgomery form (kb31.cuh) and each cell is reduced to canonical on its way
// into LDS.  A workgroup's 64 rows (64 x 313 words, 80 KB, odd pitch: conflict-free row-per-lane
// writes) then leave as one contiguous row-major span in 16-byte stores.  Rows >= n are the
// permutation of zero, the reference's dummy row (trace.rs), so the buffer needs no clearing.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/zkm_hip.h"
#include "../../include/zkm_tracegen.h"
#include "kb31.cuh"
#include "p2_rc.inc"

namespace zkm {
extern thread_local std::string g_last_error;
}
using zkm::g_last_error;

static_assert(sizeof(zkm_poseidon2_event) == 128, "Poseidon2Io<KoalaBear> layout");

namespace zkm::rtg {

constexpr int W = 16, NE = 8, NI = 13;
constexpr int C_EXT = 0, C_INT = C_EXT + NE * W, C_S0 = C_INT + W, C_OUT = C_S0 + NI - 1, C_ESB = C_OUT + W,
              C_ISB = C_ESB + NE * W, COLS = C_ISB + NI;
static_assert(COLS == ZKM_POSEIDON2_WIDE_DEG3_WIDTH, "PermutationSBox width");
constexpr int ROWS = 64;  // rows per workgroup (one wave)

// internal diagonal (poseidon2_wide/mod.rs:85-102) and round constants
constexpr uint32_t P = kb::P;
__constant__ uint32_t kDiag[W];     // Montgomery, uploaded at first use
__constant__ uint32_t kRc[30][W];   // RC_16_30 (crates/primitives/src/lib.rs:19), Montgomery

__device__ __forceinline__ void m4(uint32_t *x) {  // apply_m_4 (poseidon2_wide/mod.rs:40-54)
    const uint32_t t01 = kb::add(x[0], x[1]), t23 = kb::add(x[2], x[3]);
    const uint32_t t0123 = kb::add(t01, t23);
    const uint32_t t01123 = kb::add(t0123, x[1]), t01233 = kb::add(t0123, x[3]);
    const uint32_t y3 = kb::add(t01233, kb::dbl(x[0]));
    const uint32_t y1 = kb::add(t01123, kb::dbl(x[2]));
    x[0] = kb::add(t01123, t01);
    x[2] = kb::add(t01233, t23);
    x[1] = y1;
    x[3] = y3;
}

__device__ __forceinline__ void external_linear(uint32_t *s) {
#pragma unroll
    for (int j = 0; j < W; j += 4) m4(s + j);
    uint32_t sums[4];
#pragma unroll
    for (int k = 0; k < 4; k++) sums[k] = kb::add(kb::add(s[k], s[4 + k]), kb::add(s[8 + k], s[12 + k]));
#pragma unroll
    for (int j = 0; j < W; j++) s[j] = kb::add(s[j], sums[j & 3]);
}

__global__ __launch_bounds__(ROWS) void k_p2wide_rows(const uint32_t *__restrict__ ev, uint64_t n, uint32_t repr,
                                                      uint32_t *__restrict__ out, uint64_t nrows) {
    extern __shared__ uint32_t tile[];  // ROWS x COLS (pitch COLS, odd)
    const uint32_t t = threadIdx.x;
    const uint64_t row0 = (uint64_t)blockIdx.x * ROWS, row = row0 + t;
    uint32_t *my = tile + t * COLS;
    auto put = [&](int c, uint32_t v) { my[c] = kb::from_mont(v); };
    uint32_t s[W];
#pragma unroll
    for (int i = 0; i < W; i++) {
        const uint32_t x = row < n ? ev[row * 32 + i] : 0u;  // Poseidon2Io: input[16] then output[16]
        s[i] = repr == ZKM_REPR_MONTGOMERY ? (x < P ? x : x - P) : kb::to_mont(x);
        put(C_EXT + i, s[i]);
    }
    auto external_round = [&](int r) {
        if (r == 0) external_linear(s);
        const int rnd = r < NE / 2 ? r : r + NI;
#pragma unroll
        for (int i = 0; i < W; i++) {
            const uint32_t a = kb::add(s[i], kRc[rnd][i]);
            s[i] = kb::cube(a);
            put(C_ESB + r * W + i, s[i]);
        }
        external_linear(s);
        const int nxt = r == NE / 2 - 1 ? C_INT : r == NE - 1 ? C_OUT : C_EXT + (r + 1) * W;
#pragma unroll
        for (int i = 0; i < W; i++) put(nxt + i, s[i]);
    };
    for (int r = 0; r < NE / 2; r++) external_round(r);
    for (int r = 0; r < NI; r++) {
        const uint32_t a = kb::add(s[0], kRc[r + NE / 2][0]);
        s[0] = kb::cube(a);
        put(C_ISB + r, s[0]);
        uint32_t sum = s[0];
#pragma unroll
        for (int j = 1; j < W; j++) sum = kb::add(sum, s[j]);
#pragma unroll
        for (int j = 0; j < W; j++) s[j] = kb::add(kb::mul(s[j], kDiag[j]), sum);
        if (r < NI - 1) put(C_S0 + r, s[0]);
    }
#pragma unroll
    for (int i = 0; i < W; i++) put(C_EXT + (NE / 2) * W + i, s[i]);
    for (int r = NE / 2; r < NE; r++) external_round(r);
    __syncthreads();
    const uint64_t rows = nrows - row0 < (uint64_t)ROWS ? nrows - row0 : (uint64_t)ROWS;
    const uint32_t quads = (uint32_t)(rows * COLS / 4);  // rows is a multiple of 16
    uint4 *dst = reinterpret_cast<uint4 *>(out + row0 * COLS);
    for (uint32_t q = t; q < quads; q += ROWS) {
        const uint32_t *src = tile + 4 * q;
        dst[q] = make_uint4(src[0], src[1], src[2], src[3]);
    }
}

}  // namespace zkm::rtg

using namespace zkm::rtg;

extern "C" int zkm_poseidon2_wide_events_to_trace(const zkm_poseidon2_event *events, uint64_t n, uint32_t repr,
                                                  uint32_t *trace, uint64_t height, void *stream) {
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1)) ||
        (repr != ZKM_REPR_CANONICAL && repr != ZKM_REPR_MONTGOMERY)) {
        g_last_error = "zkm_poseidon2_wide_events_to_trace: bad arguments (need n <= height, height a power of two "
                       ">= 16, repr canonical or Montgomery)";
        return ZKM_ERR_ARG;
    }
    // round constants and diagonal in Montgomery form, uploaded once per process (device constant memory)
    static const hipError_t up = [] {
        uint32_t rc[30][W];
        for (int r = 0; r < 30; r++)
            for (int i = 0; i < W; i++) rc[r][i] = kb::to_mont(kP2RoundConstCanon[r][i]);
        hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(kRc), rc, sizeof(rc));
        uint32_t d[W];
        const uint32_t dc[W] = {P - 2, 1, 2, (P + 1) >> 1, 3, 4, (P - 1) >> 1, P - 3, P - 4, P - ((P - 1) >> 8),
                                P - ((P - 1) >> 3), P - 127, (P - 1) >> 8, (P - 1) >> 3, (P - 1) >> 4, 127};
        for (int i = 0; i < W; i++) d[i] = kb::to_mont(dc[i]);
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(kDiag), d, sizeof(d));
        return e;
    }();
    if (up != hipSuccess) {
        g_last_error = std::string("zkm_poseidon2_wide_events_to_trace: constant upload: ") + hipGetErrorString(up);
        return ZKM_ERR_HIP;
    }
    const size_t lds = (size_t)ROWS * COLS * sizeof(uint32_t);
    static const hipError_t attr =
        hipFuncSetAttribute((const void *)k_p2wide_rows, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)attr;
    hipLaunchKernelGGL(k_p2wide_rows, dim3((uint32_t)(height / ROWS + (height % ROWS != 0))), dim3(ROWS), lds,
                       (hipStream_t)stream, (const uint32_t *)events, n, repr, trace, height);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_poseidon2_wide_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}
