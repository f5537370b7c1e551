// Device trace generation for the recursion machine's Poseidon2WideDeg3 chip: the reference's
// poseidon2_wide_event_to_row_koalabear(input, row, sbox_state = true) (crates/recursion/core/src/
// sys.rs:102-106, include/poseidon2_wide.hpp) as one whole-trace kernel.  See include/zkm_tracegen.h.
//
// Each 16-lane row of a wavefront owns one trace row: the permutation of its event's input in the
// 16-lane form (lane l holds state word l, linear layers as DPP adds), every round state, s0 column and
// s-box cube written as it is produced (columns/permutation.rs:20-72 layout: external states [8][16],
// internal state [16], s0 [12], output [16], external s-boxes [8][16], internal s-boxes [13]).  The
// arithmetic stays in Montgomery form (kb31.cuh) and each cell is reduced to canonical on its way
// into LDS; a workgroup's 16 rows (20 KB) then leave as one contiguous row-major span in 16-byte
// stores.  Rows >= n are the permutation of zero, the reference's dummy row (trace.rs), so the buffer
// needs no clearing.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/zkm_hip.h"
#include "../../include/zkm_tracegen.h"
#include "kb31.cuh"
#include "p2.cuh"

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
constexpr int ROWS = 16, NTH = 16 * ROWS;  // rows per workgroup, 16 lanes per row

constexpr uint32_t P = kb::P;
static_assert(ROWS * COLS % 4 == 0, "tile of whole 16-byte stores");

// One row per 16-lane DPP row of the wavefront (the p2x16 form of p2.cuh, lane l holds state word l):
// each lane writes its own words of every round state and external s-box, lane 0 the internal s-boxes
// and s0 columns.  16 rows per 256-thread workgroup: a 20 KB LDS tile, so a CU keeps 8 workgroups.
__global__ __launch_bounds__(NTH) void k_p2wide_rows(const uint32_t *__restrict__ ev, uint64_t n, uint32_t repr,
                                                     uint32_t *__restrict__ out, uint64_t nrows) {
    using namespace kb;
    __shared__ uint32_t tile[ROWS * COLS];
    const uint32_t t = threadIdx.x, rl = t >> 4, l = t & 15;
    const uint64_t row0 = (uint64_t)blockIdx.x * ROWS, row = row0 + rl;
    uint32_t *my = tile + rl * COLS;
    const p2x16::Lane c = p2x16::lane_consts((int)l);
    const uint32_t x0 = row < n ? ev[row * 32 + l] : 0u;  // Poseidon2Io: input[16] then output[16]
    uint32_t x = repr == ZKM_REPR_MONTGOMERY ? (x0 < P ? x0 : x0 - P) : to_mont(x0);
    my[C_EXT + l] = from_mont(x);
    x = p2x16::external(x);
#pragma unroll
    for (int r = 0; r < NE / 2; r++) {
        x = cube(add(x, c.rc[r]));
        my[C_ESB + r * W + l] = from_mont(x);
        x = p2x16::external(x);
        my[(r == NE / 2 - 1 ? C_INT : C_EXT + (r + 1) * W) + l] = from_mont(x);
    }
#pragma unroll
    for (int r = 0; r < NI; r++) {
        const uint32_t y = cube(add(x, p2::RC.inr[r]));
        if (l == 0) {
            x = y;
            my[C_ISB + r] = from_mont(y);
        }
        uint32_t sum = add(x, p2x16::dpp<p2x16::ROR(1)>(x));
        sum = add(sum, p2x16::dpp<p2x16::ROR(2)>(sum));
        sum = add(sum, p2x16::dpp<p2x16::ROR(4)>(sum));
        sum = add(sum, p2x16::dpp<p2x16::ROR(8)>(sum));
        x = add(mul(x, c.dg), sum);
        if (l == 0 && r < NI - 1) my[C_S0 + r] = from_mont(x);
    }
    my[C_EXT + (NE / 2) * W + l] = from_mont(x);
#pragma unroll
    for (int r = NE / 2; r < NE; r++) {
        x = cube(add(x, c.rc[r]));
        my[C_ESB + r * W + l] = from_mont(x);
        x = p2x16::external(x);
        my[(r == NE - 1 ? C_OUT : C_EXT + (r + 1) * W) + l] = from_mont(x);
    }
    __syncthreads();
    // the tile's rows are one contiguous span of the row-major trace (nrows is a multiple of 16)
    uint4 *dst = reinterpret_cast<uint4 *>(out + row0 * COLS);
    for (uint32_t q = t; q < ROWS * COLS / 4; q += NTH) {
        const uint32_t *src = tile + 4 * q;
        dst[q] = make_uint4(src[0], src[1], src[2], src[3]);
    }
}

// ExpReverseBitsLen: one thread per event walks its rows in order (accum_i = accum_{i-1}^2 * multiplier_i,
// the square-and-multiply of x^rev(e)); events are short (one row per exponent bit).
__global__ __launch_bounds__(256) void k_exp_rev_rows(const uint32_t *__restrict__ base, const uint32_t *__restrict__ bits,
                                                      const uint64_t *__restrict__ off, uint64_t n, uint32_t repr,
                                                      uint32_t *__restrict__ out) {
    using namespace kb;
    const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    auto in = [&](uint32_t v) { return repr == ZKM_REPR_MONTGOMERY ? (v < P ? v : v - P) : to_mont(v); };
    const uint32_t x = in(base[e]);
    uint32_t acc = ONE;
    for (uint64_t r = off[e]; r < off[e + 1]; r++) {
        const uint32_t b = in(bits[r]);
        const uint32_t mult = b == ONE ? x : ONE;
        const uint32_t psq = mul(acc, acc), psqm = mul(psq, mult);
        acc = psqm;
        uint32_t *row = out + r * ZKM_EXP_REVERSE_BITS_LEN_WIDTH;
        row[0] = from_mont(x);
        row[1] = from_mont(b);
        row[2] = from_mont(psq);
        row[3] = from_mont(psqm);
        row[4] = from_mont(acc);
        row[5] = from_mont(mul(acc, acc));
        row[6] = from_mont(mult);
    }
}

// Recursion chips whose main rows are their events (zkm_recursion_events_to_trace): with k events of w words
// per row the trace's word j (row-major) is event word j, so one pass writes every word of the trace, 16
// bytes per thread: event words converted to canonical, zero past the events.
__global__ __launch_bounds__(256) void k_event_rows(const uint32_t *__restrict__ ev, uint64_t n_words, uint32_t repr,
                                                    uint32_t *__restrict__ out, uint64_t total_words) {
    using namespace kb;
    const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t w0 = 4 * q;
    if (w0 >= total_words) return;
    auto canon = [&](uint32_t v) { return repr == ZKM_REPR_MONTGOMERY ? from_mont(v < P ? v : v - P) : (v < P ? v : v - P); };
    uint32_t v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = w0 + i < n_words ? canon(ev[w0 + i]) : 0u;
    reinterpret_cast<uint4 *>(out)[q] = make_uint4(v[0], v[1], v[2], v[3]);
}

}  // namespace zkm::rtg

using namespace zkm::rtg;

extern "C" int zkm_recursion_events_to_trace(uint32_t chip, const uint32_t *events, uint64_t n, uint32_t repr,
                                             uint32_t *trace, uint64_t height, void *stream) {
    // (words per event, events per row), indexed by ZKM_REC_CHIP_*
    static const uint32_t layout[8][2] = {{3, 4}, {12, 4}, {13, 1}, {5, 1}, {33, 1}, {1, 1}, {4, 2}, {1, 0}};
    if (chip > ZKM_REC_CHIP_MEMORY_CONST || !trace || (n && !events) || height < 16 || (height & (height - 1)) ||
        (repr != ZKM_REPR_CANONICAL && repr != ZKM_REPR_MONTGOMERY) ||
        (chip == ZKM_REC_CHIP_MEMORY_CONST ? n != 0 : n > height * layout[chip][1])) {
        g_last_error = "zkm_recursion_events_to_trace: bad arguments (known chip, n events fitting height rows, "
                       "height a power of two >= 16, repr canonical or Montgomery)";
        return ZKM_ERR_ARG;
    }
    const uint64_t w = layout[chip][0], width = chip == ZKM_REC_CHIP_MEMORY_CONST ? 1 : w * layout[chip][1];
    const uint64_t total = height * width;  // a multiple of 16: height is
    hipLaunchKernelGGL(k_event_rows, dim3((uint32_t)((total / 4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       events, n * w, repr, trace, total);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_recursion_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

extern "C" int zkm_poseidon2_wide_events_to_trace(const zkm_poseidon2_event *events, uint64_t n, uint32_t repr,
                                                  uint32_t *trace, uint64_t height, void *stream) {
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1)) ||
        (repr != ZKM_REPR_CANONICAL && repr != ZKM_REPR_MONTGOMERY)) {
        g_last_error = "zkm_poseidon2_wide_events_to_trace: bad arguments (need n <= height, height a power of two "
                       ">= 16, repr canonical or Montgomery)";
        return ZKM_ERR_ARG;
    }
    hipLaunchKernelGGL(k_p2wide_rows, dim3((uint32_t)(height / ROWS)), dim3(NTH), 0, (hipStream_t)stream,
                       (const uint32_t *)events, n, repr, trace, height);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_poseidon2_wide_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

extern "C" int zkm_exp_reverse_bits_events_to_trace(const uint32_t *base, const uint32_t *bits, const uint64_t *offsets,
                                                    uint64_t n, uint32_t repr, uint32_t *trace, uint64_t height,
                                                    void *stream) {
    if (!trace || !offsets || (n && (!base || !bits)) || height < 16 || (height & (height - 1)) ||
        (repr != ZKM_REPR_CANONICAL && repr != ZKM_REPR_MONTGOMERY)) {
        g_last_error = "zkm_exp_reverse_bits_events_to_trace: bad arguments (height a power of two >= 16, repr "
                       "canonical or Montgomery)";
        return ZKM_ERR_ARG;
    }
    hipStream_t s = (hipStream_t)stream;
    hipError_t err = hipMemsetAsync(trace, 0, (size_t)height * ZKM_EXP_REVERSE_BITS_LEN_WIDTH * 4, s);
    if (err == hipSuccess && n) {
        hipLaunchKernelGGL(k_exp_rev_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, base, bits, offsets, n,
                           repr, trace);
        err = hipGetLastError();
    }
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_exp_reverse_bits_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}
