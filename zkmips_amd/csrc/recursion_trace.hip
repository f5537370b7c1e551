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
#include "p2_rows.cuh"

namespace zkm {
extern thread_local std::string g_last_error;
}
using zkm::g_last_error;

static_assert(sizeof(zkm_poseidon2_event) == 128, "Poseidon2Io<KoalaBear> layout");

namespace zkm::rtg {

using p2rows::COLS;
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
    const uint32_t x0 = row < n ? ev[row * 32 + l] : 0u;  // Poseidon2Io: input[16] then output[16]
    p2rows::fill(repr == ZKM_REPR_MONTGOMERY ? (x0 < P ? x0 : x0 - P) : to_mont(x0), l, my);
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

// Preprocessed rows of the recursion chips from their instruction records (zkm_recursion_instrs_to_trace):
// one thread per trace row, the chip's instr_to_row for each of the row's entries, zero padding rows.
template <int CHIP>
__global__ __launch_bounds__(256) void k_instr_rows(const uint32_t *__restrict__ rec, uint64_t n, uint32_t repr,
                                                    uint32_t *__restrict__ out, uint64_t height, uint32_t width) {
    using namespace kb;
    const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= height) return;
    auto F = [&](uint32_t v) { return repr == ZKM_REPR_MONTGOMERY ? from_mont(v < P ? v : v - P) : (v < P ? v : v - P); };
    uint32_t *row = out + r * width;
    for (uint32_t c = 0; c < width; c++) row[c] = 0;
    constexpr uint32_t NEG1 = P - 1;
    if constexpr (CHIP == ZKM_REC_CHIP_BASE_ALU || CHIP == ZKM_REC_CHIP_EXT_ALU) {
        // alu_base.hpp / alu_ext.hpp instr_to_row: addrs, one-hot opcode, mult; four entries per row
        for (int e = 0; e < 4; e++) {
            const uint64_t i = 4 * r + e;
            if (i >= n) break;
            const uint32_t *q = rec + 5 * i;
            uint32_t *o = row + 8 * e;
            o[0] = F(q[0]); o[1] = F(q[1]); o[2] = F(q[2]);
            if (q[3] < 4) o[3 + q[3]] = 1;
            o[7] = F(q[4]);
        }
    } else if constexpr (CHIP == ZKM_REC_CHIP_BATCH_FRI) {  // batch_fri.hpp: is_real, is_end, the four addrs
        if (r < n) {
            const uint32_t *q = rec + 5 * r;
            row[0] = 1; row[1] = q[4] ? 1u : 0u;
            row[2] = F(q[0]); row[3] = F(q[1]); row[4] = F(q[2]); row[5] = F(q[3]);
        }
    } else if constexpr (CHIP == ZKM_REC_CHIP_SELECT) {  // select.hpp: is_real, addrs, mults
        if (r < n) {
            row[0] = 1;
            for (int c = 0; c < 7; c++) row[1 + c] = F(rec[7 * r + c]);
        }
    } else if constexpr (CHIP == ZKM_REC_CHIP_FRI_FOLD) {  // fri_fold.hpp (z, alpha, x read once per instruction)
        if (r < n) {
            const uint32_t *q = rec + 12 * r;
            const uint32_t first = q[11] ? 1u : 0u, nf = first ? NEG1 : 0u;
            row[0] = first;
            row[1] = F(q[0]); row[2] = nf;
            row[3] = F(q[1]); row[4] = nf;
            row[5] = F(q[2]); row[6] = nf;
            row[7] = F(q[3]); row[8] = NEG1;
            row[9] = F(q[4]); row[10] = NEG1;
            row[11] = F(q[5]); row[12] = NEG1;
            row[13] = F(q[6]); row[14] = NEG1;
            row[15] = F(q[7]); row[16] = F(q[8]);
            row[17] = F(q[9]); row[18] = F(q[10]);
            row[19] = 1;
        }
    } else if constexpr (CHIP == ZKM_REC_CHIP_PUBLIC_VALUES) {  // public_values.hpp: digest element r
        if (r < n) {
            row[r] = 1;
            row[8] = F(rec[r]);
            row[9] = NEG1;
        }
    } else if constexpr (CHIP == ZKM_REC_CHIP_MEMORY_VAR) {  // mem/variable.rs: (addr, mult) x 2
        for (int e = 0; e < 2; e++) {
            const uint64_t i = 2 * r + e;
            if (i >= n) break;
            row[2 * e] = F(rec[2 * i]);
            row[2 * e + 1] = F(rec[2 * i + 1]);
        }
    } else if constexpr (CHIP == ZKM_REC_CHIP_MEMORY_CONST) {  // mem/constant.rs: (value[4], addr, mult) x 2
        for (int e = 0; e < 2; e++) {
            const uint64_t i = 2 * r + e;
            if (i >= n) break;
            for (int c = 0; c < 6; c++) row[6 * e + c] = F(rec[6 * i + c]);
        }
    } else if constexpr (CHIP == ZKM_REC_CHIP_EXP_REVERSE_BITS) {  // exp_reverse_bits.hpp, row i of an event
        if (r < n) {
            const uint32_t *q = rec + 6 * r;
            const uint32_t i = q[4], L = q[5];
            const bool first = i == 0, last = i + 1 == L;
            row[0] = F(q[0]); row[1] = first ? NEG1 : 0u;
            row[2] = F(q[1]); row[3] = NEG1;
            row[4] = F(q[2]); row[5] = last ? F(q[3]) : 0u;
            row[6] = i; row[7] = first; row[8] = last; row[9] = 1;
        }
    } else {  // ZKM_REC_CHIP_POSEIDON2_WIDE: poseidon2_wide.hpp instr_to_row
        if (r < n) {
            const uint32_t *q = rec + 48 * r;
            for (int c = 0; c < 16; c++) {
                row[c] = F(q[c]);
                row[16 + 2 * c] = F(q[16 + c]);
                row[17 + 2 * c] = F(q[32 + c]);
            }
            row[48] = NEG1;
        }
    }
}

}  // namespace zkm::rtg

using namespace zkm::rtg;

extern "C" int zkm_recursion_instrs_to_trace(uint32_t chip, const uint32_t *instrs, uint64_t n, uint32_t repr,
                                             uint32_t *trace, uint64_t height, void *stream) {
    // (record words, entries per row, preprocessed width), indexed by ZKM_REC_CHIP_*
    static const uint32_t layout[10][3] = {{5, 4, 32}, {5, 4, 32}, {5, 1, 6},  {7, 1, 8},  {12, 1, 20},
                                           {1, 1, 10}, {2, 2, 4}, {6, 2, 12}, {6, 1, 10}, {48, 1, 49}};
    if (chip > ZKM_REC_CHIP_POSEIDON2_WIDE || !trace || (n && !instrs) || height < 16 || (height & (height - 1)) ||
        (repr != ZKM_REPR_CANONICAL && repr != ZKM_REPR_MONTGOMERY) || n > height * layout[chip][1] ||
        (chip == ZKM_REC_CHIP_PUBLIC_VALUES && n > 8)) {
        g_last_error = "zkm_recursion_instrs_to_trace: bad arguments (known chip, n instructions fitting height "
                       "rows, height a power of two >= 16, repr canonical or Montgomery)";
        return ZKM_ERR_ARG;
    }
    const dim3 g((uint32_t)((height + 255) / 256)), b(256);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t w = layout[chip][2];
    switch (chip) {
        case 0: hipLaunchKernelGGL(k_instr_rows<0>, g, b, 0, s, instrs, n, repr, trace, height, w); break;
        case 1: hipLaunchKernelGGL(k_instr_rows<1>, g, b, 0, s, instrs, n, repr, trace, height, w); break;
        case 2: hipLaunchKernelGGL(k_instr_rows<2>, g, b, 0, s, instrs, n, repr, trace, height, w); break;
        case 3: hipLaunchKernelGGL(k_instr_rows<3>, g, b, 0, s, instrs, n, repr, trace, height, w); break;
        case 4: hipLaunchKernelGGL(k_instr_rows<4>, g, b, 0, s, instrs, n, repr, trace, height, w); break;
        case 5: hipLaunchKernelGGL(k_instr_rows<5>, g, b, 0, s, instrs, n, repr, trace, height, w); break;
        case 6: hipLaunchKernelGGL(k_instr_rows<6>, g, b, 0, s, instrs, n, repr, trace, height, w); break;
        case 7: hipLaunchKernelGGL(k_instr_rows<7>, g, b, 0, s, instrs, n, repr, trace, height, w); break;
        case 8: hipLaunchKernelGGL(k_instr_rows<8>, g, b, 0, s, instrs, n, repr, trace, height, w); break;
        default: hipLaunchKernelGGL(k_instr_rows<9>, g, b, 0, s, instrs, n, repr, trace, height, w); break;
    }
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_recursion_instrs_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

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
