// One Poseidon2-16 permutation row in the PermutationSBox column layout (recursion/core/src/chips/
// poseidon2_wide/columns/permutation.rs:20-72; include/poseidon2_wide.hpp populate_perm): external round
// states [8][16], internal state [16], s0 [12], output [16], external s-box cubes [8][16], internal s-box
// cubes [13] -- 313 canonical words.  The same columns open the MIPS Poseidon2Permute chip's row
// (core/machine/src/syscall/precompiles/poseidon2/columns.rs: Poseidon2Degree3Cols first).
//
// Computed by the 16 lanes of one 16-lane DPP row of a wavefront (p2.cuh's p2x16 form: lane l holds state
// word l, the linear layers as DPP adds): each lane writes its own words of every round state and external
// s-box, lane 0 the internal s-boxes and s0 columns, into `my` (the row's first column, typically LDS).
#pragma once
#include "kb31.cuh"
#include "p2.cuh"

namespace zkm::p2rows {

constexpr int W = 16, NE = 8, NI = 13;
constexpr int C_EXT = 0, C_INT = C_EXT + NE * W, C_S0 = C_INT + W, C_OUT = C_S0 + NI - 1, C_ESB = C_OUT + W,
              C_ISB = C_ESB + NE * W, COLS = C_ISB + NI;

// x: state word l in Montgomery form (< P); returns output word l in Montgomery form
__device__ __forceinline__ uint32_t fill(uint32_t x, uint32_t l, uint32_t *my) {
    using namespace kb;
    const p2x16::Lane c = p2x16::lane_consts((int)l);
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
    return x;
}

}  // namespace zkm::p2rows
