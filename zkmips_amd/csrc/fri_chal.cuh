// One FRI round of the device Fiat-Shamir transcript (DuplexChallenger semantics of the host
// Challenger, crates/recursion/circuit/src/challenger.rs:60-233: observe the round commitment's 8 words,
// sample beta as 4 words), run by a whole workgroup: wave 0 computes the permutations in the 16-lane form
// (its four rows alike), every thread takes the barriers.  Records the root for the proof and the fold
// arguments (beta / 2, beta^2).  Used by k_fri_chal and, fused, by the subtree launch that finishes a
// FRI round's tree (one launch fewer per round).
#pragma once
#include "open_kernels.hpp"
#include "p2.cuh"

namespace zkm {

struct ChalShared {
    uint32_t st[16], in[8], out[8];
    int nin, nout;
};

// root: the round commitment (8 words, global or LDS)
__device__ __forceinline__ void fri_chal_block(ChalShared &sh, DevChallenger *c, const uint32_t *root,
                                               uint32_t *root_out, uint32_t *fargs) {
    using namespace kb;
    const int tid = threadIdx.x, l = tid & 15;
    if (tid < 16) sh.st[tid] = c->st[tid];
    if (tid < 8) { sh.in[tid] = c->in[tid]; sh.out[tid] = c->out[tid]; root_out[tid] = root[tid]; }
    if (tid == 0) { sh.nin = (int)c->nin; sh.nout = (int)c->nout; }
    __syncthreads();
    const p2x16::Lane lc = p2x16::lane_consts(l);
    auto duplex = [&]() {
        uint32_t x = 0;
        if (tid < 64) x = p2x16::permute(l < sh.nin ? sh.in[l] : sh.st[l], lc);
        __syncthreads();
        if (tid < 16) sh.st[tid] = x;
        if (tid < 8) sh.out[tid] = x;
        if (tid == 0) { sh.nin = 0; sh.nout = 8; }
        __syncthreads();
    };
    for (int k = 0; k < 8; k++) {  // observe(root[k])
        if (tid == 0) { sh.nout = 0; sh.in[sh.nin] = root[k]; sh.nin++; }
        __syncthreads();
        if (sh.nin == 8) duplex();
    }
    uint32_t beta[4];
    for (int k = 0; k < 4; k++) {  // sample()
        if (sh.nin || !sh.nout) duplex();
        beta[k] = sh.out[sh.nout - 1];
        __syncthreads();
        if (tid == 0) sh.nout--;
        __syncthreads();
    }
    if (tid == 0) {
        const ef b{{beta[0], beta[1], beta[2], beta[3]}};
        const ef hb = ef_mul_base(b, halve(ONE)), b2 = ef_mul(b, b);
        for (int e = 0; e < 4; e++) { fargs[e] = hb.c[e]; fargs[4 + e] = b2.c[e]; }
    }
    if (tid < 16) c->st[tid] = sh.st[tid];
    if (tid < 8) { c->in[tid] = sh.in[tid]; c->out[tid] = sh.out[tid]; }
    if (tid == 0) { c->nin = (uint32_t)sh.nin; c->nout = (uint32_t)sh.nout; }
}

}  // namespace zkm
