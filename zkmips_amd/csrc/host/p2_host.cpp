// Host Poseidon2-16 over many states for the recursion runtime's witness generation (the Poseidon2
// instructions of a compress program: recursion/core/src/runtime/mod.rs Poseidon2 opcode).  The same
// permutation code as the GPU kernels (p2.cuh, host instantiation; checked against the oracle by
// tools/check/p2_host_check.cpp / tests/test_host.py), canonical words in and out; sixteen states at a time
// in AVX-512 lanes where the CPU has them (p2_simd.cpp).  Single-threaded: the callers are witness-generation
// worker processes, one per core.
#include <cstddef>
#include <cstdint>

#include "../p2.cuh"

namespace zkm_host {
uint64_t p2_simd_permute(const uint32_t *in, size_t in_stride, uint32_t *out, size_t out_stride, uint64_t n);
}

extern "C" void zkm_host_poseidon2_permute(const uint32_t *in, uint32_t *out, uint64_t n) {
    for (int64_t i = (int64_t)zkm_host::p2_simd_permute(in, 16, out, 16, n); i < (int64_t)n; i++) {
        uint32_t st[16];
        for (int j = 0; j < 16; j++) st[j] = kb::to_mont(in[16 * i + j] % kb::P);
        p2::permute(st);
        for (int j = 0; j < 16; j++) out[16 * i + j] = kb::from_mont(st[j]);
    }
}
