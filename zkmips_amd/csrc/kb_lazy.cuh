// Lazy-reduction building blocks for KoalaBear on gfx950 (host + device): 64-bit multiply-add
// chains with one Montgomery reduction per chain, and split-constant accumulators.  Used by the
// Poseidon2 permutation (p2.cuh), the openings / FRI kernels and the JIT quotient kernels (this
// file is embedded in the hiprtc prelude).
//
// Device code pins the instruction selection with inline asm: one v_mad_u64_u32 per product-sum
// (left alone the compiler splits a*b + c into v_mul_lo + v_mul_hi + adds).  Reductions are
// kb::redc2 (kb31.cuh): t < P 2^32 -> [0, 2P) in 4 issue slots.
#pragma once
#include "kb31.cuh"

namespace kb {

#ifdef __HIP_DEVICE_COMPILE__
__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {  // c in VGPRs
    uint64_t t, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(t), "=s"(cc) : "v"(a), "v"(b), "v"(c));
    return t;
}
__device__ __forceinline__ uint64_t prod64_ks(uint32_t a, uint32_t k) {  // a k, k uniform (SGPR)
    uint64_t t, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(t), "=s"(cc) : "v"(a), "s"(k));
    return t;
}
__device__ __forceinline__ uint64_t mad64_ks(uint32_t a, uint32_t k, uint64_t c) {  // k uniform (SGPR)
    uint64_t t, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(t), "=s"(cc) : "v"(a), "s"(k), "v"(c));
    return t;
}
// c + a and c + 2a for 64-bit c: a v_mad_u64_u32 with an inline-constant multiplier takes the
// 32-bit operand as is (v_lshl_add_u64 would first need a zeroed high word, one more v_mov)
__device__ __forceinline__ uint64_t add_w(uint64_t c, uint32_t a) {
    uint64_t t, cc;
    asm("v_mad_u64_u32 %0, %1, %2, 1, %3" : "=v"(t), "=s"(cc) : "v"(a), "v"(c));
    return t;
}
__device__ __forceinline__ uint64_t add_w2(uint64_t c, uint32_t a) {
    uint64_t t, cc;
    asm("v_mad_u64_u32 %0, %1, %2, 2, %3" : "=v"(t), "=s"(cc) : "v"(a), "v"(c));
    return t;
}
// Per-use scalar constants.  In a loop around the permutation (sponge, PoW) the compiler hoists
// the ~300 distinct round/injection constants into SGPRs, runs out, and spills them to VGPR lanes
// (a v_readlane per use).  A volatile s_mov at the point of use keeps them as immediates.
__device__ __forceinline__ uint32_t kc32(uint32_t k) {
    uint32_t r;
    asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "i"(k));
    return r;
}
__device__ __forceinline__ uint64_t kc64(uint64_t k) {
    uint32_t lo, hi;
    asm volatile("s_mov_b32 %0, %2\n\ts_mov_b32 %1, %3" : "=s"(lo), "=s"(hi) : "i"((uint32_t)k), "i"((uint32_t)(k >> 32)));
    return ((uint64_t)hi << 32) | lo;
}
#else
KB_HD uint32_t kc32(uint32_t k) { return k; }
KB_HD uint64_t kc64(uint64_t k) { return k; }
KB_HD uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }
KB_HD uint64_t mad64_ks(uint32_t a, uint32_t k, uint64_t c) { return (uint64_t)a * k + c; }
KB_HD uint64_t prod64_ks(uint32_t a, uint32_t k) { return (uint64_t)a * k; }
KB_HD uint64_t add_w(uint64_t c, uint32_t a) { return c + a; }
KB_HD uint64_t add_w2(uint64_t c, uint32_t a) { return c + 2 * (uint64_t)a; }
#endif
#ifdef __HIP_DEVICE_COMPILE__
__device__ __forceinline__ uint64_t mad64_add(uint32_t a, uint32_t b, uint64_t k) {  // a b + k, k uniform
    uint64_t t, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(t), "=s"(cc) : "v"(a), "v"(b), "s"(k));
    return t;
}
#else
KB_HD uint64_t mad64_add(uint32_t a, uint32_t b, uint64_t k) { return (uint64_t)a * b + k; }
#endif
constexpr uint32_t MONT_2_16 = (uint32_t)(((uint64_t)1 << 48) % P);  // 2^16 in Montgomery form

// sum of lazy terms (< P 2^32) -> canonical Montgomery value: redc(acc) R^2 / R = acc mod p
KB_HD uint32_t acc_mod(uint64_t acc) { return mul(redc(acc), R2); }

// Accumulator of x_k * u_k (x per thread, u a uniform EF constant) with the constant split into
// 16-bit halves: products < 2^47, so up to 2^16 terms accumulate in 64 bits with no reduction.
// value() = sum x_k u_k / R (the Montgomery product sum).
struct EfAcc {
    uint64_t lo[4], hi[4];
    KB_HD void zero() {
        for (int e = 0; e < 4; e++) { lo[e] = 0; hi[e] = 0; }
    }
    KB_HD void term(uint32_t x, uint32_t u, int e) {
        lo[e] = mad64_ks(x, u & 0xffffu, lo[e]);
        hi[e] = mad64_ks(x, u >> 16, hi[e]);
    }
    // += x * u  (x base field)
    KB_HD void base(uint32_t x, const uint32_t *u) {
        for (int e = 0; e < 4; e++) term(x, u[e], e);
    }
    // += x * u  (x extension field, u uniform): X^4 = 3, the wrap terms use 3 u_g
    KB_HD void ext(const ef &x, const uint32_t *u) {
        uint32_t u3[4];
        for (int g = 1; g < 4; g++) u3[g] = add(dbl(u[g]), u[g]);
        for (int f = 0; f < 4; f++)
            for (int g = 0; g < 4; g++) {
                const int e = f + g;
                if (e < 4) term(x.c[f], u[g], e);
                else term(x.c[f], u3[g], e - 4);
            }
    }
    KB_HD ef value() const {
        ef r;
        for (int e = 0; e < 4; e++) r.c[e] = add(redc(lo[e]), mul(redc(hi[e]), MONT_2_16));
        return r;
    }
};

// base + x0 u0 + x1 u1 (EF, u uniform): one product pair per component and one lazy reduction
KB_HD ef ef_dot2(const ef &base, uint32_t x0, const uint32_t *u0, uint32_t x1, const uint32_t *u1) {
    ef r;
    for (int e = 0; e < 4; e++) {
        const uint32_t t = redc2(mad64_ks(x0, u0[e], prod64_ks(x1, u1[e])));  // x0 u0 + x1 u1 < 2P^2 -> [0, 2P)
        r.c[e] = add(base.c[e], umin(t, t - P));
    }
    return r;
}

}  // namespace kb
