// KoalaBear field (p = 2^31 - 2^24 + 1) and its quartic extension EF = F[X]/(X^4 - 3),
// Montgomery form with R = 2^32, for host and gfx950 device code.
//
// Reference anchors: crates/core/machine/include/kb31_t.hpp:458-475 (MOD, MONTY_MU, RR),
// EF binomial W = 3 (crates/recursion/gnark-ffi/go/zkm/koalabear/koalabear.go:247-268).
//
// Every value held in device memory by this library is in Montgomery form; the C ABI converts
// at the boundary (canonical or Montgomery input, canonical proof bytes by default).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define KB_HD __host__ __device__ __forceinline__

namespace kb {

constexpr uint32_t P = 0x7f000001u;
constexpr uint32_t MU = 0x81000001u;       // P^{-1} mod 2^32
constexpr uint32_t R2 = 0x17f7efe4u;       // 2^64 mod P
constexpr uint32_t ONE = 0x01fffffeu;      // 2^32 mod P  (Montgomery 1)
constexpr uint32_t GENERATOR = 3u;
constexpr int TWO_ADICITY = 24;

KB_HD uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
// a + b < 2P < 2^32: s - P wraps above s exactly when s < P
KB_HD uint32_t add(uint32_t a, uint32_t b) {
    uint32_t s = a + b;
    return umin(s, s - P);
}
// a - b wraps exactly when a < b; adding P then lands in [0, P) below the wrapped value
KB_HD uint32_t sub(uint32_t a, uint32_t b) {
    uint32_t d = a - b;
    return umin(d, d + P);
}
KB_HD uint32_t neg(uint32_t a) { return a ? P - a : 0u; }
KB_HD uint32_t dbl(uint32_t a) { return add(a, a); }

KB_HD uint32_t umulhi(uint32_t a, uint32_t b) {
#ifdef __HIP_DEVICE_COMPILE__
    return __umulhi(a, b);
#else
    return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}

// Montgomery reduction with m = -t_lo P^-1: t + m P is a multiple of 2^32 and, for t < P 2^32,
// (t + m P) / 2^32 lies in [0, 2P).  On gfx950 that is one v_mul_lo_u32 and one v_mad_u64_u32
// (the quotient is the high word of the mad), so a reduction costs 4 issue slots, and the lazy
// result needs no offset to stay non-negative.
constexpr uint32_t MUN = 0x7effffffu;  // -P^{-1} mod 2^32
#ifdef __HIP_DEVICE_COMPILE__
__device__ __forceinline__ uint32_t redc2(uint64_t t) {  // t < P 2^32 -> [0, 2P)
    const uint32_t m = (uint32_t)t * MUN;
    uint64_t u, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(u), "=s"(cc) : "v"(m), "s"(P), "v"(t));
    return (uint32_t)(u >> 32);
}
__device__ __forceinline__ uint64_t prod64(uint32_t a, uint32_t b) {  // one v_mad_u64_u32 (addend 0)
    uint64_t u, cc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(u), "=s"(cc) : "v"(a), "v"(b));
    return u;
}
#else
KB_HD uint32_t redc2(uint64_t t) {
    const uint32_t m = (uint32_t)t * MUN;
    return (uint32_t)((t + (uint64_t)m * P) >> 32);
}
KB_HD uint64_t prod64(uint32_t a, uint32_t b) { return (uint64_t)a * b; }
#endif
KB_HD uint32_t redc(uint64_t t) {  // t < P 2^32 -> [0, P)
    const uint32_t r = redc2(t);
    return umin(r, r - P);
}
KB_HD uint32_t mul(uint32_t a, uint32_t b) { return redc(prod64(a, b)); }
// a * b / R in [0, 2P), unreduced, for a * b < P * 2^32
KB_HD uint32_t mul_lazy(uint32_t a, uint32_t b) { return redc2(prod64(a, b)); }
KB_HD uint32_t sqr(uint32_t a) { return mul(a, a); }
KB_HD uint32_t to_mont(uint32_t x) { return mul(x % P, R2); }
KB_HD uint32_t from_mont(uint32_t x) { return redc((uint64_t)x); }
// a^2 stays lazy in (0, 2P): (2P) * a < P * 2^32 keeps the second reduction exact
KB_HD uint32_t cube(uint32_t a) { return mul(mul_lazy(a, a), a); }

KB_HD uint32_t pow(uint32_t a, uint64_t e) {
    uint32_t r = ONE;
    while (e) {
        if (e & 1) r = mul(r, a);
        a = sqr(a);
        e >>= 1;
    }
    return r;
}
KB_HD uint32_t inv(uint32_t a) { return pow(a, P - 2); }
KB_HD uint32_t halve(uint32_t a) { return (a & 1) ? (uint32_t)(((uint64_t)a + P) >> 1) : (a >> 1); }

// primitive 2^bits-th root of unity (Montgomery): GENERATOR^((p-1)/2^bits)
inline uint32_t two_adic_gen(int bits) { return pow(to_mont(GENERATOR), (uint64_t)(P - 1) >> bits); }

KB_HD uint32_t rev_bits(uint32_t x, int bits) {
#ifdef __HIP_DEVICE_COMPILE__
    return bits ? (__brev(x) >> (32 - bits)) : 0u;
#else
    uint32_t r = 0;
    for (int i = 0; i < bits; i++) { r = (r << 1) | (x & 1u); x >>= 1; }
    return r;
#endif
}

// ------------------------------------------------------------------ extension field
struct ef {
    uint32_t c[4];
};

KB_HD ef ef_zero() { return ef{{0u, 0u, 0u, 0u}}; }
KB_HD ef ef_one() { return ef{{ONE, 0u, 0u, 0u}}; }
KB_HD ef ef_base(uint32_t a) { return ef{{a, 0u, 0u, 0u}}; }
KB_HD ef ef_add(const ef &a, const ef &b) {
    return ef{{add(a.c[0], b.c[0]), add(a.c[1], b.c[1]), add(a.c[2], b.c[2]), add(a.c[3], b.c[3])}};
}
KB_HD ef ef_sub(const ef &a, const ef &b) {
    return ef{{sub(a.c[0], b.c[0]), sub(a.c[1], b.c[1]), sub(a.c[2], b.c[2]), sub(a.c[3], b.c[3])}};
}
KB_HD ef ef_neg(const ef &a) { return ef{{neg(a.c[0]), neg(a.c[1]), neg(a.c[2]), neg(a.c[3])}}; }
KB_HD ef ef_add_base(ef a, uint32_t b) { a.c[0] = add(a.c[0], b); return a; }
KB_HD ef ef_mul_base(const ef &a, uint32_t b) {
    return ef{{mul(a.c[0], b), mul(a.c[1], b), mul(a.c[2], b), mul(a.c[3], b)}};
}
KB_HD bool ef_eq(const ef &a, const ef &b) {
    return a.c[0] == b.c[0] && a.c[1] == b.c[1] && a.c[2] == b.c[2] && a.c[3] == b.c[3];
}
KB_HD bool ef_is_zero(const ef &a) { return (a.c[0] | a.c[1] | a.c[2] | a.c[3]) == 0u; }

// (a0 + a1 X + a2 X^2 + a3 X^3)(b0 + ...) mod X^4 - 3.
// With 3 b1, 3 b2, 3 b3 reduced first, every coefficient is four products, summed in two pairs
// (each pair < 2 p^2 < P * 2^32) with one Montgomery reduction per pair: 8 reductions and 10 additions.
KB_HD ef ef_mul(const ef &a, const ef &b) {
    const uint64_t a0 = a.c[0], a1 = a.c[1], a2 = a.c[2], a3 = a.c[3];
    const uint64_t b0 = b.c[0], b1 = b.c[1], b2 = b.c[2], b3 = b.c[3];
    const uint64_t t1 = add(dbl(b.c[1]), b.c[1]), t2 = add(dbl(b.c[2]), b.c[2]), t3 = add(dbl(b.c[3]), b.c[3]);
    // c0 = a0b0 + 3(a1b3 + a2b2 + a3b1)
    const uint32_t c0 = add(redc(a0 * b0 + a1 * t3), redc(a2 * t2 + a3 * t1));
    // c1 = a0b1 + a1b0 + 3(a2b3 + a3b2)
    const uint32_t c1 = add(redc(a0 * b1 + a1 * b0), redc(a2 * t3 + a3 * t2));
    // c2 = a0b2 + a1b1 + a2b0 + 3 a3b3
    const uint32_t c2 = add(redc(a0 * b2 + a1 * b1), redc(a2 * b0 + a3 * t3));
    // c3 = a0b3 + a1b2 + a2b1 + a3b0
    const uint32_t c3 = add(redc(a0 * b3 + a1 * b2), redc(a2 * b1 + a3 * b0));
    return ef{{c0, c1, c2, c3}};
}
KB_HD ef ef_sqr(const ef &a) { return ef_mul(a, a); }

KB_HD ef ef_pow(ef a, uint64_t e) {
    ef r = ef_one();
    while (e) {
        if (e & 1) r = ef_mul(r, a);
        a = ef_sqr(a);
        e >>= 1;
    }
    return r;
}

// Frobenius x -> x^p on F[X]/(X^4 - 3): X^p = z X with z = 3^((p-1)/4) = 0x7e010002 (a 4th root of 1).
constexpr uint32_t FROB_Z = 0x7b020407u;  // Montgomery form of 0x7e010002
KB_HD ef ef_frobenius(const ef &a) {
    const uint32_t z = FROB_Z;
    uint32_t z2 = mul(z, z), z3 = mul(z2, z);
    return ef{{a.c[0], mul(a.c[1], z), mul(a.c[2], z2), mul(a.c[3], z3)}};
}
// a^{-1} = a^{p + p^2 + p^3} / N(a)
KB_HD ef ef_inv(const ef &a) {
    ef f1 = ef_frobenius(a);
    ef f2 = ef_frobenius(f1);
    ef f3 = ef_frobenius(f2);
    ef t = ef_mul(ef_mul(f1, f2), f3);
    ef n = ef_mul(a, t);
    return ef_mul_base(t, inv(n.c[0]));
}

}  // namespace kb
