/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into or called by the
 * product path (zkmips_amd/, include/).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker.
 *
 * KoalaBear field F_p, p = 2^31 - 2^24 + 1, and its binomial extension
 * EF = F[X]/(X^4 - 3), restated in CANONICAL representation (plain residues
 * in [0,p)), independently of the product's Montgomery code.
 *
 * Reference anchors:
 *   - p, Montgomery constants: crates/core/machine/include/kb31_t.hpp:460-475
 *   - EF = F[X]/(X^4 - W), W = 3: crates/recursion/gnark-ffi/go/zkm/koalabear/koalabear.go:247-268
 *   - two-adic generators = powers of 3^127 (Plonky3 KoalaBear)
 */
#pragma once
#include <stdint.h>
#include <string.h>

#define KB_P 0x7f000001u
#define KB_TWO_ADICITY 24
#define KB_GENERATOR 3u
#define KB_W 3u

typedef uint32_t kb_t;
typedef struct { kb_t c[4]; } ef_t;

static inline kb_t kb_add(kb_t a, kb_t b) { uint32_t s = a + b; return s >= KB_P ? s - KB_P : s; }
static inline kb_t kb_sub(kb_t a, kb_t b) { return a >= b ? a - b : a + KB_P - b; }
static inline kb_t kb_neg(kb_t a) { return a ? KB_P - a : 0; }
static inline kb_t kb_mul(kb_t a, kb_t b) { return (kb_t)(((uint64_t)a * b) % KB_P); }
static inline kb_t kb_from_u64(uint64_t x) { return (kb_t)(x % KB_P); }

static inline kb_t kb_pow(kb_t a, uint64_t e) {
    kb_t r = 1;
    while (e) { if (e & 1) r = kb_mul(r, a); a = kb_mul(a, a); e >>= 1; }
    return r;
}
static inline kb_t kb_inv(kb_t a) { return kb_pow(a, KB_P - 2); }
static inline kb_t kb_halve(kb_t a) { return (a & 1) ? (kb_t)(((uint64_t)a + KB_P) >> 1) : a >> 1; }

/* primitive 2^bits-th root of unity: 3^((p-1)/2^bits) */
static inline kb_t kb_two_adic_gen(int bits) {
    return kb_pow(KB_GENERATOR, (uint64_t)(KB_P - 1) >> bits);
}

static inline ef_t ef_zero(void) { ef_t r; memset(&r, 0, sizeof r); return r; }
static inline ef_t ef_one(void) { ef_t r = ef_zero(); r.c[0] = 1; return r; }
static inline ef_t ef_from_base(kb_t a) { ef_t r = ef_zero(); r.c[0] = a; return r; }
static inline int ef_eq(ef_t a, ef_t b) { return !memcmp(&a, &b, sizeof a); }
static inline int ef_is_zero(ef_t a) { return !(a.c[0] | a.c[1] | a.c[2] | a.c[3]); }
static inline ef_t ef_add(ef_t a, ef_t b) { for (int i = 0; i < 4; i++) a.c[i] = kb_add(a.c[i], b.c[i]); return a; }
static inline ef_t ef_sub(ef_t a, ef_t b) { for (int i = 0; i < 4; i++) a.c[i] = kb_sub(a.c[i], b.c[i]); return a; }
static inline ef_t ef_neg(ef_t a) { for (int i = 0; i < 4; i++) a.c[i] = kb_neg(a.c[i]); return a; }
static inline ef_t ef_add_base(ef_t a, kb_t b) { a.c[0] = kb_add(a.c[0], b); return a; }
static inline ef_t ef_mul_base(ef_t a, kb_t b) { for (int i = 0; i < 4; i++) a.c[i] = kb_mul(a.c[i], b); return a; }

static inline ef_t ef_mul(ef_t a, ef_t b) {
    /* schoolbook product folded with X^4 = W; products < 2^62, so up to four share one reduction */
    const uint64_t a0 = a.c[0], a1 = a.c[1], a2 = a.c[2], a3 = a.c[3];
    const uint64_t b0 = b.c[0], b1 = b.c[1], b2 = b.c[2], b3 = b.c[3];
    const uint64_t h0 = (a1 * b3 + a2 * b2 + a3 * b1) % KB_P, h1 = (a2 * b3 + a3 * b2) % KB_P, h2 = (a3 * b3) % KB_P;
    ef_t r;
    r.c[0] = (kb_t)((a0 * b0 + KB_W * h0) % KB_P);
    r.c[1] = (kb_t)((a0 * b1 + a1 * b0 + KB_W * h1) % KB_P);
    r.c[2] = (kb_t)((a0 * b2 + a1 * b1 + a2 * b0 + KB_W * h2) % KB_P);
    r.c[3] = (kb_t)((a0 * b3 + a1 * b2 + a2 * b1 + a3 * b0) % KB_P);
    return r;
}
static inline ef_t ef_square(ef_t a) { return ef_mul(a, a); }
static inline ef_t ef_pow(ef_t a, uint64_t e) {
    ef_t r = ef_one();
    while (e) { if (e & 1) r = ef_mul(r, a); a = ef_mul(a, a); e >>= 1; }
    return r;
}

/* inverse via a^(p^4-2) computed as norm trick: a^{-1} = a^{r-1} / N(a),
 * r = 1 + p + p^2 + p^3.  Frobenius on F[X]/(X^4-W): X^p = W^((p-1)/4) X. */
static inline ef_t ef_frobenius(ef_t a) {
    /* X^{p} = z X with z = W^((p-1)/4) */
    static kb_t z;
    if (!z) z = kb_pow(KB_W, (KB_P - 1) / 4);
    ef_t r;
    kb_t zi = 1;
    for (int i = 0; i < 4; i++) { r.c[i] = kb_mul(a.c[i], zi); zi = kb_mul(zi, z); }
    return r;
}
static inline ef_t ef_inv(ef_t a) {
    ef_t f1 = ef_frobenius(a);
    ef_t f2 = ef_frobenius(f1);
    ef_t f3 = ef_frobenius(f2);
    ef_t t = ef_mul(ef_mul(f1, f2), f3); /* a^{p+p^2+p^3} */
    ef_t n = ef_mul(a, t);               /* norm, lies in F */
    kb_t ninv = kb_inv(n.c[0]);
    return ef_mul_base(t, ninv);
}
static inline ef_t ef_div(ef_t a, ef_t b) { return ef_mul(a, ef_inv(b)); }

/* reverse the low `bits` bits of x (x < 2^bits) */
static inline uint32_t rev_bits(uint32_t x, int bits) {
    x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
    x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
    x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
    x = __builtin_bswap32(x);
    return bits ? x >> (32 - bits) : 0;
}
static inline int log2_exact(uint64_t n) { int l = 0; while ((1ull << l) < n) l++; return l; }
