// Host Poseidon2-16 over KoalaBear, sixteen permutations at a time in AVX-512 lanes, for the compress nodes'
// witness generation (the recursion runtime's Poseidon2 instructions, rec_exec.cpp; the batch helper of
// p2_host.cpp).  Structure of arrays: vector j holds element j of sixteen states, so every round is lane-wise
// and needs no shuffles.  The permutation is the reference's poseidon2_init configuration as p2.cuh restates
// it (crates/primitives/src/lib.rs:1107-1122: initial external layer, 4 full rounds, 13 partial rounds on
// element 0, 4 full rounds, S-box x^3; M4 blocks + column sums, internal diagonal of air.rs:12-29), in plain
// Montgomery arithmetic: every value canonical in [0, P) between operations.  Selected at run time (the CPU's
// AVX-512F flag); without it the callers keep the one-state code.  Checked against the oracle's permutation in
// tests/test_host.py.
#include <immintrin.h>

#include <cstddef>
#include <cstdint>

namespace {
constexpr uint32_t P = 0x7f000001u;

#include "../p2_rc.inc"

constexpr uint64_t pw(uint64_t a, uint64_t e) {
    uint64_t r = 1;
    for (a %= P; e; e >>= 1, a = a * a % P)
        if (e & 1) r = r * a % P;
    return r;
}
constexpr uint32_t inv(uint64_t a) { return (uint32_t)pw(a, P - 2); }
constexpr uint32_t neg(uint32_t x) { return x ? P - x : 0; }
constexpr uint32_t mont(uint64_t x) { return (uint32_t)(((x % P) << 32) % P); }
constexpr uint32_t mu() {  // P^-1 mod 2^32 (Newton)
    uint32_t x = 1;
    for (int i = 0; i < 5; i++) x *= 2u - P * x;
    return x;
}

struct Consts {
    uint32_t ext[8][16];  // full rounds (Montgomery)
    uint32_t inr[13];     // partial rounds, element 0
    uint32_t diag[16];    // internal diagonal V (Montgomery)
};
constexpr Consts make() {
    Consts c{};
    for (int r = 0; r < 4; r++)
        for (int i = 0; i < 16; i++) {
            c.ext[r][i] = mont(kP2RoundConstCanon[r][i]);
            c.ext[r + 4][i] = mont(kP2RoundConstCanon[r + 17][i]);
        }
    for (int r = 0; r < 13; r++) c.inr[r] = mont(kP2RoundConstCanon[4 + r][0]);
    const uint32_t v[16] = {neg(2), 1, 2, inv(2), 3, 4, neg(inv(2)), neg(3), neg(4), inv(1u << 8), inv(8),
                            inv(1u << 24), neg(inv(1u << 8)), neg(inv(8)), neg(inv(16)), neg(inv(1u << 24))};
    for (int i = 0; i < 16; i++) c.diag[i] = mont(v[i]);
    return c;
}
constexpr Consts C = make();
constexpr uint32_t MU = mu();
constexpr uint32_t R2 = (uint32_t)pw(2, 64);  // mont(x, R2) = x R

#define AVX512 __attribute__((target("avx512f")))

// a b / 2^32 mod P for a b < 2^32 P: (a b - q P) / 2^32 in (-P, P), q = a b P^-1 mod 2^32
AVX512 inline __m512i mmul(__m512i a, __m512i b) {
    const __m512i p = _mm512_set1_epi32((int)P), m = _mm512_set1_epi32((int)MU);
    const __m512i pe = _mm512_mul_epu32(a, b);
    const __m512i po = _mm512_mul_epu32(_mm512_srli_epi64(a, 32), _mm512_srli_epi64(b, 32));
    const __m512i de = _mm512_sub_epi64(pe, _mm512_mul_epu32(_mm512_mul_epu32(pe, m), p));
    const __m512i dd = _mm512_sub_epi64(po, _mm512_mul_epu32(_mm512_mul_epu32(po, m), p));
    const __m512i r = _mm512_mask_blend_epi32((__mmask16)0xAAAA, _mm512_srli_epi64(de, 32), dd);
    return _mm512_min_epu32(r, _mm512_add_epi32(r, p));  // (-P, 0) wrapped -> + P
}
AVX512 inline __m512i madd(__m512i a, __m512i b) {  // a, b < P
    const __m512i s = _mm512_add_epi32(a, b);
    return _mm512_min_epu32(s, _mm512_sub_epi32(s, _mm512_set1_epi32((int)P)));
}
AVX512 inline __m512i cube(__m512i x) { return mmul(mmul(x, x), x); }

AVX512 inline void external(__m512i s[16]) {
    for (int j = 0; j < 16; j += 4) {  // M4 = [[2,3,1,1],[1,2,3,1],[1,1,2,3],[3,1,1,2]]
        const __m512i t01 = madd(s[j], s[j + 1]), t23 = madd(s[j + 2], s[j + 3]);
        const __m512i t0123 = madd(t01, t23);
        const __m512i t01123 = madd(t0123, s[j + 1]), t01233 = madd(t0123, s[j + 3]);
        const __m512i y0 = s[j], y2 = s[j + 2];
        s[j] = madd(t01123, t01);
        s[j + 1] = madd(t01123, madd(y2, y2));
        s[j + 2] = madd(t01233, t23);
        s[j + 3] = madd(t01233, madd(y0, y0));
    }
    __m512i sum[4];
    for (int k = 0; k < 4; k++) sum[k] = madd(madd(s[k], s[4 + k]), madd(s[8 + k], s[12 + k]));
    for (int j = 0; j < 16; j++) s[j] = madd(s[j], sum[j & 3]);
}

AVX512 inline void full_round(__m512i s[16], const uint32_t rc[16]) {
    for (int j = 0; j < 16; j++) s[j] = cube(madd(s[j], _mm512_set1_epi32((int)rc[j])));
    external(s);
}

AVX512 void permute16(__m512i s[16]) {
    external(s);
    for (int r = 0; r < 4; r++) full_round(s, C.ext[r]);
    for (int r = 0; r < 13; r++) {
        s[0] = cube(madd(s[0], _mm512_set1_epi32((int)C.inr[r])));
        __m512i a = madd(s[0], s[1]), b = madd(s[2], s[3]);
        for (int j = 4; j < 16; j += 2) {
            a = madd(a, s[j]);
            b = madd(b, s[j + 1]);
        }
        const __m512i sum = madd(a, b);
        for (int j = 0; j < 16; j++) s[j] = madd(mmul(s[j], _mm512_set1_epi32((int)C.diag[j])), sum);
    }
    for (int r = 4; r < 8; r++) full_round(s, C.ext[r]);
}

AVX512 uint64_t run(const uint32_t *in, size_t in_stride, uint32_t *out, size_t out_stride, uint64_t n) {
    const __m512i lane = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    const __m512i ii = _mm512_mullo_epi32(lane, _mm512_set1_epi32((int)in_stride));
    const __m512i oi = _mm512_mullo_epi32(lane, _mm512_set1_epi32((int)out_stride));
    const __m512i r2 = _mm512_set1_epi32((int)R2), one = _mm512_set1_epi32(1);
    const uint64_t full = n & ~(uint64_t)15;
    for (uint64_t b = 0; b < full; b += 16) {
        __m512i s[16];
        const int *src = (const int *)(in + b * in_stride);
        for (int j = 0; j < 16; j++) s[j] = mmul(_mm512_i32gather_epi32(_mm512_add_epi32(ii, _mm512_set1_epi32(j)), src, 4), r2);
        permute16(s);
        int *dst = (int *)(out + b * out_stride);
        for (int j = 0; j < 16; j++) _mm512_i32scatter_epi32(dst, _mm512_add_epi32(oi, _mm512_set1_epi32(j)), mmul(s[j], one), 4);
    }
    if (n - full < 4) return full;  // (fewer than 4: the one-state code is faster than a padded batch)
    if (full < n) {  // the last n % 16 states through a padded batch
        alignas(64) uint32_t t[16][16] = {};
        const uint64_t k = n - full;
        for (uint64_t i = 0; i < k; i++)
            for (int j = 0; j < 16; j++) t[j][i] = in[(full + i) * in_stride + j];
        __m512i s[16];
        for (int j = 0; j < 16; j++) s[j] = mmul(_mm512_load_si512((const void *)t[j]), r2);
        permute16(s);
        for (int j = 0; j < 16; j++) _mm512_store_si512((void *)t[j], mmul(s[j], one));
        for (uint64_t i = 0; i < k; i++)
            for (int j = 0; j < 16; j++) out[(full + i) * out_stride + j] = t[j][i];
    }
    return n;
}
}  // namespace

namespace zkm_host {
// Permutes the first states of n (state i: 16 canonical words at in + i in_stride, written to out + i
// out_stride; in and out may be the same states; a last n % 16 >= 4 in one padded batch) and returns how many
// it did, 0 without AVX-512F: the caller's one-state code does the rest.  Strides below 2^27 words.
uint64_t p2_simd_permute(const uint32_t *in, size_t in_stride, uint32_t *out, size_t out_stride, uint64_t n) {
    static const bool ok = __builtin_cpu_supports("avx512f");
    if (!ok || in_stride >= (1u << 27) || out_stride >= (1u << 27)) return 0;
    return run(in, in_stride, out, out_stride, n);
}
}  // namespace zkm_host
