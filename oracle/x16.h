/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).
 *
 * KoalaBear arithmetic on 16 lanes (AVX-512F, Montgomery multiplication with R = 2^32) shared by the
 * CPU baseline's batched Poseidon2 (p2x16.c) and coset LDE (lde_x16.c).  mmul(a, bR) = a*b: with one
 * operand pre-multiplied by R (twiddles, round constants) data can stay canonical.
 */
#pragma once
#include <immintrin.h>
#include <stdint.h>

#include "kb31.h"

#define TGT __attribute__((target("avx512f")))

extern uint32_t ORC_X16_MU;
int orc_x16_available(void);
uint32_t orc_x16_to_mont(uint32_t x);

TGT static inline __m512i vp(void) { return _mm512_set1_epi32((int)KB_P); }

TGT static inline __m512i madd(__m512i a, __m512i b) {
    __m512i s = _mm512_add_epi32(a, b);
    return _mm512_min_epu32(s, _mm512_sub_epi32(s, vp()));
}

TGT static inline __m512i msub(__m512i a, __m512i b) {
    __m512i d = _mm512_sub_epi32(a, b);
    return _mm512_min_epu32(d, _mm512_add_epi32(d, vp()));
}

/* a * b * 2^-32 mod p for a, b < p */
TGT static inline __m512i mmul(__m512i a, __m512i b) {
    const __m512i mu = _mm512_set1_epi32((int)ORC_X16_MU), p = vp();
    __m512i a_odd = _mm512_srli_epi64(a, 32), b_odd = _mm512_srli_epi64(b, 32);
    __m512i pe = _mm512_mul_epu32(a, b), po = _mm512_mul_epu32(a_odd, b_odd);
    __m512i qe = _mm512_mul_epu32(pe, mu), qo = _mm512_mul_epu32(po, mu);
    __m512i te = _mm512_add_epi64(pe, _mm512_mul_epu32(qe, p));
    __m512i to = _mm512_add_epi64(po, _mm512_mul_epu32(qo, p));
    __m512i t = _mm512_mask_blend_epi32(0xAAAA, _mm512_srli_epi64(te, 32), to);
    return _mm512_min_epu32(t, _mm512_sub_epi32(t, p));
}
