/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).
 *
 * The coset LDE of dft.c (orc_coset_lde_bitrev) for the CPU baseline: 16 columns at a time as one
 * h x 16 block whose rows are AVX-512 vectors, so every butterfly is a 16-lane vector operation on
 * contiguous memory and the row-major gather/scatter moves whole 64-byte rows.  Same output bit for bit
 * (the transform is exact arithmetic).  Stages run with every thread on one block; once a stage's
 * butterfly span fits a cache-sized tile, each thread finishes all remaining stages of its tile.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle_internal.h"
#include "x16.h"

#define TILE_LOG 11  /* 2^11 rows x 64 B = 128 KiB */
#define PAR_MIN (1u << 14)  /* smaller blocks stay on the calling thread (no team start-up per stage) */

/* twiddles w_n^j * R (Montgomery form), j < n/2 */
static uint32_t *twm_cache[2][32];
static const uint32_t *twiddles_mont(int logn, int inverse) {
    uint32_t *t = __atomic_load_n(&twm_cache[inverse][logn], __ATOMIC_ACQUIRE);
    if (t) return t;
    size_t h = ((size_t)1 << logn) >> 1;
    t = (uint32_t *)malloc(sizeof(uint32_t) * (h ? h : 1));
    kb_t w = kb_two_adic_gen(logn);
    if (inverse) w = kb_inv(w);
    kb_t x = 1;
    for (size_t j = 0; j < h; j++) { t[j] = orc_x16_to_mont(x); x = kb_mul(x, w); }
    uint32_t *expect = NULL;
    if (!__atomic_compare_exchange_n(&twm_cache[inverse][logn], &expect, t, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
        free(t);
        t = expect;
    }
    return t;
}

/* one DIF stage of span m = 2^s over rows [lo, hi) of a (rows are 16-lane vectors) */
TGT static inline void dif_stage(uint32_t *a, size_t lo, size_t hi, int s, int logn, const uint32_t *tw) {
    const size_t m = (size_t)1 << s, h = m >> 1, stride = ((size_t)1 << logn) >> s;
    for (size_t k = lo; k < hi; k += m)
        for (size_t j = 0; j < h; j++) {
            __m512i *pu = (__m512i *)(a + 16 * (k + j)), *pv = (__m512i *)(a + 16 * (k + j + h));
            __m512i u = _mm512_load_si512(pu), v = _mm512_load_si512(pv);
            _mm512_store_si512(pu, madd(u, v));
            _mm512_store_si512(pv, mmul(msub(u, v), _mm512_set1_epi32((int)tw[j * stride])));
        }
}

/* natural-order input, bit-reversed output, on an n x 16 block */
TGT static void dif16(uint32_t *a, int logn, const uint32_t *tw) {
    const size_t n = (size_t)1 << logn;
    int s = logn;
    for (; s > TILE_LOG; s--) {  /* wide stages: all threads over the butterflies of the stage */
        const size_t m = (size_t)1 << s, h = m >> 1, stride = n >> s;
#pragma omp parallel for schedule(static) if (n >= PAR_MIN)
        for (size_t b = 0; b < n / 2; b++) {
            const size_t k = (b / h) * m, j = b % h;
            __m512i *pu = (__m512i *)(a + 16 * (k + j)), *pv = (__m512i *)(a + 16 * (k + j + h));
            __m512i u = _mm512_load_si512(pu), v = _mm512_load_si512(pv);
            _mm512_store_si512(pu, madd(u, v));
            _mm512_store_si512(pv, mmul(msub(u, v), _mm512_set1_epi32((int)tw[j * stride])));
        }
    }
    const size_t tile = (size_t)1 << s;  /* remaining stages stay inside tiles of 2^s rows */
#pragma omp parallel for schedule(static) if (n > tile)
    for (size_t t0 = 0; t0 < n; t0 += tile)
        for (int ss = s; ss >= 1; ss--) dif_stage(a, t0, t0 + tile, ss, logn, tw);
}

TGT void orc_coset_lde_bitrev_x16(const kb_t *evals, size_t h, size_t w, int log_blowup, kb_t shift, kb_t *out) {
    const int logh = log2_exact(h), logH = logh + log_blowup;
    const size_t H = (size_t)1 << logH;
    const uint32_t *twi = twiddles_mont(logh, 1), *twf = twiddles_mont(logH, 0);
    uint32_t *A = (uint32_t *)aligned_alloc(64, 64 * h), *E = (uint32_t *)aligned_alloc(64, 64 * H);
    uint32_t *sm = (uint32_t *)malloc(sizeof(uint32_t) * h);  /* (shift^i / h) * R */
    const kb_t hinv = kb_inv((kb_t)(h % KB_P));
#pragma omp parallel for schedule(static) if (h >= PAR_MIN)
    for (size_t c0 = 0; c0 < h; c0 += 4096) {
        kb_t x = kb_mul(hinv, kb_pow(shift, c0));
        for (size_t i = c0; i < h && i < c0 + 4096; i++) { sm[i] = orc_x16_to_mont(x); x = kb_mul(x, shift); }
    }
    for (size_t c0 = 0; c0 < w; c0 += 16) {
        const size_t g = w - c0 < 16 ? w - c0 : 16;
#pragma omp parallel for schedule(static) if (h >= PAR_MIN)
        for (size_t i = 0; i < h; i++) {
            uint32_t *row = A + 16 * i;
            memcpy(row, evals + i * w + c0, 4 * g);
            if (g < 16) memset(row + g, 0, 4 * (16 - g));
        }
        dif16(A, logh, twi);
#pragma omp parallel for schedule(static) if (H >= PAR_MIN)
        for (size_t i = 0; i < H; i++) {
            __m512i v = _mm512_setzero_si512();
            if (i < h)
                v = mmul(_mm512_load_si512((const void *)(A + 16 * (size_t)rev_bits((uint32_t)i, logh))),
                         _mm512_set1_epi32((int)sm[i]));
            _mm512_store_si512((void *)(E + 16 * i), v);
        }
        dif16(E, logH, twf);
#pragma omp parallel for schedule(static) if (H >= PAR_MIN)
        for (size_t i = 0; i < H; i++) memcpy(out + i * w + c0, E + 16 * i, 4 * g);
    }
    free(A);
    free(E);
    free(sm);
}
