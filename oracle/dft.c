/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).
 *
 * Coset LDE restated from the semantics the reference relies on:
 *   TwoAdicFriPcs::commit = coset_lde_batch(evals, log_blowup, GENERATOR/domain.shift)
 *   followed by bit_reverse_rows  (call sites crates/stark/src/prover.rs:277,403,497,
 *   crates/stark/src/machine.rs:397; Radix2DitParallel, kb31_poseidon2.rs:179).
 * Row i of the committed LDE is the evaluation at shift' * w_{2n}^{rev(i)}, which the
 * verifier pins in crates/recursion/circuit/src/fri.rs:134-150 (x = g * w^rev(index)).
 * Exact arithmetic: any correct DFT algorithm gives identical output; this one is the
 * textbook iterative radix-2 (bit-reverse + DIT), one column at a time.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle_internal.h"

void orc_dft_natural(kb_t *a, int logn, int inverse) {
    size_t n = (size_t)1 << logn;
    for (size_t i = 0; i < n; i++) {
        size_t j = rev_bits((uint32_t)i, logn);
        if (j > i) { kb_t t = a[i]; a[i] = a[j]; a[j] = t; }
    }
    for (int s = 1; s <= logn; s++) {
        size_t m = (size_t)1 << s, h = m >> 1;
        kb_t wm = kb_two_adic_gen(s);
        if (inverse) wm = kb_inv(wm);
        kb_t *tw = (kb_t *)malloc(h * sizeof(kb_t));
        tw[0] = 1;
        for (size_t j = 1; j < h; j++) tw[j] = kb_mul(tw[j - 1], wm);
        for (size_t k = 0; k < n; k += m)
            for (size_t j = 0; j < h; j++) {
                kb_t u = a[k + j], v = kb_mul(a[k + j + h], tw[j]);
                a[k + j] = kb_add(u, v);
                a[k + j + h] = kb_sub(u, v);
            }
        free(tw);
    }
    if (inverse) {
        kb_t ninv = kb_inv((kb_t)(n % KB_P));
        for (size_t i = 0; i < n; i++) a[i] = kb_mul(a[i], ninv);
    }
}

/* coefficients (natural order) of the poly interpolating column `col` of a row-major
 * matrix over H_n */
void orc_interpolate_col(const kb_t *m, size_t h, size_t w, size_t col, kb_t *coeffs) {
    for (size_t i = 0; i < h; i++) coeffs[i] = m[i * w + col];
    orc_dft_natural(coeffs, log2_exact(h), 1);
}

/* w_n^j (or w_n^-j), j < n/2, for n = 2^logn: built once per (logn, direction) and kept */
static kb_t *tw_cache[2][32];
static const kb_t *twiddles(int logn, int inverse) {
    kb_t *t = __atomic_load_n(&tw_cache[inverse][logn], __ATOMIC_ACQUIRE);
    if (t) return t;
    size_t h = ((size_t)1 << logn) >> 1;
    t = (kb_t *)malloc(sizeof(kb_t) * (h ? h : 1));
    kb_t w = kb_two_adic_gen(logn);
    if (inverse) w = kb_inv(w);
    kb_t x = 1;
    for (size_t j = 0; j < h; j++) { t[j] = x; x = kb_mul(x, w); }
    kb_t *expect = NULL;
    if (!__atomic_compare_exchange_n(&tw_cache[inverse][logn], &expect, t, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
        free(t);
        t = expect;
    }
    return t;
}

/* decimation-in-frequency radix-2 transform: natural-order input, bit-reversed output */
static void dif(kb_t *a, int logn, const kb_t *tw) {
    size_t n = (size_t)1 << logn;
    for (int s = logn; s >= 1; s--) {
        size_t m = (size_t)1 << s, h = m >> 1, stride = n >> s;
        for (size_t k = 0; k < n; k += m)
            for (size_t j = 0; j < h; j++) {
                kb_t u = a[k + j], v = a[k + j + h];
                a[k + j] = kb_add(u, v);
                a[k + j + h] = kb_mul(kb_sub(u, v), tw[j * stride]);
            }
    }
}

/* evals: h x w row-major, treated as evaluations over H_h (natural order).
 * out: (h << log_blowup) x w row-major, bit-reversed rows, row i = p(shift * w^{rev(i)}).
 * Per column: inverse DIF (coefficients, bit-reversed), reorder and scale by shift^i / h, zero-extend,
 * forward DIF, whose bit-reversed output is already the committed row order.  Columns go in groups
 * of 8 so the row-major gather and scatter touch whole cache lines. */
#define LDE_G 8
void orc_coset_lde_bitrev(const kb_t *evals, size_t h, size_t w, int log_blowup, kb_t shift, kb_t *out) {
    int logh = log2_exact(h);
    int logH = logh + log_blowup;
    size_t H = (size_t)1 << logH;
    if (h >= 16 && orc_p2x16_available()) {  /* 16 columns per AVX-512 block (lde_x16.c) */
        orc_coset_lde_bitrev_x16(evals, h, w, log_blowup, shift, out);
        return;
    }
    const kb_t *twi = twiddles(logh, 1), *twf = twiddles(logH, 0);
    const kb_t hinv = kb_inv((kb_t)(h % KB_P));
#pragma omp parallel for schedule(dynamic, 1)
    for (size_t c0 = 0; c0 < w; c0 += LDE_G) {
        const size_t g = w - c0 < LDE_G ? w - c0 : LDE_G;
        kb_t *buf = (kb_t *)malloc(sizeof(kb_t) * h * g), *ext = (kb_t *)malloc(sizeof(kb_t) * H * g);
        for (size_t i = 0; i < h; i++)
            for (size_t k = 0; k < g; k++) buf[k * h + i] = evals[i * w + c0 + k];
        for (size_t k = 0; k < g; k++) {
            kb_t *b = buf + k * h, *e = ext + k * H;
            dif(b, logh, twi);
            kb_t s = hinv;
            for (size_t i = 0; i < h; i++) { e[i] = kb_mul(b[rev_bits((uint32_t)i, logh)], s); s = kb_mul(s, shift); }
            memset(e + h, 0, sizeof(kb_t) * (H - h));
            dif(e, logH, twf);
        }
        for (size_t i = 0; i < H; i++)
            for (size_t k = 0; k < g; k++) out[i * w + c0 + k] = ext[k * H + i];
        free(buf);
        free(ext);
    }
}

/* evaluate a natural-order coefficient vector at an extension point (Horner) */
ef_t orc_eval_coeffs_ef(const kb_t *coeffs, size_t n, ef_t z) {
    ef_t acc = ef_zero();
    for (size_t i = n; i-- > 0;) acc = ef_add_base(ef_mul(acc, z), coeffs[i]);
    return acc;
}
