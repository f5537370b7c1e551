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

/* evals: h x w row-major, treated as evaluations over H_h (natural order).
 * out: (h << log_blowup) x w row-major, bit-reversed rows, row i = p(shift * w^{rev(i)}). */
void orc_coset_lde_bitrev(const kb_t *evals, size_t h, size_t w, int log_blowup, kb_t shift, kb_t *out) {
    int logh = log2_exact(h);
    int logH = logh + log_blowup;
    size_t H = (size_t)1 << logH;
#pragma omp parallel for schedule(dynamic, 1)
    for (size_t c = 0; c < w; c++) {
        kb_t *buf = (kb_t *)calloc(H, sizeof(kb_t));
        for (size_t i = 0; i < h; i++) buf[i] = evals[i * w + c];
        orc_dft_natural(buf, logh, 1);
        kb_t s = 1;
        for (size_t i = 0; i < h; i++) { buf[i] = kb_mul(buf[i], s); s = kb_mul(s, shift); }
        orc_dft_natural(buf, logH, 0);
        for (size_t i = 0; i < H; i++) out[i * w + c] = buf[rev_bits((uint32_t)i, logH)];
        free(buf);
    }
}

/* evaluate a natural-order coefficient vector at an extension point (Horner) */
ef_t orc_eval_coeffs_ef(const kb_t *coeffs, size_t n, ef_t z) {
    ef_t acc = ef_zero();
    for (size_t i = n; i-- > 0;) acc = ef_add_base(ef_mul(acc, z), coeffs[i]);
    return acc;
}
