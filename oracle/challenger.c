/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).
 *
 * DuplexChallenger<KoalaBear, Poseidon2KoalaBear<16>, 16, 8>
 * (crates/stark/src/kb31_poseidon2.rs:180), semantics pinned by the in-circuit
 * restatement crates/recursion/circuit/src/challenger.rs:89-233:
 *   observe: clear outputs, push input, duplex when 8 inputs are pending;
 *   sample : duplex if inputs pending or outputs empty, then POP FROM THE END;
 *   duplex : state[0..n] = inputs, permute, outputs = state[0..8];
 *   sample_ext = 4 samples (coeffs 0..3); sample_bits(b) = low b bits of canonical;
 *   check_witness = observe(w); sample_bits(b) == 0.
 * Grinding: the reference's witness search is a parallel find_any (nondeterministic);
 * the canonical witness here is the SMALLEST valid one.
 */
#include "oracle_internal.h"

void orc_chal_init(orc_chal_t *c) { memset(c, 0, sizeof *c); }

static void duplex(orc_chal_t *c) {
    for (int i = 0; i < c->nin; i++) c->st[i] = c->in[i];
    c->nin = 0;
    orc_p2_permute(c->st);
    memcpy(c->out, c->st, sizeof c->out);
    c->nout = 8;
}

void orc_chal_observe(orc_chal_t *c, kb_t v) {
    c->nout = 0;
    c->in[c->nin++] = v;
    if (c->nin == 8) duplex(c);
}
void orc_chal_observe_slice(orc_chal_t *c, const kb_t *v, size_t n) {
    for (size_t i = 0; i < n; i++) orc_chal_observe(c, v[i]);
}
void orc_chal_observe_digest(orc_chal_t *c, digest_t d) { orc_chal_observe_slice(c, d.v, 8); }
void orc_chal_observe_ef(orc_chal_t *c, ef_t e) { orc_chal_observe_slice(c, e.c, 4); }

kb_t orc_chal_sample(orc_chal_t *c) {
    if (c->nin != 0 || c->nout == 0) duplex(c);
    return c->out[--c->nout];
}
ef_t orc_chal_sample_ef(orc_chal_t *c) {
    ef_t e;
    for (int i = 0; i < 4; i++) e.c[i] = orc_chal_sample(c);
    return e;
}
uint32_t orc_chal_sample_bits(orc_chal_t *c, int bits) {
    return orc_chal_sample(c) & ((1u << bits) - 1);
}
int orc_chal_check_witness(orc_chal_t *c, int bits, kb_t w) {
    orc_chal_observe(c, w);
    return orc_chal_sample_bits(c, bits) == 0;
}
kb_t orc_chal_grind(orc_chal_t *c, int bits) {
    for (kb_t w = 0; w < KB_P; w++) {
        orc_chal_t t = *c;
        if (orc_chal_check_witness(&t, bits, w)) {
            orc_chal_check_witness(c, bits, w);
            return w;
        }
    }
    return 0;
}
