/* ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).  Poseidon2-16 restatement. */
#include "poseidon2.h"
#include "p2_rc.h"

#define RF 8
#define RP 13

/* internal diagonal V (canonical), crates/core/machine/src/operations/poseidon2/air.rs:12-29 */
static const kb_t DIAG[16] = {
    KB_P - 2, 1, 2, (KB_P + 1) >> 1, 3, 4, (KB_P - 1) >> 1, KB_P - 3, KB_P - 4,
    KB_P - ((KB_P - 1) >> 8), KB_P - ((KB_P - 1) >> 3), KB_P - 127,
    (KB_P - 1) >> 8, (KB_P - 1) >> 3, (KB_P - 1) >> 4, 127,
};

static void m4(kb_t *x) {
    /* apply_m_4 (air.rs:31-42): matrix [[2,3,1,1],[1,2,3,1],[1,1,2,3],[3,1,1,2]] */
    kb_t t01 = kb_add(x[0], x[1]);
    kb_t t23 = kb_add(x[2], x[3]);
    kb_t t0123 = kb_add(t01, t23);
    kb_t t01123 = kb_add(t0123, x[1]);
    kb_t t01233 = kb_add(t0123, x[3]);
    kb_t n3 = kb_add(t01233, kb_add(x[0], x[0]));
    kb_t n1 = kb_add(t01123, kb_add(x[2], x[2]));
    kb_t n0 = kb_add(t01123, t01);
    kb_t n2 = kb_add(t01233, t23);
    x[0] = n0; x[1] = n1; x[2] = n2; x[3] = n3;
}

static void external_layer(kb_t *s) {
    for (int j = 0; j < 16; j += 4) m4(s + j);
    kb_t sums[4];
    for (int k = 0; k < 4; k++) sums[k] = kb_add(kb_add(s[k], s[4 + k]), kb_add(s[8 + k], s[12 + k]));
    for (int j = 0; j < 16; j++) s[j] = kb_add(s[j], sums[j & 3]);
}

static void internal_layer(kb_t *s) {
    kb_t sum = 0;
    for (int i = 0; i < 16; i++) sum = kb_add(sum, s[i]);
    for (int i = 0; i < 16; i++) s[i] = kb_add(kb_mul(s[i], DIAG[i]), sum);
}

static inline kb_t cube(kb_t x) { return kb_mul(kb_mul(x, x), x); }

void orc_p2_permute(kb_t st[16]) {
    external_layer(st);
    for (int r = 0; r < RF / 2; r++) {
        for (int i = 0; i < 16; i++) st[i] = cube(kb_add(st[i], ORC_P2_RC[r][i]));
        external_layer(st);
    }
    for (int r = 0; r < RP; r++) {
        st[0] = cube(kb_add(st[0], ORC_P2_RC[RF / 2 + r][0]));
        internal_layer(st);
    }
    for (int r = RF / 2; r < RF; r++) {
        for (int i = 0; i < 16; i++) st[i] = cube(kb_add(st[i], ORC_P2_RC[r + RP][i]));
        external_layer(st);
    }
}

digest_t orc_p2_hash(const kb_t *in, size_t n) {
    orc_sponge_t s;
    orc_sponge_init(&s);
    orc_sponge_absorb(&s, in, n);
    return orc_sponge_finish(&s);
}

digest_t orc_p2_compress(digest_t l, digest_t r) {
    kb_t st[16];
    memcpy(st, l.v, 32);
    memcpy(st + 8, r.v, 32);
    orc_p2_permute(st);
    digest_t d;
    memcpy(d.v, st, 32);
    return d;
}
