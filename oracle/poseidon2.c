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

/* Linear layers accumulate in 64 bits and reduce once per output element (every intermediate is a
 * small multiple of p, far below 2^64); S-box inputs x + rc stay below 2^32. */
static inline kb_t red(uint64_t x) { return (kb_t)(x % KB_P); }

static void external_layer(kb_t *s) {
    /* apply_m_4 (air.rs:31-42): matrix [[2,3,1,1],[1,2,3,1],[1,1,2,3],[3,1,1,2]] per 4-block,
     * then add the column sums over the four blocks (air.rs:44-56) */
    uint64_t t[16];
    for (int j = 0; j < 16; j += 4) {
        uint64_t x0 = s[j], x1 = s[j + 1], x2 = s[j + 2], x3 = s[j + 3];
        uint64_t t01 = x0 + x1, t23 = x2 + x3, t0123 = t01 + t23;
        uint64_t t01123 = t0123 + x1, t01233 = t0123 + x3;
        t[j] = t01123 + t01;
        t[j + 1] = t01123 + 2 * x2;
        t[j + 2] = t01233 + t23;
        t[j + 3] = t01233 + 2 * x0;
    }
    uint64_t sums[4];
    for (int k = 0; k < 4; k++) sums[k] = t[k] + t[4 + k] + t[8 + k] + t[12 + k];
    for (int j = 0; j < 16; j++) s[j] = red(t[j] + sums[j & 3]);
}

static void internal_layer(kb_t *s) {
    uint64_t sum = 0;
    for (int i = 0; i < 16; i++) sum += s[i];
    for (int i = 0; i < 16; i++) s[i] = red((uint64_t)s[i] * DIAG[i] + sum);
}

/* (x + rc)^3 with x, rc < p */
static inline kb_t sbox(kb_t x, kb_t rc) {
    uint64_t y = (uint64_t)x + rc;
    return red((uint64_t)red(y * y) * y);
}

void orc_p2_permute(kb_t st[16]) {
    external_layer(st);
    for (int r = 0; r < RF / 2; r++) {
        for (int i = 0; i < 16; i++) st[i] = sbox(st[i], ORC_P2_RC[r][i]);
        external_layer(st);
    }
    for (int r = 0; r < RP; r++) {
        st[0] = sbox(st[0], ORC_P2_RC[RF / 2 + r][0]);
        internal_layer(st);
    }
    for (int r = RF / 2; r < RF; r++) {
        for (int i = 0; i < 16; i++) st[i] = sbox(st[i], ORC_P2_RC[r + RP][i]);
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
