/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h header).
 *
 * Poseidon2-16 over KoalaBear as configured by the reference:
 *   poseidon2_init: RF = 8, RP = 13, constants RC_16_30
 *     (crates/primitives/src/lib.rs:1107-1122; same split in
 *      crates/stark/src/kb31_poseidon2.rs:184-199)
 *   x^3 S-box, M4-based external layer, 1 + diag(V) internal layer
 *     (crates/recursion/core/include/poseidon2.hpp:20-71,
 *      crates/recursion/core/include/poseidon2_wide.hpp:10-145,
 *      crates/core/machine/src/operations/poseidon2/air.rs:12-56)
 *   PaddingFreeSponge<Perm,16,8,8> (kb31_poseidon2.rs:173; semantics pinned by
 *     crates/recursion/circuit/src/hash.rs:40-50)
 *   TruncatedPermutation<Perm,2,8,16> (kb31_poseidon2.rs:175;
 *     crates/recursion/compiler/src/circuit/builder.rs:167-177)
 */
#pragma once
#include "kb31.h"

#define P2_WIDTH 16
#define P2_RATE 8
#define DIGEST_ELEMS 8

typedef struct { kb_t v[DIGEST_ELEMS]; } digest_t;

void orc_p2_permute(kb_t st[P2_WIDTH]);
/* sponge over a flat list of field elements */
digest_t orc_p2_hash(const kb_t *in, size_t n);
digest_t orc_p2_compress(digest_t l, digest_t r);

/* incremental sponge absorbing row slices of several matrices in order */
typedef struct { kb_t st[P2_WIDTH]; int pos; int any; } orc_sponge_t;
static inline void orc_sponge_init(orc_sponge_t *s) { memset(s, 0, sizeof *s); }
static inline void orc_sponge_absorb(orc_sponge_t *s, const kb_t *in, size_t n) {
    for (size_t i = 0; i < n; i++) {
        s->st[s->pos++] = in[i];
        s->any = 1;
        if (s->pos == P2_RATE) { orc_p2_permute(s->st); s->pos = 0; }
    }
}
static inline digest_t orc_sponge_finish(orc_sponge_t *s) {
    if (s->pos != 0) orc_p2_permute(s->st);
    digest_t d;
    memcpy(d.v, s->st, sizeof d.v);
    return d;
}
