/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).
 * Internal declarations of the CPU restatement of the reference's per-shard
 * STARK prover (crates/stark/src/prover.rs CpuProver::commit/open) and of the
 * Plonky3 PCS/FRI semantics pinned by crates/recursion/circuit/src/fri.rs.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>
#include "kb31.h"
#include "poseidon2.h"

/* ------------------------------------------------------------------ dft.c */
void orc_dft_natural(kb_t *a, int logn, int inverse);
void orc_interpolate_col(const kb_t *m, size_t h, size_t w, size_t col, kb_t *coeffs);
void orc_coset_lde_bitrev(const kb_t *evals, size_t h, size_t w, int log_blowup, kb_t shift, kb_t *out);
void orc_coset_lde_bitrev_x16(const kb_t *evals, size_t h, size_t w, int log_blowup, kb_t shift, kb_t *out);
ef_t orc_eval_coeffs_ef(const kb_t *coeffs, size_t n, ef_t z);

/* ----------------------------------------------------------------- mmcs.c */
typedef struct {
    const kb_t *data; /* row-major */
    size_t height, width;
} orc_mat_t;

typedef struct {
    int nmats;
    orc_mat_t *mats;      /* commit order (borrowed or owned, see owns) */
    int owns;
    int log_max_height;
    digest_t **layers;    /* layers[0] = leaves (max_height), ..., layers[L] = root */
    int nlayers;
} orc_tree_t;

void orc_tree_build(orc_tree_t *t, orc_mat_t *mats, int nmats, int owns);
/* p2x16.c: 16 Poseidon2 states per AVX-512 batch (same digests as poseidon2.c) */
int orc_p2x16_available(void);
void orc_p2x16_hash_rows(const orc_mat_t *mats, const int *group, int ng, size_t row0, digest_t *out);
void orc_p2x16_compress_pairs(const digest_t *in, digest_t *out);
void orc_p2x16_compress2(const digest_t *a, const digest_t *b, digest_t *out);
void orc_tree_free(orc_tree_t *t);
digest_t orc_tree_root(const orc_tree_t *t);
/* rows: per matrix, pointer into the matrix (no copy); path: log_max_height digests */
void orc_tree_open(const orc_tree_t *t, size_t index, const kb_t **rows, digest_t *path);
/* verify: dims heights in matrix order; values per matrix (widths given) */
int orc_verify_batch(digest_t commit, int nmats, const size_t *heights, const size_t *widths,
                     const kb_t *const *values, size_t index, const digest_t *path, int path_len);

/* ----------------------------------------------------------- challenger.c */
typedef struct {
    kb_t st[16];
    kb_t in[8]; int nin;
    kb_t out[8]; int nout;
} orc_chal_t;
void orc_chal_init(orc_chal_t *c);
void orc_chal_observe(orc_chal_t *c, kb_t v);
void orc_chal_observe_slice(orc_chal_t *c, const kb_t *v, size_t n);
void orc_chal_observe_digest(orc_chal_t *c, digest_t d);
void orc_chal_observe_ef(orc_chal_t *c, ef_t e);
kb_t orc_chal_sample(orc_chal_t *c);
ef_t orc_chal_sample_ef(orc_chal_t *c);
uint32_t orc_chal_sample_bits(orc_chal_t *c, int bits);
int orc_chal_check_witness(orc_chal_t *c, int bits, kb_t w);
kb_t orc_chal_grind(orc_chal_t *c, int bits);

/* -------------------------------------------------------------- machine.c */
enum { OP_END = 0, OP_MAIN_L, OP_MAIN_N, OP_PREP_L, OP_PREP_N, OP_CONST, OP_PV,
       OP_IS_FIRST, OP_IS_LAST, OP_IS_TRANS, OP_ADD, OP_SUB, OP_MUL, OP_NEG, OP_EMIT,
       OP_LET, OP_GET /* shared subexpressions: LET s pops into value slot s, GET s pushes it */ };

typedef struct { int nterms; uint32_t *cols; kb_t *weights; kb_t constant; } orc_vpc_t;
typedef struct { uint32_t kind, scope; int nvalues; orc_vpc_t *values; orc_vpc_t mult; int is_send; } orc_lookup_t;

typedef struct {
    char name[64];
    int prep_width, main_width, commit_scope, local_only, log_qd, num_main_constraints;
    int code_len; uint32_t *code;
    int n_slots; /* 1 + the largest LET slot (0 without shared subexpressions) */
    int nlocal; orc_lookup_t *local; /* local-scope lookups: sends then receives (stable) */
    int nsends, nrecvs;
    int perm_width_ef; /* 0 if no local lookups, else ceil(nlocal/batch)+1 */
    int num_constraints;
} orc_chip_t;

typedef struct { int num_pv; int nchips; orc_chip_t *chips; } orc_machine_t;

int orc_machine_parse(orc_machine_t *m, const uint32_t *w, size_t n);
void orc_machine_free(orc_machine_t *m);
kb_t orc_vpc_apply(const orc_vpc_t *v, const kb_t *prep, const kb_t *main);
ef_t orc_vpc_apply_ef(const orc_vpc_t *v, const ef_t *prep, const ef_t *main);

/* ----------------------------------------------------------------- config */
#define LOG_BLOWUP 1
#define POW_BITS 16
#define CURVE_START_X {637514027u, 1595065213u, 1998064738u, 72333738u, 1211544370u, 822986770u, 1518535784u}
#define CURVE_START_Y {1604177449u, 90440090u, 259343427u, 140470264u, 1162099742u, 941559812u, 1064053343u}
