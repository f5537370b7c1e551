/* ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).  Shard prover/verifier restatement. */
#pragma once
#include "oracle_internal.h"

typedef struct {
    int num_queries;   /* FRI_QUERIES, default 84 (crates/stark/src/kb31_poseidon2.rs:208-212) */
    int pow_bits;      /* 16 */
    int log_blowup;    /* 1 */
    int montgomery_bytes; /* serialize field elements as Montgomery u32 instead of canonical */
} orc_config_t;

typedef struct {
    const orc_machine_t *m;
    orc_config_t cfg;
    digest_t commit;
    kb_t pc_start;
    kb_t gcs[14];
    int ntraces;
    int *trace_chip;        /* machine chip index of each preprocessed trace (pk order) */
    orc_tree_t tree;        /* owns the LDEs */
    kb_t **traces;          /* owned copies, row-major */
    size_t *heights;
} orc_pk_t;

/* ---- proof object (mirrors ShardProof, crates/stark/src/types.rs:77-83) ---- */
typedef struct { int w; ef_t *local, *next; } orc_air_open_t;
typedef struct {
    orc_air_open_t prep, main, perm;
    int nq; ef_t *quot;     /* nq chunks x 4 EF */
    kb_t gcs[14];
    ef_t lcs;
    int log_degree;
} orc_chip_open_t;
typedef struct { int nmats; size_t *widths; kb_t **vals; int path_len; digest_t *path; } orc_batch_open_t;
typedef struct { ef_t sibling; int path_len; digest_t *path; } orc_step_t;
typedef struct { int nrounds; orc_batch_open_t *input; int nsteps; orc_step_t *steps; } orc_query_t;
typedef struct {
    int ncommits; digest_t *commits;
    int nqueries; orc_query_t *queries;
    ef_t final_poly; kb_t pow_witness;
} orc_fri_t;
typedef struct {
    digest_t main_commit, perm_commit, quot_commit;
    int nchips; orc_chip_open_t *chips;
    orc_fri_t fri;
    char (*ord_names)[64]; /* chip_ordering, sorted by index */
    int npv; kb_t *pv;
} orc_proof_t;

int orc_setup(orc_pk_t *pk, const orc_machine_t *m, orc_config_t cfg, const kb_t *const *prep_traces,
              const size_t *prep_heights, kb_t pc_start, const kb_t *gcs);
void orc_pk_free(orc_pk_t *pk);
void orc_pk_observe(const orc_pk_t *pk, orc_chal_t *ch);

/* traces: one per shard chip (machine chip index chip_idx[i]), row-major canonical */
int orc_prove_shard(const orc_pk_t *pk, int n, const int *chip_idx, const kb_t *const *traces,
                    const size_t *heights, const kb_t *pv, int npv, orc_chal_t *ch, orc_proof_t *out);
int orc_verify_shard(const orc_pk_t *vk, const orc_proof_t *p, orc_chal_t *ch);
void orc_proof_free(orc_proof_t *p);

size_t orc_proof_serialize(const orc_proof_t *p, const orc_config_t *cfg, uint8_t **out);
size_t orc_serialize_digest_map(const uint32_t *keys, const uint64_t *vals, uint64_t n, int montgomery, uint8_t **out);
int orc_proof_deserialize(orc_proof_t *p, const orc_config_t *cfg, const uint8_t *b, size_t n);
