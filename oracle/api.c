/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).
 * Flat C entry points for ctypes (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 * Challenger state words: st[16], nin, in[8], nout, out[8]  (34 x u32, canonical values).
 */
#include <stdlib.h>
#include "stark.h"

static void chal_load(orc_chal_t *c, const uint32_t *s) {
    memcpy(c->st, s, 64); c->nin = (int)s[16]; memcpy(c->in, s + 17, 32); c->nout = (int)s[25]; memcpy(c->out, s + 26, 32);
}
static void chal_store(const orc_chal_t *c, uint32_t *s) {
    memcpy(s, c->st, 64); s[16] = (uint32_t)c->nin; memcpy(s + 17, c->in, 32); s[25] = (uint32_t)c->nout; memcpy(s + 26, c->out, 32);
}

void orc_api_p2_permute(uint32_t *st) { orc_p2_permute(st); }
void orc_api_hash(const uint32_t *in, uint64_t n, uint32_t *out) { digest_t d = orc_p2_hash(in, n); memcpy(out, d.v, 32); }
void orc_api_compress(const uint32_t *l, const uint32_t *r, uint32_t *out) {
    digest_t a, b; memcpy(a.v, l, 32); memcpy(b.v, r, 32);
    digest_t d = orc_p2_compress(a, b); memcpy(out, d.v, 32);
}
void orc_api_lde(const uint32_t *evals, uint64_t h, uint64_t w, int log_blowup, uint32_t shift, uint32_t *out) {
    orc_coset_lde_bitrev(evals, h, w, log_blowup, shift, out);
}
void orc_api_dft(uint32_t *a, int logn, int inverse) { orc_dft_natural(a, logn, inverse); }
void orc_api_merkle_root(int nmats, const uint32_t *const *mats, const uint64_t *heights, const uint64_t *widths, uint32_t *root) {
    orc_mat_t *m = (orc_mat_t *)malloc(sizeof(orc_mat_t) * nmats);
    for (int i = 0; i < nmats; i++) { m[i].data = mats[i]; m[i].height = heights[i]; m[i].width = widths[i]; }
    orc_tree_t t;
    orc_tree_build(&t, m, nmats, 0);
    digest_t d = orc_tree_root(&t);
    memcpy(root, d.v, 32);
    orc_tree_free(&t);
    free(m);
}
/* commit = LDE(blowup 2, shift 3) of every matrix, bit-reversed, then MMCS root */
void orc_api_commit_root(int nmats, const uint32_t *const *mats, const uint64_t *heights, const uint64_t *widths, uint32_t *root) {
    orc_mat_t *m = (orc_mat_t *)malloc(sizeof(orc_mat_t) * nmats);
    for (int i = 0; i < nmats; i++) {
        kb_t *o = (kb_t *)malloc(sizeof(kb_t) * heights[i] * 2 * (widths[i] ? widths[i] : 1));
        if (widths[i]) orc_coset_lde_bitrev(mats[i], heights[i], widths[i], 1, KB_GENERATOR, o);
        m[i].data = o; m[i].height = heights[i] * 2; m[i].width = widths[i];
    }
    orc_tree_t t;
    orc_tree_build(&t, m, nmats, 1);
    digest_t d = orc_tree_root(&t);
    memcpy(root, d.v, 32);
    orc_tree_free(&t);
}

void orc_api_chal_observe(uint32_t *s, const uint32_t *v, uint64_t n) {
    orc_chal_t c; chal_load(&c, s); orc_chal_observe_slice(&c, v, n); chal_store(&c, s);
}
void orc_api_chal_sample(uint32_t *s, uint32_t *out, uint64_t n) {
    orc_chal_t c; chal_load(&c, s); for (uint64_t i = 0; i < n; i++) out[i] = orc_chal_sample(&c); chal_store(&c, s);
}
uint32_t orc_api_chal_grind(uint32_t *s, int bits) {
    orc_chal_t c; chal_load(&c, s); kb_t w = orc_chal_grind(&c, bits); chal_store(&c, s); return w;
}

void *orc_api_machine_new(const uint32_t *desc, uint64_t n) {
    orc_machine_t *m = (orc_machine_t *)calloc(1, sizeof *m);
    if (orc_machine_parse(m, desc, n)) { free(m); return NULL; }
    return m;
}
void orc_api_machine_free(void *m) { orc_machine_free((orc_machine_t *)m); free(m); }
int orc_api_machine_info(void *mh, int chip, int32_t *info /* prep,main,perm_ef,log_qd,nconstraints,local_only,scope */) {
    orc_machine_t *m = (orc_machine_t *)mh;
    if (chip < 0 || chip >= m->nchips) return -1;
    orc_chip_t *c = &m->chips[chip];
    info[0] = c->prep_width; info[1] = c->main_width; info[2] = c->perm_width_ef; info[3] = c->log_qd;
    info[4] = c->num_constraints; info[5] = c->local_only; info[6] = c->commit_scope;
    return 0;
}

void *orc_api_setup(void *mh, int num_queries, int pow_bits, int montgomery, const uint32_t *const *prep,
                    const uint64_t *prep_heights, uint32_t pc_start, const uint32_t *gcs, uint32_t *commit_out,
                    int log_blowup) {
    orc_machine_t *m = (orc_machine_t *)mh;
    orc_pk_t *pk = (orc_pk_t *)calloc(1, sizeof *pk);
    orc_config_t cfg = {num_queries, pow_bits, log_blowup, montgomery};
    size_t *h = (size_t *)calloc(m->nchips + 1, sizeof(size_t));
    for (int i = 0; i < m->nchips; i++) h[i] = prep_heights[i];
    int rc = orc_setup(pk, m, cfg, (const kb_t *const *)prep, h, pc_start, gcs);
    free(h);
    if (rc) { free(pk); return NULL; }
    memcpy(commit_out, pk->commit.v, 32);
    return pk;
}
void orc_api_pk_free(void *pk) { orc_pk_free((orc_pk_t *)pk); free(pk); }
void orc_api_pk_observe(void *pk, uint32_t *s) { orc_chal_t c; chal_load(&c, s); orc_pk_observe((orc_pk_t *)pk, &c); chal_store(&c, s); }

int orc_api_prove(void *pkh, int n, const int *chip_idx, const uint32_t *const *traces, const uint64_t *heights,
                  const uint32_t *pv, int npv, uint32_t *chal_state, uint8_t **out, uint64_t *len) {
    orc_pk_t *pk = (orc_pk_t *)pkh;
    orc_chal_t c; chal_load(&c, chal_state);
    size_t *h = (size_t *)malloc(sizeof(size_t) * (n + 1));
    for (int i = 0; i < n; i++) h[i] = heights[i];
    orc_proof_t p;
    int rc = orc_prove_shard(pk, n, chip_idx, (const kb_t *const *)traces, h, pv, npv, &c, &p);
    free(h);
    chal_store(&c, chal_state);
    if (rc && rc != -5) return rc;
    *len = orc_proof_serialize(&p, &pk->cfg, out);
    orc_proof_free(&p);
    return rc;
}
int orc_api_verify(void *pkh, const uint8_t *b, uint64_t n, uint32_t *chal_state) {
    orc_pk_t *pk = (orc_pk_t *)pkh;
    orc_proof_t p;
    if (orc_proof_deserialize(&p, &pk->cfg, b, n)) { orc_proof_free(&p); return -100; }
    orc_chal_t c; chal_load(&c, chal_state);
    int rc = orc_verify_shard(pk, &p, &c);
    chal_store(&c, chal_state);
    orc_proof_free(&p);
    return rc;
}
void orc_api_free_bytes(uint8_t *b) { free(b); }
