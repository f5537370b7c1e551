/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).
 *
 * Canonical proof bytes: bincode-1 (fixint, little-endian) layout of ShardProof
 * (crates/stark/src/types.rs:77-83; FriProof field order as used by
 * crates/recursion/circuit/src/fri.rs:43-66,411-465).  Vec => u64 length + items,
 * fixed arrays (digest [F;8], EF [F;4], septic digest [F;14]) => no length, usize => u64.
 * chip_ordering (a hashbrown::HashMap in the reference, iteration order nondeterministic)
 * is written sorted by index (canonical rule).  Field elements are written
 * canonical by default, Montgomery (x * 2^32 mod p) when cfg->montgomery_bytes.
 */
#include <stdlib.h>
#include "stark.h"

typedef struct { uint8_t *b; size_t n, cap; } wbuf_t;
static void wput(wbuf_t *w, const void *p, size_t n) {
    if (w->n + n > w->cap) { w->cap = (w->n + n) * 2 + 1024; w->b = (uint8_t *)realloc(w->b, w->cap); }
    memcpy(w->b + w->n, p, n); w->n += n;
}
static void wu64(wbuf_t *w, uint64_t v) { wput(w, &v, 8); }
static void wu32(wbuf_t *w, uint32_t v) { wput(w, &v, 4); }
static int g_mont;
static void wf(wbuf_t *w, kb_t x) { wu32(w, g_mont ? (uint32_t)(((uint64_t)x << 32) % KB_P) : x); }
static void wef(wbuf_t *w, ef_t e) { for (int i = 0; i < 4; i++) wf(w, e.c[i]); }
static void wdig(wbuf_t *w, digest_t d) { for (int i = 0; i < 8; i++) wf(w, d.v[i]); }
static void wefvec(wbuf_t *w, const ef_t *v, int n) { wu64(w, n); for (int i = 0; i < n; i++) wef(w, v[i]); }
static void wdigvec(wbuf_t *w, const digest_t *d, int n) { wu64(w, n); for (int i = 0; i < n; i++) wdig(w, d[i]); }

size_t orc_proof_serialize(const orc_proof_t *p, const orc_config_t *cfg, uint8_t **out) {
    wbuf_t w = {0, 0, 0};
    g_mont = cfg->montgomery_bytes;
    wdig(&w, p->main_commit); wdig(&w, p->perm_commit); wdig(&w, p->quot_commit);
    wu64(&w, p->nchips);
    for (int i = 0; i < p->nchips; i++) {
        const orc_chip_open_t *c = &p->chips[i];
        wefvec(&w, c->prep.local, c->prep.w); wefvec(&w, c->prep.next, c->prep.w);
        wefvec(&w, c->main.local, c->main.w); wefvec(&w, c->main.next, c->main.w);
        wefvec(&w, c->perm.local, c->perm.w); wefvec(&w, c->perm.next, c->perm.w);
        wu64(&w, c->nq);
        for (int j = 0; j < c->nq; j++) wefvec(&w, c->quot + 4 * j, 4);
        for (int j = 0; j < 14; j++) wf(&w, c->gcs[j]);
        wef(&w, c->lcs);
        wu64(&w, c->log_degree);
    }
    const orc_fri_t *f = &p->fri;
    wdigvec(&w, f->commits, f->ncommits);
    wu64(&w, f->nqueries);
    for (int q = 0; q < f->nqueries; q++) {
        const orc_query_t *qq = &f->queries[q];
        wu64(&w, qq->nrounds);
        for (int t = 0; t < qq->nrounds; t++) {
            const orc_batch_open_t *bo = &qq->input[t];
            wu64(&w, bo->nmats);
            for (int m = 0; m < bo->nmats; m++) {
                wu64(&w, bo->widths[m]);
                for (size_t c = 0; c < bo->widths[m]; c++) wf(&w, bo->vals[m][c]);
            }
            wdigvec(&w, bo->path, bo->path_len);
        }
        wu64(&w, qq->nsteps);
        for (int s = 0; s < qq->nsteps; s++) { wef(&w, qq->steps[s].sibling); wdigvec(&w, qq->steps[s].path, qq->steps[s].path_len); }
    }
    wef(&w, f->final_poly);
    wf(&w, f->pow_witness);
    wu64(&w, p->nchips);
    for (int i = 0; i < p->nchips; i++) {
        size_t l = strlen(p->ord_names[i]);
        wu64(&w, l); wput(&w, p->ord_names[i], l); wu64(&w, i);
    }
    wu64(&w, p->npv);
    for (int i = 0; i < p->npv; i++) wf(&w, p->pv[i]);
    *out = w.b;
    return w.n;
}

/* ------------------------------------------------------------------ reader */
typedef struct { const uint8_t *b; size_t n, p; int err; } rbuf_t;
static void rget(rbuf_t *r, void *d, size_t n) {
    if (r->p + n > r->n) { r->err = 1; memset(d, 0, n); return; }
    memcpy(d, r->b + r->p, n); r->p += n;
}
static uint64_t ru64(rbuf_t *r) { uint64_t v; rget(r, &v, 8); return v; }
static kb_t rf(rbuf_t *r) {
    uint32_t v; rget(r, &v, 4);
    if (v >= KB_P) r->err = 1;
    /* Montgomery -> canonical: v * 2^-32 */
    return g_mont ? kb_mul(v % KB_P, kb_inv(kb_from_u64(1ull << 32))) : v;
}
static ef_t ref(rbuf_t *r) { ef_t e; for (int i = 0; i < 4; i++) e.c[i] = rf(r); return e; }
static digest_t rdig(rbuf_t *r) { digest_t d; for (int i = 0; i < 8; i++) d.v[i] = rf(r); return d; }
static size_t rlen(rbuf_t *r, size_t max) { uint64_t v = ru64(r); if (v > max) { r->err = 1; return 0; } return (size_t)v; }
static ef_t *refvec(rbuf_t *r, int *n) {
    size_t l = rlen(r, 1 << 16); *n = (int)l;
    ef_t *v = (ef_t *)calloc(l + 1, sizeof(ef_t));
    for (size_t i = 0; i < l; i++) v[i] = ref(r);
    return v;
}
static digest_t *rdigvec(rbuf_t *r, int *n) {
    size_t l = rlen(r, 64); *n = (int)l;
    digest_t *d = (digest_t *)calloc(l + 1, sizeof(digest_t));
    for (size_t i = 0; i < l; i++) d[i] = rdig(r);
    return d;
}

int orc_proof_deserialize(orc_proof_t *p, const orc_config_t *cfg, const uint8_t *b, size_t n) {
    rbuf_t r = {b, n, 0, 0};
    memset(p, 0, sizeof *p);
    g_mont = cfg->montgomery_bytes;
    p->main_commit = rdig(&r); p->perm_commit = rdig(&r); p->quot_commit = rdig(&r);
    p->nchips = (int)rlen(&r, 256);
    p->chips = (orc_chip_open_t *)calloc(p->nchips + 1, sizeof(orc_chip_open_t));
    for (int i = 0; i < p->nchips && !r.err; i++) {
        orc_chip_open_t *c = &p->chips[i];
        int w2;
        c->prep.local = refvec(&r, &c->prep.w); c->prep.next = refvec(&r, &w2); if (w2 != c->prep.w) r.err = 1;
        c->main.local = refvec(&r, &c->main.w); c->main.next = refvec(&r, &w2); if (w2 != c->main.w) r.err = 1;
        c->perm.local = refvec(&r, &c->perm.w); c->perm.next = refvec(&r, &w2); if (w2 != c->perm.w) r.err = 1;
        c->nq = (int)rlen(&r, 16);
        c->quot = (ef_t *)calloc(4 * c->nq + 1, sizeof(ef_t));
        for (int j = 0; j < c->nq; j++) {
            int l; ef_t *v = refvec(&r, &l);
            if (l != 4) r.err = 1; else memcpy(c->quot + 4 * j, v, 4 * sizeof(ef_t));
            free(v);
        }
        for (int j = 0; j < 14; j++) c->gcs[j] = rf(&r);
        c->lcs = ref(&r);
        c->log_degree = (int)ru64(&r);
    }
    orc_fri_t *f = &p->fri;
    f->commits = rdigvec(&r, &f->ncommits);
    f->nqueries = (int)rlen(&r, 4096);
    f->queries = (orc_query_t *)calloc(f->nqueries + 1, sizeof(orc_query_t));
    for (int q = 0; q < f->nqueries && !r.err; q++) {
        orc_query_t *qq = &f->queries[q];
        qq->nrounds = (int)rlen(&r, 8);
        qq->input = (orc_batch_open_t *)calloc(qq->nrounds + 1, sizeof(orc_batch_open_t));
        for (int t = 0; t < qq->nrounds && !r.err; t++) {
            orc_batch_open_t *bo = &qq->input[t];
            bo->nmats = (int)rlen(&r, 256);
            bo->widths = (size_t *)calloc(bo->nmats + 1, sizeof(size_t));
            bo->vals = (kb_t **)calloc(bo->nmats + 1, sizeof(kb_t *));
            for (int m = 0; m < bo->nmats; m++) {
                bo->widths[m] = rlen(&r, 1 << 16);
                bo->vals[m] = (kb_t *)calloc(bo->widths[m] + 1, sizeof(kb_t));
                for (size_t c = 0; c < bo->widths[m]; c++) bo->vals[m][c] = rf(&r);
            }
            bo->path = rdigvec(&r, &bo->path_len);
        }
        qq->nsteps = (int)rlen(&r, 64);
        qq->steps = (orc_step_t *)calloc(qq->nsteps + 1, sizeof(orc_step_t));
        for (int s = 0; s < qq->nsteps && !r.err; s++) {
            qq->steps[s].sibling = ref(&r);
            qq->steps[s].path = rdigvec(&r, &qq->steps[s].path_len);
        }
    }
    f->final_poly = ref(&r);
    f->pow_witness = rf(&r);
    int nord = (int)rlen(&r, 256);
    if (nord != p->nchips) r.err = 1;
    p->ord_names = (char (*)[64])calloc(nord + 1, 64);
    for (int i = 0; i < nord && !r.err; i++) {
        size_t l = rlen(&r, 63);
        rget(&r, p->ord_names[i], l);
        if (ru64(&r) != (uint64_t)i) r.err = 1;
    }
    p->npv = (int)rlen(&r, 1 << 12);
    p->pv = (kb_t *)calloc(p->npv + 1, sizeof(kb_t));
    for (int i = 0; i < p->npv; i++) p->pv[i] = rf(&r);
    if (r.p != r.n) r.err = 1;
    return r.err ? -1 : 0;
}

/* bincode-1 of a BTreeMap<[F; 8], usize> (the prover's vk map, crates/prover/src/shapes.rs:370-379,
 * loaded at crates/prover/src/lib.rs:232): u64 length, then per entry the digest with no length
 * prefix and the usize as u64 — the same field/length conventions as the proof serializer above. */
size_t orc_serialize_digest_map(const uint32_t *keys, const uint64_t *vals, uint64_t n, int montgomery, uint8_t **out) {
    wbuf_t w = {0, 0, 0};
    g_mont = montgomery;
    wu64(&w, n);
    for (uint64_t i = 0; i < n; i++) {
        digest_t d; memcpy(d.v, keys + 8 * i, 32);
        wdig(&w, d); wu64(&w, vals[i]);
    }
    *out = w.b;
    return w.n;
}
