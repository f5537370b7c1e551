/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).
 *
 * CPU restatement of the per-shard prover the reference runs:
 *   CpuProver::commit  crates/stark/src/prover.rs:258-292
 *   CpuProver::open    crates/stark/src/prover.rs:298-653
 *   StarkMachine::setup crates/stark/src/machine.rs:332-439
 *   generate_permutation_trace crates/stark/src/permutation.rs:102-196
 *   quotient_values    crates/stark/src/quotient.rs:19-171
 * and of the Plonky3 TwoAdicFriPcs::open / FRI prover whose semantics are pinned by the
 * verifier restatement crates/recursion/circuit/src/fri.rs:34-405 (not vendored: Plonky3 fork
 * ProjectZKM/Plonky3@faa24ca4597eebeecbf71b194b71c7d1a99b3f01).
 */
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include "stark.h"

/* ORC_TIMING=1: per-phase wall times of orc_prove_shard on stderr (profiling the CPU baseline) */
static double t_last;
static void phase(const char *name) {
    static int on = -1;
    if (on < 0) on = getenv("ORC_TIMING") != NULL;
    const double t = omp_get_wtime();
    if (on && name) fprintf(stderr, "orc %-14s %8.3f s\n", name, t - t_last);
    t_last = t;
}

/* ---------------- constraint evaluators (base = prover, ext = verifier) ---------------- */
static inline ef_t ef_mul_kb(ef_t a, kb_t b) { return ef_mul_base(a, b); }
#define FN eval_chip_base
#define V kb_t
#define VADD kb_add
#define VSUB kb_sub
#define VMUL kb_mul
#define VNEG kb_neg
#define VCONST(x) (x)
#define EF_MUL_V ef_mul_kb
#define APPLY_VPC orc_vpc_apply
#include "air_eval.inc"
#undef FN
#undef V
#undef VADD
#undef VSUB
#undef VMUL
#undef VNEG
#undef VCONST
#undef EF_MUL_V
#undef APPLY_VPC
#define FN eval_chip_ext
#define V ef_t
#define VADD ef_add
#define VSUB ef_sub
#define VMUL ef_mul
#define VNEG ef_neg
#define VCONST(x) ef_from_base(x)
#define EF_MUL_V ef_mul
#define APPLY_VPC orc_vpc_apply_ef
#include "air_eval.inc"

/* ------------------------------------------------------------------ helpers */
static const kb_t CSX[7] = CURVE_START_X, CSY[7] = CURVE_START_Y;

typedef struct { int idx; size_t h; const char *name; } ord_t;
static int cmp_ord(const void *a, const void *b) {
    const ord_t *x = (const ord_t *)a, *y = (const ord_t *)b;
    if (x->h != y->h) return x->h > y->h ? -1 : 1;
    return strcmp(x->name, y->name);
}

static kb_t *lde_of(const kb_t *evals, size_t h, size_t w, kb_t shift, int log_blowup) {
    kb_t *out = (kb_t *)malloc(sizeof(kb_t) * (h << log_blowup) * (w ? w : 1));
    if (w) orc_coset_lde_bitrev(evals, h, w, log_blowup, shift, out);
    return out;
}

/* Montgomery's batch inversion, in independent chunks (one field inversion per chunk) so the
 * chunks run in parallel; every element must be non-zero. */
#define BI_CHUNK 4096
static void batch_inverse(ef_t *v, size_t n) {
#pragma omp parallel for schedule(static)
    for (size_t c0 = 0; c0 < n; c0 += BI_CHUNK) {
        size_t m = n - c0 < BI_CHUNK ? n - c0 : BI_CHUNK;
        ef_t pre[BI_CHUNK], acc = ef_one();
        for (size_t i = 0; i < m; i++) { pre[i] = acc; acc = ef_mul(acc, v[c0 + i]); }
        ef_t inv = ef_inv(acc);
        for (size_t i = m; i-- > 0;) { ef_t t = ef_mul(inv, pre[i]); inv = ef_mul(inv, v[c0 + i]); v[c0 + i] = t; }
    }
}
static void batch_inverse_kb(kb_t *v, size_t n) {
#pragma omp parallel for schedule(static)
    for (size_t c0 = 0; c0 < n; c0 += BI_CHUNK) {
        size_t m = n - c0 < BI_CHUNK ? n - c0 : BI_CHUNK;
        kb_t pre[BI_CHUNK], acc = 1;
        for (size_t i = 0; i < m; i++) { pre[i] = acc; acc = kb_mul(acc, v[c0 + i]); }
        kb_t inv = kb_inv(acc);
        for (size_t i = m; i-- > 0;) { kb_t t = kb_mul(inv, pre[i]); inv = kb_mul(inv, v[c0 + i]); v[c0 + i] = t; }
    }
}

/* pw[k] = g^k for k < n (parallel: each chunk starts from its own power) */
static kb_t *powers(kb_t g, size_t n) {
    kb_t *pw = (kb_t *)malloc(sizeof(kb_t) * (n ? n : 1));
#pragma omp parallel for schedule(static)
    for (size_t c0 = 0; c0 < n; c0 += BI_CHUNK) {
        kb_t x = kb_pow(g, c0);
        for (size_t i = c0; i < n && i < c0 + BI_CHUNK; i++) { pw[i] = x; x = kb_mul(x, g); }
    }
    return pw;
}

/* opened value of every column of a committed LDE (bit-reversed, 2^lb * n rows) at z, by
 * barycentric interpolation over the low coset D = GENERATOR * H_n: its first n rows, where row r
 * holds p(3 w_n^{rev_n(r)}).  With x = z / 3:
 *     p(z) = (x^n - 1) / n * sum_j p(3 w^j) * w^j / (x - w^j). */
static void open_matrix_at(const orc_mat_t *lde, int log_blowup, ef_t z, ef_t *out) {
    size_t H = lde->height, n = H >> log_blowup, w = lde->width;
    int logn = log2_exact(n);
    ef_t x = ef_mul_base(z, kb_inv(KB_GENERATOR));
    kb_t *om = powers(kb_two_adic_gen(logn), n);
    ef_t *wt = (ef_t *)malloc(sizeof(ef_t) * n);
#pragma omp parallel for schedule(static)
    for (size_t j = 0; j < n; j++) wt[j] = ef_sub(x, ef_from_base(om[j]));
    batch_inverse(wt, n);
#pragma omp parallel for schedule(static)
    for (size_t j = 0; j < n; j++) wt[j] = ef_mul_base(wt[j], om[j]);
    ef_t pre = ef_mul_base(ef_sub(ef_pow(x, n), ef_one()), kb_inv((kb_t)(n % KB_P)));
    /* rows in storage order (row r holds point j = rev(r)), every column accumulated per row: the
     * matrix streams once; per-thread partial sums are added in thread order */
    int nt = omp_get_max_threads();
    ef_t *part = (ef_t *)calloc((size_t)nt * (w ? w : 1), sizeof(ef_t));
#pragma omp parallel
    {
        ef_t *acc = part + (size_t)omp_get_thread_num() * w;
#pragma omp for schedule(static)
        for (size_t r = 0; r < n; r++) {
            const ef_t wr = wt[rev_bits((uint32_t)r, logn)];
            const kb_t *row = lde->data + r * w;
            for (size_t c = 0; c < w; c++) acc[c] = ef_add(acc[c], ef_mul_base(wr, row[c]));
        }
    }
    for (size_t c = 0; c < w; c++) {
        ef_t acc = ef_zero();
        for (int t = 0; t < nt; t++) acc = ef_add(acc, part[(size_t)t * w + c]);
        out[c] = ef_mul(pre, acc);
    }
    free(part);
    free(wt);
    free(om);
}

/* ------------------------------------------------------------------- setup */
int orc_setup(orc_pk_t *pk, const orc_machine_t *m, orc_config_t cfg, const kb_t *const *prep_traces,
              const size_t *prep_heights, kb_t pc_start, const kb_t *gcs) {
    memset(pk, 0, sizeof *pk);
    pk->m = m;
    pk->cfg = cfg;
    pk->pc_start = pc_start;
    memcpy(pk->gcs, gcs, sizeof pk->gcs);
    ord_t *o = (ord_t *)malloc(sizeof(ord_t) * (m->nchips + 1));
    int n = 0;
    for (int c = 0; c < m->nchips; c++)
        if (m->chips[c].prep_width > 0) { o[n].idx = c; o[n].h = prep_heights[c]; o[n].name = m->chips[c].name; n++; }
    if (n == 0) { free(o); return -1; } /* Plonky3 MerkleTree::new panics on an empty batch */
    qsort(o, n, sizeof(ord_t), cmp_ord);
    pk->ntraces = n;
    pk->trace_chip = (int *)malloc(sizeof(int) * n);
    pk->traces = (kb_t **)malloc(sizeof(kb_t *) * n);
    pk->heights = (size_t *)malloc(sizeof(size_t) * n);
    orc_mat_t *mats = (orc_mat_t *)malloc(sizeof(orc_mat_t) * n);
    for (int i = 0; i < n; i++) {
        int c = o[i].idx;
        size_t h = o[i].h, w = m->chips[c].prep_width;
        pk->trace_chip[i] = c;
        pk->heights[i] = h;
        pk->traces[i] = (kb_t *)malloc(sizeof(kb_t) * h * w);
        memcpy(pk->traces[i], prep_traces[c], sizeof(kb_t) * h * w);
        mats[i].data = lde_of(pk->traces[i], h, w, KB_GENERATOR, cfg.log_blowup);
        mats[i].height = h << cfg.log_blowup;
        mats[i].width = w;
    }
    orc_tree_build(&pk->tree, mats, n, 1);
    pk->commit = orc_tree_root(&pk->tree);
    free(o);
    return 0;
}

void orc_pk_free(orc_pk_t *pk) {
    orc_tree_free(&pk->tree);
    for (int i = 0; i < pk->ntraces; i++) free(pk->traces[i]);
    free(pk->traces); free(pk->heights); free(pk->trace_chip);
    memset(pk, 0, sizeof *pk);
}

/* StarkProvingKey::observe_into, crates/stark/src/machine.rs:77-85 */
void orc_pk_observe(const orc_pk_t *pk, orc_chal_t *ch) {
    orc_chal_observe_digest(ch, pk->commit);
    orc_chal_observe(ch, pk->pc_start);
    orc_chal_observe_slice(ch, pk->gcs, 14);
    orc_chal_observe(ch, 0);
}

static int pk_index_of_chip(const orc_pk_t *pk, int chip) {
    for (int i = 0; i < pk->ntraces; i++) if (pk->trace_chip[i] == chip) return i;
    return -1;
}

/* ------------------------------------------------------------ permutation trace */
static void gen_perm_trace(const orc_chip_t *ch, const kb_t *prep, const kb_t *main, size_t h,
                           ef_t alpha, ef_t beta, ef_t *perm /* h x pw */, ef_t *lcs) {
    int pw = ch->perm_width_ef;
    *lcs = ef_zero();
    if (!pw) return;
    int batch = 1 << ch->log_qd, nb = pw - 1;
    const int nl = ch->nlocal;
    size_t W = ch->main_width, PWd = ch->prep_width;
    /* rows in chunks: every lookup denominator of the chunk inverted with one field inversion */
    const size_t RB = 256;
    ef_t bpw[256];
    bpw[0] = beta;
    for (int v = 1; v < 256; v++) bpw[v] = ef_mul(bpw[v - 1], beta);
#pragma omp parallel for schedule(static)
    for (size_t r0 = 0; r0 < h; r0 += RB) {
        const size_t rn = h - r0 < RB ? h - r0 : RB;
        ef_t *d = (ef_t *)malloc(sizeof(ef_t) * rn * nl), *pre = (ef_t *)malloc(sizeof(ef_t) * rn * nl);
        kb_t *mu = (kb_t *)malloc(sizeof(kb_t) * rn * nl);
        for (size_t r = 0; r < rn; r++) {
            const kb_t *ml = main + (r0 + r) * W;
            const kb_t *pl = prep ? prep + (r0 + r) * PWd : NULL;
            for (int i = 0; i < nl; i++) {
                const orc_lookup_t *lk = &ch->local[i];
                ef_t x = ef_add(alpha, ef_from_base(lk->kind));
                for (int v = 0; v < lk->nvalues && v < 256; v++)
                    x = ef_add(x, ef_mul_base(bpw[v], orc_vpc_apply(&lk->values[v], pl, ml)));
                kb_t m = orc_vpc_apply(&lk->mult, pl, ml);
                d[r * nl + i] = x;
                mu[r * nl + i] = lk->is_send ? m : kb_neg(m);
            }
        }
        const size_t k = rn * nl;
        ef_t acc = ef_one();
        for (size_t j = 0; j < k; j++) { pre[j] = acc; acc = ef_mul(acc, d[j]); }
        ef_t inv = ef_inv(acc);
        for (size_t j = k; j-- > 0;) { ef_t t = ef_mul(inv, pre[j]); inv = ef_mul(inv, d[j]); d[j] = t; }
        for (size_t r = 0; r < rn; r++)
            for (int b = 0; b < nb; b++) {
                ef_t sum = ef_zero();
                for (int i = b * batch; i < nl && i < (b + 1) * batch; i++)
                    sum = ef_add(sum, ef_mul_base(d[r * nl + i], mu[r * nl + i]));
                perm[(r0 + r) * pw + b] = sum;
            }
        free(d); free(pre); free(mu);
    }
    ef_t run = ef_zero();
    for (size_t r = 0; r < h; r++) {
        for (int b = 0; b < nb; b++) run = ef_add(run, perm[r * pw + b]);
        perm[r * pw + nb] = run;
    }
    *lcs = run;
}

/* ------------------------------------------------------------------- prover */
typedef struct { int round, mat; int npts; ef_t pts[2]; ef_t *vals[2]; } open_req_t;

int orc_prove_shard(const orc_pk_t *pk, int n, const int *chip_idx, const kb_t *const *traces,
                    const size_t *heights, const kb_t *pv, int npv, orc_chal_t *ch, orc_proof_t *out) {
    const orc_machine_t *m = pk->m;
    const int lb = pk->cfg.log_blowup;
    memset(out, 0, sizeof *out);
    phase(NULL);
    /* ---- commit (prover.rs:258-292): sort by (height desc, name) ---- */
    ord_t *o = (ord_t *)malloc(sizeof(ord_t) * n);
    for (int i = 0; i < n; i++) { o[i].idx = i; o[i].h = heights[i]; o[i].name = m->chips[chip_idx[i]].name; }
    qsort(o, n, sizeof(ord_t), cmp_ord);
    const orc_chip_t **chips = (const orc_chip_t **)malloc(sizeof(void *) * n);
    const kb_t **tr = (const kb_t **)malloc(sizeof(void *) * n);
    size_t *hs = (size_t *)malloc(sizeof(size_t) * n);
    int *cidx = (int *)malloc(sizeof(int) * n);
    orc_mat_t *main_mats = (orc_mat_t *)malloc(sizeof(orc_mat_t) * n);
    for (int i = 0; i < n; i++) {
        cidx[i] = chip_idx[o[i].idx];
        chips[i] = &m->chips[cidx[i]];
        tr[i] = traces[o[i].idx];
        hs[i] = heights[o[i].idx];
        if (chips[i]->log_qd > lb) { fprintf(stderr, "oracle: log_qd > log_blowup unsupported\n"); return -1; }
        main_mats[i].data = lde_of(tr[i], hs[i], chips[i]->main_width, KB_GENERATOR, lb);
        main_mats[i].height = hs[i] << lb;
        main_mats[i].width = chips[i]->main_width;
    }
    phase("main_lde");
    orc_tree_t main_tree;
    orc_tree_build(&main_tree, main_mats, n, 1);
    out->main_commit = orc_tree_root(&main_tree);
    out->nchips = n;
    out->ord_names = (char (*)[64])calloc(n, 64);
    for (int i = 0; i < n; i++) strcpy(out->ord_names[i], chips[i]->name);
    out->npv = npv;
    out->pv = (kb_t *)malloc(sizeof(kb_t) * (npv + 1));
    memcpy(out->pv, pv, sizeof(kb_t) * npv);

    phase("main_commit");
    /* ---- open (prover.rs:298-653) ---- */
    orc_chal_observe_slice(ch, pv, m->num_pv);
    orc_chal_observe_digest(ch, out->main_commit);
    ef_t perm_ch[2];
    perm_ch[0] = orc_chal_sample_ef(ch);
    perm_ch[1] = orc_chal_sample_ef(ch);

    out->chips = (orc_chip_open_t *)calloc(n, sizeof(orc_chip_open_t));
    kb_t **perm_flat = (kb_t **)malloc(sizeof(kb_t *) * n);
    orc_mat_t *perm_mats = (orc_mat_t *)malloc(sizeof(orc_mat_t) * n);
    for (int i = 0; i < n; i++) {
        const orc_chip_t *c = chips[i];
        int pki = pk_index_of_chip(pk, cidx[i]);
        const kb_t *prep = pki >= 0 ? pk->traces[pki] : NULL;
        if (pki >= 0 && pk->heights[pki] != hs[i]) { fprintf(stderr, "oracle: prep/main height mismatch\n"); return -2; }
        int pw = c->perm_width_ef;
        ef_t *perm = (ef_t *)calloc(hs[i] * (pw ? pw : 1), sizeof(ef_t));
        gen_perm_trace(c, prep, tr[i], hs[i], perm_ch[0], perm_ch[1], perm, &out->chips[i].lcs);
        if (c->commit_scope == 1) {
            const kb_t *last = tr[i] + (hs[i] - 1) * c->main_width + c->main_width - 14;
            memcpy(out->chips[i].gcs, last, 14 * sizeof(kb_t));
        } else {
            memcpy(out->chips[i].gcs, CSX, 7 * sizeof(kb_t));
            memcpy(out->chips[i].gcs + 7, CSY, 7 * sizeof(kb_t));
        }
        perm_flat[i] = (kb_t *)malloc(sizeof(kb_t) * hs[i] * 4 * (pw ? pw : 1));
        memcpy(perm_flat[i], perm, sizeof(kb_t) * hs[i] * 4 * pw);
        free(perm);
        perm_mats[i].data = lde_of(perm_flat[i], hs[i], 4 * pw, KB_GENERATOR, lb);
        perm_mats[i].height = hs[i] << lb;
        perm_mats[i].width = 4 * pw;
        out->chips[i].log_degree = log2_exact(hs[i]);
    }
    phase("perm_trace_lde");
    orc_tree_t perm_tree;
    orc_tree_build(&perm_tree, perm_mats, n, 1);
    out->perm_commit = orc_tree_root(&perm_tree);
    orc_chal_observe_digest(ch, out->perm_commit);
    for (int i = 0; i < n; i++) {
        orc_chal_observe_ef(ch, out->chips[i].lcs);
        orc_chal_observe_slice(ch, out->chips[i].gcs, 14);
    }
    ef_t alpha = orc_chal_sample_ef(ch);

    phase("perm");
    /* ---- quotient values (quotient.rs) + split/commit (prover.rs:476-498) ---- */
    int nchunks = 0;
    for (int i = 0; i < n; i++) nchunks += 1 << chips[i]->log_qd;
    orc_mat_t *q_mats = (orc_mat_t *)malloc(sizeof(orc_mat_t) * nchunks);
    int qi = 0;
    for (int i = 0; i < n; i++) {
        const orc_chip_t *c = chips[i];
        size_t N = hs[i];
        int logN = log2_exact(N), lqd = c->log_qd;
        size_t Q = N << lqd;
        int logQ = logN + lqd;
        int pki = pk_index_of_chip(pk, cidx[i]);
        const orc_mat_t *prep_lde = pki >= 0 ? &pk->tree.mats[pki] : NULL;
        const orc_mat_t *main_lde = &main_tree.mats[i];
        const orc_mat_t *perm_lde = &perm_tree.mats[i];
        int nc = c->num_constraints;
        ef_t *pows = (ef_t *)malloc(sizeof(ef_t) * (nc + 1));
        ef_t a = ef_one();
        for (int k = nc - 1; k >= 0; k--) { pows[k] = a; a = ef_mul(a, alpha); }
        kb_t wQ = kb_two_adic_gen(logQ), wN_inv = kb_inv(kb_two_adic_gen(logN));
        ef_t *q = (ef_t *)malloc(sizeof(ef_t) * Q);
        size_t step = (size_t)1 << lqd;
        int pw = c->perm_width_ef;
        /* selectors on the quotient coset 3 * H_Q (zerofier_coset.rs:22-71, quotient.rs:42): the
         * three denominators of every point inverted in batches */
        kb_t *xs = powers(wQ, Q), *d1 = (kb_t *)malloc(sizeof(kb_t) * Q), *d2 = (kb_t *)malloc(sizeof(kb_t) * Q),
             *d3 = (kb_t *)malloc(sizeof(kb_t) * Q);
#pragma omp parallel for schedule(static)
        for (size_t k = 0; k < Q; k++) {
            xs[k] = kb_mul(KB_GENERATOR, xs[k]);
            d1[k] = kb_sub(xs[k], 1);
            d2[k] = kb_sub(xs[k], wN_inv);
            d3[k] = kb_sub(kb_pow(xs[k], N), 1);
        }
        batch_inverse_kb(d1, Q);
        batch_inverse_kb(d2, Q);
        batch_inverse_kb(d3, Q);
#pragma omp parallel for schedule(static)
        for (size_t k = 0; k < Q; k++) {
            size_t rl = rev_bits((uint32_t)k, logQ), rn = rev_bits((uint32_t)((k + step) % Q), logQ);
            kb_t x = xs[k];
            kb_t zh = kb_sub(kb_pow(x, N), 1);
            kb_t is_first = kb_mul(zh, d1[k]);
            kb_t is_last = kb_mul(zh, d2[k]);
            kb_t is_trans = kb_sub(x, wN_inv);
            kb_t invz = d3[k];
            const kb_t *pl = prep_lde ? prep_lde->data + rl * prep_lde->width : NULL;
            const kb_t *pn = prep_lde ? prep_lde->data + rn * prep_lde->width : NULL;
            const kb_t *ml = main_lde->data + rl * main_lde->width, *mn = main_lde->data + rn * main_lde->width;
            ef_t perm_l[pw > 0 ? pw : 1], perm_n[pw > 0 ? pw : 1];
            for (int b = 0; b < pw; b++)
                for (int e = 0; e < 4; e++) {
                    perm_l[b].c[e] = perm_lde->data[rl * perm_lde->width + 4 * b + e];
                    perm_n[b].c[e] = perm_lde->data[rn * perm_lde->width + 4 * b + e];
                }
            ef_t acc = eval_chip_base(c, pl, pn, ml, mn, perm_l, perm_n, is_first, is_last, is_trans, pv,
                                      perm_ch[0], perm_ch[1], out->chips[i].lcs, out->chips[i].gcs, pows);
            q[k] = ef_mul_base(acc, invz);
        }
        free(pows); free(xs); free(d1); free(d2); free(d3);
        /* split_evals: chunk j takes rows k = j (mod 2^lqd); domain shift 3 * wQ^j, commit shift wQ^-j */
        for (int j = 0; j < (1 << lqd); j++) {
            kb_t *chunk = (kb_t *)malloc(sizeof(kb_t) * N * 4);
            for (size_t r = 0; r < N; r++)
                for (int e = 0; e < 4; e++) chunk[r * 4 + e] = q[r * step + j].c[e];
            kb_t shift = kb_inv(kb_pow(wQ, (uint64_t)j));
            q_mats[qi].data = lde_of(chunk, N, 4, shift, lb);
            q_mats[qi].height = N << lb;
            q_mats[qi].width = 4;
            free(chunk);
            qi++;
        }
        free(q);
    }
    orc_tree_t q_tree;
    orc_tree_build(&q_tree, q_mats, nchunks, 1);
    out->quot_commit = orc_tree_root(&q_tree);
    orc_chal_observe_digest(ch, out->quot_commit);
    ef_t zeta = orc_chal_sample_ef(ch);

    phase("quotient");
    /* ---- opening points (prover.rs:503-544) and values ---- */
    orc_tree_t *trees[4] = {(orc_tree_t *)&pk->tree, &main_tree, &perm_tree, &q_tree};
    int nreq = pk->ntraces + 2 * n + nchunks;
    open_req_t *req = (open_req_t *)calloc(nreq, sizeof(open_req_t));
    int r = 0;
    for (int t = 0; t < pk->ntraces; t++, r++) {
        const orc_chip_t *c = &m->chips[pk->trace_chip[t]];
        req[r].round = 0; req[r].mat = t; req[r].pts[0] = zeta; req[r].npts = 1;
        if (!c->local_only) { req[r].pts[1] = ef_mul_base(zeta, kb_two_adic_gen(log2_exact(pk->heights[t]))); req[r].npts = 2; }
    }
    for (int i = 0; i < n; i++, r++) {
        req[r].round = 1; req[r].mat = i; req[r].pts[0] = zeta; req[r].npts = 1;
        if (!chips[i]->local_only) { req[r].pts[1] = ef_mul_base(zeta, kb_two_adic_gen(log2_exact(hs[i]))); req[r].npts = 2; }
    }
    for (int i = 0; i < n; i++, r++) {
        req[r].round = 2; req[r].mat = i; req[r].pts[0] = zeta; req[r].npts = 2;
        req[r].pts[1] = ef_mul_base(zeta, kb_two_adic_gen(log2_exact(hs[i])));
    }
    for (int j = 0; j < nchunks; j++, r++) { req[r].round = 3; req[r].mat = j; req[r].pts[0] = zeta; req[r].npts = 1; }
    for (r = 0; r < nreq; r++) {
        const orc_mat_t *mm = &trees[req[r].round]->mats[req[r].mat];
        for (int p = 0; p < req[r].npts; p++) {
            req[r].vals[p] = (ef_t *)malloc(sizeof(ef_t) * (mm->width + 1));
            open_matrix_at(mm, lb, req[r].pts[p], req[r].vals[p]);
        }
    }

    phase("open_values");
    /* ---- TwoAdicFriPcs::open: alpha, reduced openings (fri.rs:71-215 semantics) ---- */
    ef_t fri_alpha = orc_chal_sample_ef(ch);
    int log_max = 0;
    for (int t = 0; t < 4; t++) if (trees[t]->log_max_height > log_max) log_max = trees[t]->log_max_height;
    ef_t *ro[32] = {0};
    int pow_cnt[32] = {0};
    ef_t *apow = NULL; int napow = 0;
    for (r = 0; r < nreq; r++) {
        const orc_mat_t *mm = &trees[req[r].round]->mats[req[r].mat];
        int lh = log2_exact(mm->height);
        size_t H = mm->height, w = mm->width;
        if (!ro[lh]) ro[lh] = (ef_t *)calloc(H, sizeof(ef_t));
        kb_t wH = kb_two_adic_gen(lh);
        for (int p = 0; p < req[r].npts; p++) {
            int base = pow_cnt[lh];
            if (napow < base + (int)w + 1) {
                apow = (ef_t *)realloc(apow, sizeof(ef_t) * (base + w + 1));
                for (int k = napow; k < base + (int)w + 1; k++) apow[k] = k ? ef_mul(apow[k - 1], fri_alpha) : ef_one();
                napow = base + (int)w + 1;
            }
            ef_t z = req[r].pts[p];
            ef_t *den = (ef_t *)malloc(sizeof(ef_t) * H);
            kb_t *xp = powers(wH, H);
#pragma omp parallel for schedule(static)
            for (size_t i = 0; i < H; i++) {
                kb_t x = kb_mul(KB_GENERATOR, xp[rev_bits((uint32_t)i, lh)]);
                den[i] = ef_sub(z, ef_from_base(x));
            }
            free(xp);
            batch_inverse(den, H);
            /* sum_c alpha^c (p_c(z) - x_c) = B - sum_c alpha^c x_c with B = sum_c alpha^c p_c(z) */
            ef_t B = ef_zero();
            for (size_t c = 0; c < w; c++) B = ef_add(B, ef_mul(apow[base + c], req[r].vals[p][c]));
#pragma omp parallel for schedule(static)
            for (size_t i = 0; i < H; i++) {
                ef_t acc = ef_zero();
                const kb_t *row = mm->data + i * w;
                for (size_t c = 0; c < w; c++) acc = ef_add(acc, ef_mul_base(apow[base + c], row[c]));
                ro[lh][i] = ef_add(ro[lh][i], ef_mul(ef_sub(B, acc), den[i]));
            }
            free(den);
            pow_cnt[lh] += (int)w;
        }
    }
    free(apow);

    phase("fri_reduce");
    /* ---- FRI commit phase (fri.rs:34-69, 247-361 semantics) ---- */
    orc_fri_t *fri = &out->fri;
    int nrounds = log_max - lb;
    fri->ncommits = nrounds;
    fri->commits = (digest_t *)malloc(sizeof(digest_t) * (nrounds + 1));
    orc_tree_t *ftrees = (orc_tree_t *)calloc(nrounds + 1, sizeof(orc_tree_t));
    size_t cur_n = (size_t)1 << log_max;
    ef_t *cur = (ef_t *)malloc(sizeof(ef_t) * cur_n);
    memcpy(cur, ro[log_max], sizeof(ef_t) * cur_n);
    kb_t half = kb_halve(1);
    for (int rd = 0; rd < nrounds; rd++) {
        int lf = log_max - 1 - rd;
        size_t h = cur_n >> 1;
        orc_mat_t *leaf = (orc_mat_t *)malloc(sizeof(orc_mat_t));
        kb_t *ld = (kb_t *)malloc(sizeof(kb_t) * h * 8);
        memcpy(ld, cur, sizeof(ef_t) * cur_n);
        leaf->data = ld; leaf->height = h; leaf->width = 8;
        orc_tree_build(&ftrees[rd], leaf, 1, 1);
        fri->commits[rd] = orc_tree_root(&ftrees[rd]);
        orc_chal_observe_digest(ch, fri->commits[rd]);
        ef_t beta = orc_chal_sample_ef(ch);
        ef_t hb = ef_mul_base(beta, half);
        kb_t ginv = kb_inv(kb_two_adic_gen(lf + 1));
        ef_t *nx = (ef_t *)malloc(sizeof(ef_t) * h);
#pragma omp parallel for schedule(static)
        for (size_t i = 0; i < h; i++) {
            ef_t pw = ef_mul_base(hb, kb_pow(ginv, rev_bits((uint32_t)i, lf)));
            ef_t lo = cur[2 * i], hi = cur[2 * i + 1];
            nx[i] = ef_add(ef_mul(ef_add_base(pw, half), lo), ef_mul(ef_sub(ef_from_base(half), pw), hi));
        }
        free(cur);
        cur = nx; cur_n = h;
        if (ro[lf]) {
            ef_t b2 = ef_mul(beta, beta);
            for (size_t i = 0; i < h; i++) cur[i] = ef_add(cur[i], ef_mul(b2, ro[lf][i]));
        }
    }
    fri->final_poly = cur[0];
    int final_ok = 1;
    for (size_t i = 1; i < cur_n; i++) final_ok &= ef_eq(cur[i], cur[0]);
    free(cur);
    orc_chal_observe_ef(ch, fri->final_poly);
    fri->pow_witness = orc_chal_grind(ch, pk->cfg.pow_bits);

    phase("fri_commit");
    /* ---- queries ---- */
    fri->nqueries = pk->cfg.num_queries;
    fri->queries = (orc_query_t *)calloc(fri->nqueries, sizeof(orc_query_t));
    for (int qn = 0; qn < fri->nqueries; qn++) {
        size_t index = orc_chal_sample_bits(ch, log_max);
        orc_query_t *qq = &fri->queries[qn];
        qq->nrounds = 4;
        qq->input = (orc_batch_open_t *)calloc(4, sizeof(orc_batch_open_t));
        for (int t = 0; t < 4; t++) {
            orc_tree_t *tt = trees[t];
            orc_batch_open_t *bo = &qq->input[t];
            size_t ri = index >> (log_max - tt->log_max_height);
            const kb_t **rows = (const kb_t **)malloc(sizeof(void *) * tt->nmats);
            bo->nmats = tt->nmats;
            bo->path_len = tt->log_max_height;
            bo->path = (digest_t *)malloc(sizeof(digest_t) * (bo->path_len + 1));
            orc_tree_open(tt, ri, rows, bo->path);
            bo->widths = (size_t *)malloc(sizeof(size_t) * tt->nmats);
            bo->vals = (kb_t **)malloc(sizeof(kb_t *) * tt->nmats);
            for (int mi = 0; mi < tt->nmats; mi++) {
                bo->widths[mi] = tt->mats[mi].width;
                bo->vals[mi] = (kb_t *)malloc(sizeof(kb_t) * (bo->widths[mi] + 1));
                memcpy(bo->vals[mi], rows[mi], sizeof(kb_t) * bo->widths[mi]);
            }
            free(rows);
        }
        qq->nsteps = nrounds;
        qq->steps = (orc_step_t *)calloc(nrounds + 1, sizeof(orc_step_t));
        for (int rd = 0; rd < nrounds; rd++) {
            size_t idx_i = index >> rd, pair = idx_i >> 1;
            const kb_t *row;
            orc_step_t *st = &qq->steps[rd];
            st->path_len = ftrees[rd].log_max_height;
            st->path = (digest_t *)malloc(sizeof(digest_t) * (st->path_len + 1));
            orc_tree_open(&ftrees[rd], pair, &row, st->path);
            memcpy(st->sibling.c, row + 4 * ((idx_i ^ 1) & 1), sizeof(ef_t));
        }
    }

    phase("queries");
    /* ---- opened values (prover.rs:558-640) ---- */
    r = 0;
    for (int i = 0; i < n; i++) {
        orc_chip_open_t *co = &out->chips[i];
        int pki = pk_index_of_chip(pk, cidx[i]);
        int w = chips[i]->prep_width;
        co->prep.w = pki >= 0 ? w : 0;
        co->prep.local = (ef_t *)calloc(co->prep.w + 1, sizeof(ef_t));
        co->prep.next = (ef_t *)calloc(co->prep.w + 1, sizeof(ef_t));
        if (pki >= 0) {
            open_req_t *pr = &req[pki];
            memcpy(co->prep.local, pr->vals[0], sizeof(ef_t) * w);
            if (pr->npts == 2) memcpy(co->prep.next, pr->vals[1], sizeof(ef_t) * w);
        }
        open_req_t *mr = &req[pk->ntraces + i];
        co->main.w = chips[i]->main_width;
        co->main.local = (ef_t *)calloc(co->main.w + 1, sizeof(ef_t));
        co->main.next = (ef_t *)calloc(co->main.w + 1, sizeof(ef_t));
        memcpy(co->main.local, mr->vals[0], sizeof(ef_t) * co->main.w);
        if (mr->npts == 2) memcpy(co->main.next, mr->vals[1], sizeof(ef_t) * co->main.w);
        open_req_t *pr2 = &req[pk->ntraces + n + i];
        co->perm.w = 4 * chips[i]->perm_width_ef;
        co->perm.local = (ef_t *)calloc(co->perm.w + 1, sizeof(ef_t));
        co->perm.next = (ef_t *)calloc(co->perm.w + 1, sizeof(ef_t));
        memcpy(co->perm.local, pr2->vals[0], sizeof(ef_t) * co->perm.w);
        memcpy(co->perm.next, pr2->vals[1], sizeof(ef_t) * co->perm.w);
    }
    qi = pk->ntraces + 2 * n;
    for (int i = 0; i < n; i++) {
        orc_chip_open_t *co = &out->chips[i];
        co->nq = 1 << chips[i]->log_qd;
        co->quot = (ef_t *)malloc(sizeof(ef_t) * 4 * co->nq);
        for (int j = 0; j < co->nq; j++, qi++) memcpy(co->quot + 4 * j, req[qi].vals[0], sizeof(ef_t) * 4);
    }

    for (r = 0; r < nreq; r++) for (int p = 0; p < req[r].npts; p++) free(req[r].vals[p]);
    free(req);
    for (int i = 0; i < 32; i++) free(ro[i]);
    for (int rd = 0; rd < nrounds; rd++) orc_tree_free(&ftrees[rd]);
    free(ftrees);
    orc_tree_free(&main_tree); orc_tree_free(&perm_tree); orc_tree_free(&q_tree);
    for (int i = 0; i < n; i++) free(perm_flat[i]);
    free(perm_flat); free(o); free(chips); free(tr); free(hs); free(cidx);
    return final_ok ? 0 : -5;
}

void orc_proof_free(orc_proof_t *p) {
    for (int i = 0; i < p->nchips; i++) {
        orc_chip_open_t *c = &p->chips[i];
        free(c->prep.local); free(c->prep.next); free(c->main.local); free(c->main.next);
        free(c->perm.local); free(c->perm.next); free(c->quot);
    }
    free(p->chips);
    for (int q = 0; q < p->fri.nqueries; q++) {
        orc_query_t *qq = &p->fri.queries[q];
        for (int t = 0; t < qq->nrounds; t++) {
            for (int mi = 0; mi < qq->input[t].nmats; mi++) free(qq->input[t].vals[mi]);
            free(qq->input[t].vals); free(qq->input[t].widths); free(qq->input[t].path);
        }
        free(qq->input);
        for (int s = 0; s < qq->nsteps; s++) free(qq->steps[s].path);
        free(qq->steps);
    }
    free(p->fri.queries); free(p->fri.commits);
    free(p->ord_names); free(p->pv);
    memset(p, 0, sizeof *p);
}
