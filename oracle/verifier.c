/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).
 *
 * Shard verifier restated from:
 *   Verifier::verify_shard          crates/stark/src/verifier.rs:30-246
 *   verify_opening_shape / constraints / recompute_quotient  verifier.rs:248-436
 *   TwoAdicFriPcs::verify semantics crates/recursion/circuit/src/fri.rs:34-405
 *   selectors / zp at a point       crates/recursion/circuit/src/domain.rs:36-88
 * Used to check that proofs produced by the oracle (and by the GPU path) are accepted.
 */
#include <stdio.h>
#include <stdlib.h>
#include "stark.h"

#define FN eval_chip_ext_v
#define V ef_t
#define VADD ef_add
#define VSUB ef_sub
#define VMUL ef_mul
#define VNEG ef_neg
#define VCONST(x) ef_from_base(x)
#define EF_MUL_V ef_mul
#define APPLY_VPC orc_vpc_apply_ef
#include "air_eval.inc"

static const kb_t CSX[7] = CURVE_START_X, CSY[7] = CURVE_START_Y;

#define FAIL(code, msg) do { if (getenv("ORC_VERBOSE")) fprintf(stderr, "verify: %s\n", msg); ret = code; goto done; } while (0)

typedef struct { int log_n; kb_t shift; int width; int npts; ef_t pts[2]; const ef_t *vals[2]; } vmat_t;
typedef struct { digest_t commit; int nmats; vmat_t *mats; } vround_t;

static ef_t zp_at(int log_n, kb_t shift, ef_t z) {
    ef_t u = ef_mul_base(z, kb_inv(shift));
    for (int i = 0; i < log_n; i++) u = ef_mul(u, u);
    return ef_sub(u, ef_one());
}

int orc_verify_shard(const orc_pk_t *vk, const orc_proof_t *p, orc_chal_t *ch) {
    const orc_machine_t *m = vk->m;
    const int lb = vk->cfg.log_blowup;
    int ret = 0, n = p->nchips;
    int *cidx = (int *)calloc(n + 1, sizeof(int));
    vround_t rounds[4];
    memset(rounds, 0, sizeof rounds);
    for (int i = 0; i < n; i++) {
        cidx[i] = -1;
        for (int c = 0; c < m->nchips; c++) if (!strcmp(m->chips[c].name, p->ord_names[i])) cidx[i] = c;
        if (cidx[i] < 0) FAIL(-1, "unknown chip");
    }
    /* shape (verifier.rs:248-312) */
    for (int i = 0; i < n; i++) {
        const orc_chip_t *c = &m->chips[cidx[i]];
        const orc_chip_open_t *o = &p->chips[i];
        if (o->prep.w != c->prep_width || o->main.w != c->main_width || o->perm.w != 4 * c->perm_width_ef ||
            o->nq != (1 << c->log_qd) || o->log_degree < 0 || o->log_degree > 24)
            FAIL(-2, "opening shape");
    }
    orc_chal_observe_slice(ch, p->pv, m->num_pv);
    orc_chal_observe_digest(ch, p->main_commit);
    ef_t perm_ch[2];
    perm_ch[0] = orc_chal_sample_ef(ch);
    perm_ch[1] = orc_chal_sample_ef(ch);
    orc_chal_observe_digest(ch, p->perm_commit);
    for (int i = 0; i < n; i++) {
        const orc_chip_t *c = &m->chips[cidx[i]];
        const orc_chip_open_t *o = &p->chips[i];
        orc_chal_observe_ef(ch, o->lcs);
        orc_chal_observe_slice(ch, o->gcs, 14);
        if (c->commit_scope == 0 && (memcmp(o->gcs, CSX, 28) || memcmp(o->gcs + 7, CSY, 28)))
            FAIL(-3, "global sum nonzero for local chip");
        if (!c->nlocal && !ef_is_zero(o->lcs)) FAIL(-3, "local sum nonzero without local lookups");
    }
    ef_t alpha = orc_chal_sample_ef(ch);
    orc_chal_observe_digest(ch, p->quot_commit);
    ef_t zeta = orc_chal_sample_ef(ch);

    /* rounds (verifier.rs:124-205) */
    rounds[0].commit = vk->commit; rounds[0].nmats = vk->ntraces;
    rounds[0].mats = (vmat_t *)calloc(vk->ntraces + 1, sizeof(vmat_t));
    for (int t = 0; t < vk->ntraces; t++) {
        int i = -1;
        for (int k = 0; k < n; k++) if (cidx[k] == vk->trace_chip[t]) i = k;
        if (i < 0) FAIL(-4, "preprocessed chip missing from shard");
        vmat_t *vm = &rounds[0].mats[t];
        vm->log_n = log2_exact(vk->heights[t]); vm->shift = 1; vm->width = m->chips[cidx[i]].prep_width;
        vm->pts[0] = zeta; vm->vals[0] = p->chips[i].prep.local; vm->npts = 1;
        if (!m->chips[cidx[i]].local_only) {
            vm->pts[1] = ef_mul_base(zeta, kb_two_adic_gen(vm->log_n)); vm->vals[1] = p->chips[i].prep.next; vm->npts = 2;
        }
    }
    rounds[1].commit = p->main_commit; rounds[1].nmats = n;
    rounds[2].commit = p->perm_commit; rounds[2].nmats = n;
    rounds[1].mats = (vmat_t *)calloc(n, sizeof(vmat_t));
    rounds[2].mats = (vmat_t *)calloc(n, sizeof(vmat_t));
    int nchunks = 0;
    for (int i = 0; i < n; i++) nchunks += p->chips[i].nq;
    rounds[3].commit = p->quot_commit; rounds[3].nmats = nchunks;
    rounds[3].mats = (vmat_t *)calloc(nchunks + 1, sizeof(vmat_t));
    int qj = 0;
    for (int i = 0; i < n; i++) {
        const orc_chip_t *c = &m->chips[cidx[i]];
        const orc_chip_open_t *o = &p->chips[i];
        int ln = o->log_degree;
        ef_t znext = ef_mul_base(zeta, kb_two_adic_gen(ln));
        vmat_t *mm = &rounds[1].mats[i];
        mm->log_n = ln; mm->shift = 1; mm->width = c->main_width;
        mm->pts[0] = zeta; mm->vals[0] = o->main.local; mm->npts = 1;
        if (!c->local_only) { mm->pts[1] = znext; mm->vals[1] = o->main.next; mm->npts = 2; }
        vmat_t *pm = &rounds[2].mats[i];
        pm->log_n = ln; pm->shift = 1; pm->width = 4 * c->perm_width_ef;
        pm->pts[0] = zeta; pm->vals[0] = o->perm.local; pm->pts[1] = znext; pm->vals[1] = o->perm.next; pm->npts = 2;
        kb_t wQ = kb_two_adic_gen(ln + c->log_qd);
        for (int j = 0; j < o->nq; j++, qj++) {
            vmat_t *qm = &rounds[3].mats[qj];
            qm->log_n = ln; qm->shift = kb_mul(KB_GENERATOR, kb_pow(wQ, j)); qm->width = 4;
            qm->pts[0] = zeta; qm->vals[0] = o->quot + 4 * j; qm->npts = 1;
        }
    }

    /* ---- PCS verify (fri.rs:71-361) ---- */
    {
        const orc_fri_t *f = &p->fri;
        ef_t fa = orc_chal_sample_ef(ch);
        ef_t *betas = (ef_t *)malloc(sizeof(ef_t) * (f->ncommits + 1));
        for (int k = 0; k < f->ncommits; k++) { orc_chal_observe_digest(ch, f->commits[k]); betas[k] = orc_chal_sample_ef(ch); }
        orc_chal_observe_ef(ch, f->final_poly);
        if (f->nqueries != vk->cfg.num_queries) { free(betas); FAIL(-5, "query count"); }
        if (!orc_chal_check_witness(ch, vk->cfg.pow_bits, f->pow_witness)) { free(betas); FAIL(-6, "pow"); }
        int log_max = f->ncommits + lb;
        int apn = 0; ef_t *apow = NULL;
        for (int qn = 0; qn < f->nqueries && !ret; qn++) {
            size_t index = orc_chal_sample_bits(ch, log_max);
            const orc_query_t *qq = &f->queries[qn];
            if (qq->nrounds != 4 || qq->nsteps != f->ncommits) { ret = -7; break; }
            ef_t ro[32]; int lhp[32];
            for (int k = 0; k < 32; k++) { ro[k] = ef_zero(); lhp[k] = 0; }
            for (int t = 0; t < 4 && !ret; t++) {
                const vround_t *rd = &rounds[t];
                const orc_batch_open_t *bo = &qq->input[t];
                if (bo->nmats != rd->nmats) { ret = -8; break; }
                size_t *dims = (size_t *)malloc(sizeof(size_t) * (rd->nmats + 1));
                size_t *wid = (size_t *)malloc(sizeof(size_t) * (rd->nmats + 1));
                size_t bmax = 0;
                for (int k = 0; k < rd->nmats; k++) {
                    dims[k] = (size_t)1 << (rd->mats[k].log_n + lb);
                    wid[k] = rd->mats[k].width;
                    if (bo->widths[k] != wid[k]) ret = -9;
                    if (dims[k] > bmax) bmax = dims[k];
                }
                int lbm = log2_exact(bmax);
                size_t ridx = index >> (log_max - lbm);
                if (!ret && (bo->path_len != lbm ||
                             !orc_verify_batch(rd->commit, rd->nmats, dims, wid, (const kb_t *const *)bo->vals, ridx, bo->path, bo->path_len)))
                    ret = -10;
                for (int k = 0; k < rd->nmats && !ret; k++) {
                    const vmat_t *vm = &rd->mats[k];
                    int lh = vm->log_n + lb;
                    size_t idx = (index >> (log_max - lh)) & (((size_t)1 << lh) - 1);
                    kb_t x = kb_mul(KB_GENERATOR, kb_pow(kb_two_adic_gen(lh), rev_bits((uint32_t)idx, lh)));
                    for (int pt = 0; pt < vm->npts; pt++) {
                        ef_t acc = ef_zero();
                        for (int c = 0; c < vm->width; c++) {
                            int pw = lhp[lh]++;
                            while (apn <= pw) { apow = (ef_t *)realloc(apow, sizeof(ef_t) * (apn + 1)); apow[apn] = apn ? ef_mul(apow[apn - 1], fa) : ef_one(); apn++; }
                            acc = ef_add(acc, ef_mul(apow[pw], ef_sub(vm->vals[pt][c], ef_from_base(bo->vals[k][c]))));
                        }
                        ro[lh] = ef_add(ro[lh], ef_div(acc, ef_sub(vm->pts[pt], ef_from_base(x))));
                    }
                }
                free(dims); free(wid);
            }
            if (ret) break;
            if (!ef_is_zero(ro[lb])) { ret = -11; break; }
            /* verify_query (fri.rs:247-361) */
            ef_t folded = ro[log_max];
            kb_t x = kb_pow(kb_two_adic_gen(log_max), rev_bits((uint32_t)index, log_max));
            for (int off = 0; off < f->ncommits; off++) {
                int lfh = log_max - 1 - off;
                int bit = (index >> off) & 1;
                size_t ipair = index >> (off + 1);
                const orc_step_t *st = &qq->steps[off];
                ef_t e0 = bit ? st->sibling : folded, e1 = bit ? folded : st->sibling;
                kb_t row[8];
                memcpy(row, e0.c, 16); memcpy(row + 4, e1.c, 16);
                size_t hgt = (size_t)1 << lfh, w8 = 8;
                const kb_t *rp = row;
                if (st->path_len != lfh || !orc_verify_batch(f->commits[off], 1, &hgt, &w8, &rp, ipair, st->path, st->path_len)) { ret = -12; break; }
                kb_t xn = kb_mul(x, kb_two_adic_gen(1));
                kb_t x0 = bit ? xn : x, x1 = bit ? x : xn;
                ef_t t = ef_mul(ef_sub(betas[off], ef_from_base(x0)), ef_mul_base(ef_sub(e1, e0), kb_inv(kb_sub(x1, x0))));
                folded = ef_add(ef_add(e0, t), ef_mul(ef_mul(betas[off], betas[off]), ro[lfh]));
                x = kb_mul(x, x);
            }
            if (!ret && !ef_eq(folded, f->final_poly)) ret = -13;
        }
        free(apow); free(betas);
        if (ret) FAIL(ret, "fri");
    }

    /* ---- constraints at zeta (verifier.rs:316-397) ---- */
    {
        ef_t total_lcs = ef_zero();
        for (int i = 0; i < n; i++) {
            const orc_chip_t *c = &m->chips[cidx[i]];
            const orc_chip_open_t *o = &p->chips[i];
            int ln = o->log_degree;
            ef_t zh = zp_at(ln, 1, zeta);
            kb_t ginv = kb_inv(kb_two_adic_gen(ln));
            ef_t is_first = ef_div(zh, ef_sub(zeta, ef_one()));
            ef_t is_last = ef_div(zh, ef_sub(zeta, ef_from_base(ginv)));
            ef_t is_trans = ef_sub(zeta, ef_from_base(ginv));
            ef_t invz = ef_inv(zh);
            /* recompute_quotient */
            int nq = o->nq;
            kb_t wQ = kb_two_adic_gen(ln + c->log_qd);
            ef_t quotient = ef_zero();
            for (int a = 0; a < nq; a++) {
                kb_t sa = kb_mul(KB_GENERATOR, kb_pow(wQ, a));
                ef_t zps = ef_one();
                for (int b = 0; b < nq; b++) {
                    if (b == a) continue;
                    kb_t sb = kb_mul(KB_GENERATOR, kb_pow(wQ, b));
                    ef_t num = zp_at(ln, sb, zeta);
                    ef_t den = zp_at(ln, sb, ef_from_base(sa));
                    zps = ef_mul(zps, ef_div(num, den));
                }
                ef_t chunk = ef_zero();
                for (int e = 0; e < 4; e++) {
                    ef_t mono = ef_zero(); mono.c[e] = 1;
                    chunk = ef_add(chunk, ef_mul(mono, o->quot[4 * a + e]));
                }
                quotient = ef_add(quotient, ef_mul(zps, chunk));
            }
            /* perm opening unflatten */
            int pw = c->perm_width_ef;
            ef_t *pl = (ef_t *)calloc(pw + 1, sizeof(ef_t)), *pn = (ef_t *)calloc(pw + 1, sizeof(ef_t));
            for (int b = 0; b < pw; b++)
                for (int e = 0; e < 4; e++) {
                    ef_t mono = ef_zero(); mono.c[e] = 1;
                    pl[b] = ef_add(pl[b], ef_mul(mono, o->perm.local[4 * b + e]));
                    pn[b] = ef_add(pn[b], ef_mul(mono, o->perm.next[4 * b + e]));
                }
            int nc = c->num_constraints;
            ef_t *pows = (ef_t *)malloc(sizeof(ef_t) * (nc + 1));
            ef_t a = ef_one();
            for (int k = nc - 1; k >= 0; k--) { pows[k] = a; a = ef_mul(a, alpha); }
            ef_t folded = eval_chip_ext_v(c, o->prep.local, o->prep.next, o->main.local, o->main.next, pl, pn,
                                          is_first, is_last, is_trans, p->pv, perm_ch[0], perm_ch[1], o->lcs, o->gcs, pows);
            free(pows); free(pl); free(pn);
            if (!ef_eq(ef_mul(folded, invz), quotient)) FAIL(-14, "ood evaluation mismatch");
            total_lcs = ef_add(total_lcs, o->lcs);
        }
        if (!ef_is_zero(total_lcs)) FAIL(-15, "local cumulative sum nonzero");
    }
done:
    for (int t = 0; t < 4; t++) free(rounds[t].mats);
    free(cidx);
    return ret;
}
