/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).
 *
 * Machine description parsing (format: include/zkm_hip.h "machine blob") and the
 * constraint semantics the reference's Chip::eval applies (crates/stark/src/chip.rs:259-271):
 *   1. the AIR's own constraints (here: a postfix program, one EMIT per assert_zero);
 *   2. eval_permutation_constraints (crates/stark/src/permutation.rs:205-347).
 * Lookup tuple fingerprints follow populate_local_permutation_row (permutation.rs:29-69).
 */
#include <stdlib.h>
#include "oracle_internal.h"

#define MAGIC 0x4D4D4B5Au

typedef struct { const uint32_t *w; size_t n, p; int err; } rd_t;
static uint32_t rd(rd_t *r) { if (r->p >= r->n) { r->err = 1; return 0; } return r->w[r->p++]; }

static void parse_vpc(rd_t *r, orc_vpc_t *v) {
    v->nterms = (int)rd(r);
    v->cols = (uint32_t *)calloc(v->nterms + 1, sizeof(uint32_t));
    v->weights = (kb_t *)calloc(v->nterms + 1, sizeof(kb_t));
    for (int i = 0; i < v->nterms; i++) { v->cols[i] = rd(r); v->weights[i] = rd(r) % KB_P; }
    v->constant = rd(r) % KB_P;
}

int orc_machine_parse(orc_machine_t *m, const uint32_t *w, size_t n) {
    rd_t r = {w, n, 0, 0};
    memset(m, 0, sizeof *m);
    if (rd(&r) != MAGIC || rd(&r) != 1) return -1;
    m->num_pv = (int)rd(&r);
    m->nchips = (int)rd(&r);
    m->chips = (orc_chip_t *)calloc(m->nchips, sizeof(orc_chip_t));
    for (int c = 0; c < m->nchips; c++) {
        orc_chip_t *ch = &m->chips[c];
        uint32_t nl = rd(&r);
        if (nl >= sizeof ch->name) return -2;
        for (uint32_t i = 0; i < (nl + 3) / 4; i++) {
            uint32_t x = rd(&r);
            for (int b = 0; b < 4 && 4 * i + b < nl; b++) ch->name[4 * i + b] = (char)((x >> (8 * b)) & 0xff);
        }
        ch->prep_width = (int)rd(&r);
        ch->main_width = (int)rd(&r);
        ch->commit_scope = (int)rd(&r);
        ch->local_only = (int)rd(&r);
        ch->log_qd = (int)rd(&r);
        ch->num_main_constraints = (int)rd(&r);
        ch->code_len = (int)rd(&r);
        ch->code = (uint32_t *)calloc(ch->code_len + 1, sizeof(uint32_t));
        for (int i = 0; i < ch->code_len; i++) ch->code[i] = rd(&r);
        ch->n_slots = 0;
        for (int pc = 0; pc < ch->code_len;) {
            uint32_t op = ch->code[pc++];
            if (op == OP_LET || op == OP_GET) {
                if (pc >= ch->code_len || ch->code[pc] >= (1u << 24)) return -5;
                if (op == OP_LET && (int)ch->code[pc] + 1 > ch->n_slots) ch->n_slots = (int)ch->code[pc] + 1;
                if (op == OP_GET && (int)ch->code[pc] >= ch->n_slots) return -5; /* use before definition */
                pc++;
            } else if (op == OP_MAIN_L || op == OP_MAIN_N || op == OP_PREP_L || op == OP_PREP_N || op == OP_CONST ||
                       op == OP_PV) {
                pc++;
            }
        }
        ch->nsends = (int)rd(&r);
        ch->nrecvs = (int)rd(&r);
        int total = ch->nsends + ch->nrecvs;
        orc_lookup_t *all = (orc_lookup_t *)calloc(total + 1, sizeof(orc_lookup_t));
        for (int i = 0; i < total; i++) {
            all[i].kind = rd(&r);
            all[i].scope = rd(&r);
            all[i].nvalues = (int)rd(&r);
            if (all[i].nvalues > 255) return -4; /* the LogUp evaluators keep beta^1..beta^256 */
            all[i].values = (orc_vpc_t *)calloc(all[i].nvalues + 1, sizeof(orc_vpc_t));
            for (int v = 0; v < all[i].nvalues; v++) parse_vpc(&r, &all[i].values[v]);
            parse_vpc(&r, &all[i].mult);
            all[i].is_send = i < ch->nsends;
        }
        /* scoped_lookups (permutation.rs:73-98): stable partition by scope; keep Local */
        ch->local = (orc_lookup_t *)calloc(total + 1, sizeof(orc_lookup_t));
        ch->nlocal = 0;
        for (int i = 0; i < total; i++)
            if (all[i].scope == 0) ch->local[ch->nlocal++] = all[i];
        free(all); /* value arrays now owned by ch->local (global ones leak: tiny, test only) */
        int batch = 1 << ch->log_qd;
        ch->perm_width_ef = ch->nlocal ? (ch->nlocal + batch - 1) / batch + 1 : 0;
        /* count_permutation_constraints (permutation.rs:355-388) */
        int pc = 0;
        if (ch->nlocal) pc += ch->perm_width_ef - 1 + 3;
        if (ch->commit_scope == 1) pc += 14;
        ch->num_constraints = ch->num_main_constraints + pc;
    }
    if (r.err) return -3;
    return 0;
}

void orc_machine_free(orc_machine_t *m) {
    for (int c = 0; c < m->nchips; c++) {
        orc_chip_t *ch = &m->chips[c];
        free(ch->code);
        for (int i = 0; i < ch->nlocal; i++) {
            for (int v = 0; v < ch->local[i].nvalues; v++) {
                free(ch->local[i].values[v].cols); free(ch->local[i].values[v].weights);
            }
            free(ch->local[i].values);
            free(ch->local[i].mult.cols); free(ch->local[i].mult.weights);
        }
        free(ch->local);
    }
    free(m->chips);
    memset(m, 0, sizeof *m);
}

kb_t orc_vpc_apply(const orc_vpc_t *v, const kb_t *prep, const kb_t *main) {
    kb_t acc = v->constant;
    for (int i = 0; i < v->nterms; i++) {
        uint32_t c = v->cols[i];
        kb_t x = (c & 0x80000000u) ? main[c & 0x7fffffffu] : prep[c];
        acc = kb_add(acc, kb_mul(x, v->weights[i]));
    }
    return acc;
}

ef_t orc_vpc_apply_ef(const orc_vpc_t *v, const ef_t *prep, const ef_t *main) {
    ef_t acc = ef_from_base(v->constant);
    for (int i = 0; i < v->nterms; i++) {
        uint32_t c = v->cols[i];
        ef_t x = (c & 0x80000000u) ? main[c & 0x7fffffffu] : prep[c];
        acc = ef_add(acc, ef_mul_base(x, v->weights[i]));
    }
    return acc;
}
