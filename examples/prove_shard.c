/*
 * prove_shard.c — a non-Python host of the C ABI (include/zkm_hip.h), the way a Rust shim or any
 * other native caller would drive MachineProver::setup / commit / open.
 *
 * Usage: prove_shard <manifest>
 * Manifest lines (whitespace separated; matrices are raw little-endian u32, row-major, canonical):
 *   blob <path>                       machine blob (zkmips_amd/machine.py MachineDesc.blob())
 *   queries <n> | pow_bits <n>
 *   prep <chip> <height> <width> <path>   preprocessed trace of machine chip <chip>
 *   trace <chip> <height> <width> <path>  main trace of the shard
 *   pv <count> <path>                 public values
 *   out <path>                        where the serialized ShardProof is written
 * Exit status: 0 ok, 1 ABI error (message on stderr), 2 usage / input error.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zkm_hip.h"

#define MAXM 64

typedef struct {
    char name[128];
    uint64_t h, w;
    uint32_t *data;
} mat_t;

static uint32_t *read_u32(const char *path, size_t n) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    uint32_t *p = (uint32_t *)malloc(n * 4 + 4);
    size_t got = p ? fread(p, 4, n, f) : 0;
    fclose(f);
    if (got != n) { free(p); return NULL; }
    return p;
}

static long file_words(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    fseek(f, 0, SEEK_END);
    long n = ftell(f) / 4;
    fclose(f);
    return n;
}

static int fail(const char *what, int rc) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, zkm_last_error());
    return 1;
}

int main(int argc, char **argv) {
    if (argc != 2) {
        fprintf(stderr, "usage: %s <manifest>\n", argv[0]);
        return 2;
    }
    FILE *mf = fopen(argv[1], "r");
    if (!mf) { perror(argv[1]); return 2; }
    char key[32], a[128], b[64], c[64], d[512];
    char blob_path[512] = "", pv_path[512] = "", out_path[512] = "";
    uint32_t queries = 84, pow_bits = 16, npv = 0;
    mat_t prep[MAXM], tr[MAXM];
    int nprep = 0, ntr = 0;
    while (fscanf(mf, "%31s", key) == 1) {
        if (!strcmp(key, "blob")) { if (fscanf(mf, "%511s", blob_path) != 1) return 2; }
        else if (!strcmp(key, "queries")) { if (fscanf(mf, "%u", &queries) != 1) return 2; }
        else if (!strcmp(key, "pow_bits")) { if (fscanf(mf, "%u", &pow_bits) != 1) return 2; }
        else if (!strcmp(key, "pv")) { if (fscanf(mf, "%u %511s", &npv, pv_path) != 2) return 2; }
        else if (!strcmp(key, "out")) { if (fscanf(mf, "%511s", out_path) != 1) return 2; }
        else if (!strcmp(key, "prep") || !strcmp(key, "trace")) {
            if (fscanf(mf, "%127s %63s %63s %511s", a, b, c, d) != 4) return 2;
            mat_t *m = !strcmp(key, "prep") ? &prep[nprep++] : &tr[ntr++];
            if (nprep > MAXM || ntr > MAXM) return 2;
            snprintf(m->name, sizeof m->name, "%s", a);
            m->h = strtoull(b, NULL, 10);
            m->w = strtoull(c, NULL, 10);
            m->data = read_u32(d, (size_t)(m->h * m->w));
            if (!m->data && (m->h * m->w) != 0) { fprintf(stderr, "cannot read %s\n", d); return 2; }
        } else {
            fprintf(stderr, "unknown manifest key %s\n", key);
            return 2;
        }
    }
    fclose(mf);
    long nblob = file_words(blob_path);
    uint32_t *blob = nblob > 0 ? read_u32(blob_path, (size_t)nblob) : NULL;
    uint32_t *pv = npv ? read_u32(pv_path, npv) : NULL;
    if (!blob || (npv && !pv) || !out_path[0]) { fprintf(stderr, "incomplete manifest\n"); return 2; }

    /* the blob header carries the chip count; chips without a "prep" line get an empty matrix */
    const uint32_t nchips = blob[3];
    zkm_matrix_t *pm = (zkm_matrix_t *)calloc(nchips, sizeof(zkm_matrix_t));
    for (uint32_t i = 0, pos = 4; i < nchips; i++) {
        const uint32_t nlen = blob[pos];
        char name[128] = {0};
        memcpy(name, &blob[pos + 1], nlen < sizeof name - 1 ? nlen : sizeof name - 1);
        pm[i].name = strdup(name);
        for (int k = 0; k < nprep; k++)
            if (!strcmp(prep[k].name, name)) {
                pm[i].data = prep[k].data;
                pm[i].height = prep[k].h;
                pm[i].width = prep[k].w;
            }
        pm[i].repr = ZKM_REPR_CANONICAL;
        /* skip this chip's words: name, widths..., constraint program, lookups */
        pos += 1 + (nlen + 3) / 4;
        const uint32_t ncode = blob[pos + 6];
        pos += 7 + ncode;
        const uint32_t nsend = blob[pos], nrecv = blob[pos + 1];
        pos += 2;
        for (uint32_t l = 0; l < nsend + nrecv; l++) {
            const uint32_t nvals = blob[pos + 2];
            pos += 3;
            for (uint32_t v = 0; v <= nvals; v++) pos += 1 + 2 * blob[pos] + 1; /* values + multiplicity */
        }
    }
    zkm_matrix_t tm[MAXM];
    for (int k = 0; k < ntr; k++)
        tm[k] = (zkm_matrix_t){tr[k].name, tr[k].data, tr[k].h, tr[k].w, ZKM_REPR_CANONICAL};

    zkm_ctx *ctx = NULL;
    int rc = zkm_init(0, &ctx);
    if (rc) return fail("zkm_init", rc);
    const zkm_config_t cfg = {queries, pow_bits, 1, 0};
    /* SepticDigest::zero (crates/stark/src/septic_digest.rs:9-14) */
    const uint32_t gcs[14] = {637514027, 1595065213, 1998064738, 72333738,  1211544370, 822986770, 1518535784,
                              1604177449, 90440090, 259343427,  140470264, 1162099742, 941559812, 1064053343};
    zkm_pk *pk = NULL;
    uint32_t vk_commit[8];
    rc = zkm_setup(ctx, blob, (size_t)nblob, &cfg, pm, nchips, 0x00400000u, gcs, &pk, vk_commit);
    if (rc) return fail("zkm_setup", rc);
    zkm_challenger_t ch;
    memset(&ch, 0, sizeof ch);
    rc = zkm_pk_observe(pk, &ch);
    if (rc) return fail("zkm_pk_observe", rc);
    uint8_t *proof = NULL;
    uint64_t len = 0;
    rc = zkm_prove_shard(ctx, pk, tm, (uint32_t)ntr, pv, npv, &ch, &proof, &len);
    if (rc) return fail("zkm_prove_shard", rc);
    FILE *of = fopen(out_path, "wb");
    if (!of || fwrite(proof, 1, len, of) != len) { perror(out_path); return 2; }
    fclose(of);
    printf("proof %llu bytes, vk commit %u %u ...\n", (unsigned long long)len, vk_commit[0], vk_commit[1]);
    zkm_free_bytes(proof);
    zkm_pk_free(pk);
    zkm_destroy(ctx);
    return 0;
}
