/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).
 *
 * MerkleTreeMmcs<_, _, PaddingFreeSponge<P,16,8,8>, TruncatedPermutation<P,2,8,16>, 8>
 * (crates/stark/src/kb31_poseidon2.rs:176-177).  Tree shape and height injection are
 * pinned by the verifier in crates/recursion/circuit/src/fri.rs:363-405 (verify_batch):
 *   leaves  = hash(concat rows of the tallest matrices, stable commit order)
 *   level up: node = compress(left, right); if matrices of that height exist:
 *             node = compress(node, hash(concat their rows)).
 * open_batch: row index >> (log_max - log_h) per matrix; path[i] = layer_i[(index>>i)^1].
 */
#include <stdlib.h>
#include "oracle_internal.h"

static int cmp_height_desc_stable(const void *a, const void *b, void *ctx) {
    const orc_mat_t *m = (const orc_mat_t *)ctx;
    int ia = *(const int *)a, ib = *(const int *)b;
    if (m[ia].height != m[ib].height) return m[ia].height > m[ib].height ? -1 : 1;
    return ia - ib;
}

static void hash_rows(const orc_mat_t *mats, const int *group, int ng, size_t row, digest_t *out) {
    orc_sponge_t s;
    orc_sponge_init(&s);
    for (int g = 0; g < ng; g++) {
        const orc_mat_t *m = &mats[group[g]];
        orc_sponge_absorb(&s, m->data + row * m->width, m->width);
    }
    *out = orc_sponge_finish(&s);
}

void orc_tree_build(orc_tree_t *t, orc_mat_t *mats, int nmats, int owns) {
    t->nmats = nmats;
    t->mats = mats;
    t->owns = owns;
    int *order = (int *)malloc(sizeof(int) * nmats);
    for (int i = 0; i < nmats; i++) order[i] = i;
    qsort_r(order, nmats, sizeof(int), cmp_height_desc_stable, mats);
    size_t maxh = mats[order[0]].height;
    t->log_max_height = log2_exact(maxh);
    t->nlayers = t->log_max_height + 1;
    t->layers = (digest_t **)calloc(t->nlayers, sizeof(digest_t *));
    /* group of tallest */
    int pos = 0, g0 = 0;
    while (pos < nmats && mats[order[pos]].height == maxh) pos++;
    g0 = pos;
    t->layers[0] = (digest_t *)malloc(sizeof(digest_t) * maxh);
    const int x16 = orc_p2x16_available();
    if (x16 && maxh >= 16) {
#pragma omp parallel for schedule(static)
        for (size_t r = 0; r < maxh; r += 16) orc_p2x16_hash_rows(mats, order, g0, r, &t->layers[0][r]);
    } else {
#pragma omp parallel for schedule(static)
        for (size_t r = 0; r < maxh; r++) hash_rows(mats, order, g0, r, &t->layers[0][r]);
    }
    size_t h = maxh;
    for (int L = 1; L < t->nlayers; L++) {
        h >>= 1;
        int gstart = pos;
        while (pos < nmats && mats[order[pos]].height == h) pos++;
        int ng = pos - gstart;
        digest_t *prev = t->layers[L - 1];
        digest_t *cur = (digest_t *)malloc(sizeof(digest_t) * h);
        if (x16 && h >= 16) {  /* 16 nodes per AVX-512 batch (p2x16.c) */
#pragma omp parallel for schedule(static)
            for (size_t i = 0; i < h; i += 16) {
                orc_p2x16_compress_pairs(prev + 2 * i, cur + i);
                if (ng) {
                    digest_t rd[16];
                    orc_p2x16_hash_rows(mats, order + gstart, ng, i, rd);
                    orc_p2x16_compress2(cur + i, rd, cur + i);
                }
            }
            t->layers[L] = cur;
            continue;
        }
#pragma omp parallel for schedule(static)
        for (size_t i = 0; i < h; i++) {
            digest_t d = orc_p2_compress(prev[2 * i], prev[2 * i + 1]);
            if (ng) {
                digest_t rd;
                hash_rows(mats, order + gstart, ng, i, &rd);
                d = orc_p2_compress(d, rd);
            }
            cur[i] = d;
        }
        t->layers[L] = cur;
    }
    free(order);
}

void orc_tree_free(orc_tree_t *t) {
    for (int i = 0; i < t->nlayers; i++) free(t->layers[i]);
    free(t->layers);
    if (t->owns) {
        for (int i = 0; i < t->nmats; i++) free((void *)t->mats[i].data);
        free(t->mats);
    }
    memset(t, 0, sizeof *t);
}

digest_t orc_tree_root(const orc_tree_t *t) { return t->layers[t->nlayers - 1][0]; }

void orc_tree_open(const orc_tree_t *t, size_t index, const kb_t **rows, digest_t *path) {
    for (int m = 0; m < t->nmats; m++) {
        int lh = log2_exact(t->mats[m].height);
        size_t ri = index >> (t->log_max_height - lh);
        rows[m] = t->mats[m].data + ri * t->mats[m].width;
    }
    for (int i = 0; i < t->log_max_height; i++) path[i] = t->layers[i][(index >> i) ^ 1];
}

int orc_verify_batch(digest_t commit, int nmats, const size_t *heights, const size_t *widths,
                     const kb_t *const *values, size_t index, const digest_t *path, int path_len) {
    int *order = (int *)malloc(sizeof(int) * nmats);
    for (int i = 0; i < nmats; i++) order[i] = i;
    /* stable sort by height desc */
    for (int i = 1; i < nmats; i++)
        for (int j = i; j > 0 && heights[order[j]] > heights[order[j - 1]]; j--) {
            int tmp = order[j]; order[j] = order[j - 1]; order[j - 1] = tmp;
        }
    size_t cur = heights[order[0]];
    int pos = 0;
    orc_sponge_t s;
    orc_sponge_init(&s);
    while (pos < nmats && heights[order[pos]] == cur) {
        orc_sponge_absorb(&s, values[order[pos]], widths[order[pos]]);
        pos++;
    }
    digest_t root = orc_sponge_finish(&s);
    for (int i = 0; i < path_len; i++) {
        int bit = (index >> i) & 1;
        root = bit ? orc_p2_compress(path[i], root) : orc_p2_compress(root, path[i]);
        cur >>= 1;
        if (pos < nmats && heights[order[pos]] == cur) {
            orc_sponge_init(&s);
            while (pos < nmats && heights[order[pos]] == cur) {
                orc_sponge_absorb(&s, values[order[pos]], widths[order[pos]]);
                pos++;
            }
            root = orc_p2_compress(root, orc_sponge_finish(&s));
        }
    }
    free(order);
    return !memcmp(&root, &commit, sizeof root) && pos == nmats;
}
