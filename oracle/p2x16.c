/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see kb31.h).
 *
 * Poseidon2-16 over KoalaBear on 16 independent states at once (AVX-512, Montgomery form), for the
 * CPU baseline's Merkle trees: the same permutation, sponge and compression as poseidon2.c, lane i
 * carrying its own state.  Values enter in canonical form, are moved to Montgomery form (x * 2^32 mod p)
 * for the rounds and leave canonical again, so every digest equals poseidon2.c's bit for bit
 * (tests/test_oracle.py compares them).  Used only when the CPU reports AVX-512F.
 */
#include <string.h>

#include "oracle_internal.h"
#include "p2_rc.h"
#include "x16.h"

#define RF 8
#define RP 13

static const kb_t DIAG_C[16] = {
    KB_P - 2, 1, 2, (KB_P + 1) >> 1, 3, 4, (KB_P - 1) >> 1, KB_P - 3, KB_P - 4,
    KB_P - ((KB_P - 1) >> 8), KB_P - ((KB_P - 1) >> 3), KB_P - 127,
    (KB_P - 1) >> 8, (KB_P - 1) >> 3, (KB_P - 1) >> 4, 127,
};

static uint32_t R2, RC_M[30][16], DIAG_M[16];
uint32_t ORC_X16_MU;
static int consts_ready;

uint32_t orc_x16_to_mont(uint32_t x) { return (uint32_t)(((uint64_t)x << 32) % KB_P); }
static uint32_t to_mont_scalar(uint32_t x) { return orc_x16_to_mont(x); }

static void init_consts(void) {
    if (consts_ready) return;
    uint32_t inv = 1;  /* p^-1 mod 2^32 by Newton iteration */
    for (int i = 0; i < 5; i++) inv *= 2u - KB_P * inv;
    ORC_X16_MU = (uint32_t)(0u - inv);
    R2 = (uint32_t)(((unsigned __int128)1 << 64) % KB_P);
    for (int r = 0; r < 30; r++)
        for (int i = 0; i < 16; i++) RC_M[r][i] = to_mont_scalar(ORC_P2_RC[r][i] % KB_P);
    for (int i = 0; i < 16; i++) DIAG_M[i] = to_mont_scalar(DIAG_C[i]);
    __sync_synchronize();
    consts_ready = 1;
}

int orc_x16_available(void) {
    static int avail = -1;
    if (avail < 0) {
        __builtin_cpu_init();
        avail = __builtin_cpu_supports("avx512f") ? 1 : 0;
        if (avail) init_consts();
    }
    return avail;
}

int orc_p2x16_available(void) { return orc_x16_available(); }

TGT static inline __m512i sbox(__m512i x, uint32_t rc) {
    __m512i y = madd(x, _mm512_set1_epi32((int)rc));
    return mmul(mmul(y, y), y);
}

TGT static void external_layer(__m512i *s) {
    /* apply_m_4 per 4-block, then the column sums over the blocks (poseidon2.c external_layer) */
    __m512i t[16];
    for (int j = 0; j < 16; j += 4) {
        __m512i x0 = s[j], x1 = s[j + 1], x2 = s[j + 2], x3 = s[j + 3];
        __m512i t01 = madd(x0, x1), t23 = madd(x2, x3), t0123 = madd(t01, t23);
        __m512i t01123 = madd(t0123, x1), t01233 = madd(t0123, x3);
        t[j] = madd(t01123, t01);
        t[j + 1] = madd(t01123, madd(x2, x2));
        t[j + 2] = madd(t01233, t23);
        t[j + 3] = madd(t01233, madd(x0, x0));
    }
    for (int k = 0; k < 4; k++) {
        __m512i sum = madd(madd(t[k], t[4 + k]), madd(t[8 + k], t[12 + k]));
        for (int j = k; j < 16; j += 4) s[j] = madd(t[j], sum);
    }
}

TGT static void internal_layer(__m512i *s) {
    __m512i sum = s[0];
    for (int i = 1; i < 16; i++) sum = madd(sum, s[i]);
    for (int i = 0; i < 16; i++) s[i] = madd(mmul(s[i], _mm512_set1_epi32((int)DIAG_M[i])), sum);
}

TGT static void permute16(__m512i *s) {
    external_layer(s);
    for (int r = 0; r < RF / 2; r++) {
        for (int i = 0; i < 16; i++) s[i] = sbox(s[i], RC_M[r][i]);
        external_layer(s);
    }
    for (int r = 0; r < RP; r++) {
        s[0] = sbox(s[0], RC_M[RF / 2 + r][0]);
        internal_layer(s);
    }
    for (int r = RF / 2; r < RF; r++) {
        for (int i = 0; i < 16; i++) s[i] = sbox(s[i], RC_M[r + RP][i]);
        external_layer(s);
    }
}

TGT static inline __m512i to_mont(__m512i x) { return mmul(x, _mm512_set1_epi32((int)R2)); }
TGT static inline __m512i from_mont(__m512i x) { return mmul(x, _mm512_set1_epi32(1)); }

/* digests of rows row0 .. row0 + 15 of the concatenated rows of mats[group[0..ng)] (poseidon2.c sponge) */
TGT void orc_p2x16_hash_rows(const orc_mat_t *mats, const int *group, int ng, size_t row0, digest_t *out) {
    __m512i st[16];
    for (int i = 0; i < 16; i++) st[i] = _mm512_setzero_si512();
    int pos = 0;
    uint32_t lane[16] __attribute__((aligned(64)));
    for (int g = 0; g < ng; g++) {
        const orc_mat_t *m = &mats[group[g]];
        const size_t w = m->width;
        const kb_t *base = m->data + row0 * w;
        for (size_t c = 0; c < w; c++) {
            for (int l = 0; l < 16; l++) lane[l] = base[(size_t)l * w + c];
            st[pos++] = to_mont(_mm512_load_si512((const void *)lane));
            if (pos == P2_RATE) { permute16(st); pos = 0; }
        }
    }
    if (pos != 0) permute16(st);
    uint32_t o[8][16] __attribute__((aligned(64)));
    for (int i = 0; i < 8; i++) _mm512_store_si512((void *)o[i], from_mont(st[i]));
    for (int l = 0; l < 16; l++)
        for (int i = 0; i < 8; i++) out[l].v[i] = o[i][l];
}

/* out[i] = compress(in[2i], in[2i + 1]) for i < 16 */
TGT void orc_p2x16_compress_pairs(const digest_t *in, digest_t *out) {
    __m512i st[16];
    uint32_t lane[16] __attribute__((aligned(64)));
    for (int e = 0; e < 16; e++) {
        for (int l = 0; l < 16; l++) lane[l] = e < 8 ? in[2 * l].v[e] : in[2 * l + 1].v[e - 8];
        st[e] = to_mont(_mm512_load_si512((const void *)lane));
    }
    permute16(st);
    uint32_t o[8][16] __attribute__((aligned(64)));
    for (int i = 0; i < 8; i++) _mm512_store_si512((void *)o[i], from_mont(st[i]));
    for (int l = 0; l < 16; l++)
        for (int i = 0; i < 8; i++) out[l].v[i] = o[i][l];
}

/* out[i] = compress(a[i], b[i]) for i < 16 */
TGT void orc_p2x16_compress2(const digest_t *a, const digest_t *b, digest_t *out) {
    __m512i st[16];
    uint32_t lane[16] __attribute__((aligned(64)));
    for (int e = 0; e < 16; e++) {
        for (int l = 0; l < 16; l++) lane[l] = e < 8 ? a[l].v[e] : b[l].v[e - 8];
        st[e] = to_mont(_mm512_load_si512((const void *)lane));
    }
    permute16(st);
    uint32_t o[8][16] __attribute__((aligned(64)));
    for (int i = 0; i < 8; i++) _mm512_store_si512((void *)o[i], from_mont(st[i]));
    for (int l = 0; l < 16; l++)
        for (int i = 0; i < 8; i++) out[l].v[i] = o[i][l];
}
