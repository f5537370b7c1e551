// Host extension-field (F[X]/(X^4 - 3) over KoalaBear) batch products for the recursion runtime's ExtAlu
// and BatchFRI instructions (recursion/core/src/runtime/mod.rs), canonical words in and out: the numpy
// form spent most of a compress node's execution in per-column Python loops.
#include <cstdint>

namespace {
constexpr uint64_t P = 0x7f000001u;
inline void ef_mul(const uint32_t *a, const uint32_t *b, uint32_t *r) {
    // r_k = sum_{i+j=k} a_i b_j + 3 sum_{i+j=k+4} a_i b_j; every term < 2^62, each sum reduced once
    uint64_t t[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) t[i + j] = (t[i + j] + (uint64_t)a[i] * b[j]) % P;
    for (int k = 0; k < 4; k++) r[k] = (uint32_t)((t[k] + (k < 3 ? 3 * t[k + 4] : 0)) % P);
}
}  // namespace

extern "C" void zkm_host_ef_mul(const uint32_t *a, const uint32_t *b, uint32_t *out, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) ef_mul(a + 4 * i, b + 4 * i, out + 4 * i);
}

// BatchFRI: per instruction row q, acc_l = sum_{i <= l} alpha_pow[q][i] * (p_at_z[q][i] - p_at_x[q][i]);
// acc (n x L x 4) receives every running value (the chip's trace rows), the last one is the result.
extern "C" void zkm_host_batch_fri(const uint32_t *alpha_pow, const uint32_t *p_at_z, const uint32_t *p_at_x,
                                   uint64_t n, uint64_t L, uint32_t *acc) {
    for (uint64_t q = 0; q < n; q++) {
        uint32_t run[4] = {0, 0, 0, 0};
        for (uint64_t i = 0; i < L; i++) {
            const uint64_t e = q * L + i;
            uint32_t d[4], t[4];
            for (int k = 0; k < 4; k++) d[k] = p_at_z[4 * e + k];
            d[0] = (uint32_t)((d[0] + P - p_at_x[e] % P) % P);
            ef_mul(alpha_pow + 4 * e, d, t);
            for (int k = 0; k < 4; k++) {
                run[k] = (uint32_t)((run[k] + (uint64_t)t[k]) % P);
                acc[4 * e + k] = run[k];
            }
        }
    }
}
