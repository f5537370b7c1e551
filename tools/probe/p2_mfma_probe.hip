// Poseidon2-16 external linear layer on MI355X: the current 64-bit VALU form against the matrix-core form
// (v_mfma_i32_16x16x64_i8) and a 32-bit lazily reduced VALU form (the analytical study is
// profiles/r04_p2_mfma_ab.txt).  Each kernel applies y <- fold31(M_E y) ITER times to register-resident states
// (M_E = circ(2 M4, M4, M4, M4), y < 2P at the permutation's internal scale, exactly the layer k_hash_leaves
// runs 9 times per permutation), 64 states per wave; the outputs of the three forms must be bit-identical.
//
// MFMA form (no cross-lane traffic): lane L of a wave (n = L & 15, h = L >> 4) holds, for each of 4 groups g,
// words 4h..4h+3 of state 16g + n.  Those 16 bytes ARE the B operand of v_mfma_i32_16x16x64_i8 (lane L holds
// B[k = 16h + j][col n]; k <-> (word 4h + j/4, byte j%4)), with each byte read as a signed limb b - 128 (xor
// 0x80; the offset is a per-row constant K = 35 * 128 * 0x01010101).  One MFMA per byte position l with
// A_l[i][(w, l')] = M_E[i][w] [l' == l] gives C_l[i][n] = sum_w M_E[i][w] (byte l of y_w - 128), and its C
// layout (lane L, register r = row 4h + r of column n) is again "words 4h..4h+3 of state 16g + n":
//   M_E y = C_0 + 2^8 C_1 + 2^16 C_2 + 2^24 C_3 + K   (|C_l| <= 35 * 128, the sum < 2^37).
// 16 MFMAs per layer per wave (4 groups x 4 limbs) and ~5 VALU ops per word.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form p2_mfma_probe.hip -o p2_mfma_probe
// (the flag keeps the MFMA results in VGPRs: without it every result word costs a v_accvgpr_read)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "p2_mfma.cuh"

typedef int v4i __attribute__((ext_vector_type(4)));

static constexpr int NT = 256;
static constexpr uint64_t K_OFF = 35ull * 128ull * 0x01010101ull;  // sum_w M_E[i][w] * 128 * (1 + 2^8 + 2^16 + 2^24)

__device__ __forceinline__ uint32_t init_word(uint32_t state, uint32_t w) {
    uint64_t x = (uint64_t)state * 0x9E3779B97F4A7C15ull + w * 0xBF58476D1CE4E5B9ull + 0x94D049BB133111EBull;
    x ^= x >> 31;
    x *= 0xD6E8FEB86659FD93ull;
    x ^= x >> 29;
    return (uint32_t)(x % (2ull * kb::P));  // the layer's input range: y < 2P
}

__device__ __forceinline__ int me(int i, int w) {  // M_E = circ(2 M4, M4, M4, M4)
    const int m4[4][4] = {{2, 3, 1, 1}, {1, 2, 3, 1}, {1, 1, 2, 3}, {3, 1, 1, 2}};
    return m4[i & 3][w & 3] * ((i >> 2) == (w >> 2) ? 2 : 1);
}

template <int ITER>
__global__ __launch_bounds__(NT) void k_valu64(uint32_t *out) {
    const uint32_t s = blockIdx.x * NT + threadIdx.x;
    uint32_t y[16];
    uint64_t v[16];
#pragma unroll
    for (int w = 0; w < 16; w++) y[w] = init_word(s, w);
    for (int it = 0; it < ITER; it++) {
        p2::external64(y, v);
#pragma unroll
        for (int w = 0; w < 16; w++) y[w] = p2::fold31(v[w]);
    }
#pragma unroll
    for (int w = 0; w < 16; w++) out[(uint64_t)s * 16 + w] = y[w];
}

// 32-bit form: inputs reduced to [0, P), every sum reduced to [0, P) by one conditional subtract (v_min of x
// and x - P as unsigned); the result is M_E y mod p, re-expressed in the fold31 range for the comparison.
__device__ __forceinline__ uint32_t am(uint32_t a, uint32_t b) {
    const uint32_t s = a + b;
    return kb::umin(s, s - kb::P);
}
template <int ITER>
__global__ __launch_bounds__(NT) void k_valu32(uint32_t *out) {
    const uint32_t s = blockIdx.x * NT + threadIdx.x;
    uint32_t y[16];
#pragma unroll
    for (int w = 0; w < 16; w++) y[w] = init_word(s, w);
    for (int it = 0; it < ITER; it++) {
        uint32_t x[16], v[16];
#pragma unroll
        for (int w = 0; w < 16; w++) x[w] = kb::umin(y[w], y[w] - kb::P);
#pragma unroll
        for (int j = 0; j < 16; j += 4) {
            const uint32_t t01 = am(x[j], x[j + 1]), t23 = am(x[j + 2], x[j + 3]), t0123 = am(t01, t23);
            const uint32_t t01123 = am(t0123, x[j + 1]), t01233 = am(t0123, x[j + 3]);
            v[j] = am(t01123, t01);
            v[j + 1] = am(t01123, am(x[j + 2], x[j + 2]));
            v[j + 2] = am(t01233, t23);
            v[j + 3] = am(t01233, am(x[j], x[j]));
        }
        uint32_t sums[4];
#pragma unroll
        for (int k = 0; k < 4; k++) sums[k] = am(am(v[k], v[4 + k]), am(v[8 + k], v[12 + k]));
#pragma unroll
        for (int w = 0; w < 16; w++) y[w] = am(v[w], sums[w & 3]);  // < P: already in the fold31 range
    }
#pragma unroll
    for (int w = 0; w < 16; w++) out[(uint64_t)s * 16 + w] = y[w] % kb::P;
}

template <int ITER>
__global__ __launch_bounds__(NT) void k_mfma(uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63, n = lane & 15, h = lane >> 4;
    const uint32_t base = (blockIdx.x * NT + threadIdx.x - lane);  // 64 states per wave
    // A_l: lane (row i = n, group h) holds A[i][k = 16h + j], k <-> (word 4h + j / 4, byte j % 4)
    v4i A[4];
#pragma unroll
    for (int l = 0; l < 4; l++) {
        int d[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {  // dword q = bytes 4q..4q+3 = word 4h + q, bytes 0..3
            const int c = me((int)n, (int)(4 * h + q));
            d[q] = (int)((uint32_t)(c & 0xff) << (8 * l));
        }
        A[l] = v4i{d[0], d[1], d[2], d[3]};
    }
    uint32_t y[4][4];  // [group][r] = word 4h + r of state 16g + n
#pragma unroll
    for (int g = 0; g < 4; g++)
#pragma unroll
        for (int r = 0; r < 4; r++) y[g][r] = init_word(base + 16 * g + n, 4 * h + r);
    const v4i zero = {0, 0, 0, 0};
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const v4i B = {(int)(y[g][0] ^ 0x80808080u), (int)(y[g][1] ^ 0x80808080u), (int)(y[g][2] ^ 0x80808080u),
                           (int)(y[g][3] ^ 0x80808080u)};
            const v4i c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], B, zero, 0, 0, 0);
            const v4i c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1], B, zero, 0, 0, 0);
            const v4i c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[2], B, zero, 0, 0, 0);
            const v4i c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[3], B, zero, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int lo = c0[r] + (c1[r] << 8) + (c2[r] << 16);  // |lo| < 2^29
                const uint64_t v = (uint64_t)((int64_t)lo + ((int64_t)c3[r] << 24) + (int64_t)K_OFF);
                y[g][r] = p2::fold31(v);
            }
        }
    }
#pragma unroll
    for (int g = 0; g < 4; g++)
#pragma unroll
        for (int r = 0; r < 4; r++) out[(uint64_t)(base + 16 * g + n) * 16 + 4 * h + r] = y[g][r];
}

// The whole permutation: p2::permute (one lane per state) against p2m::permute (zkmips_amd/csrc/p2_mfma.cuh:
// the external layers on the matrix cores, 64 states per wave), ITERP permutations per state.
template <int ITERP>
__global__ __launch_bounds__(NT) void k_perm_valu(uint32_t *out) {
    const uint32_t st = blockIdx.x * NT + threadIdx.x;
    uint32_t s[16];
#pragma unroll
    for (int w = 0; w < 16; w++) s[w] = init_word(st, w) % kb::P;
    for (int it = 0; it < ITERP; it++) p2::permute(s);
#pragma unroll
    for (int w = 0; w < 16; w++) out[(uint64_t)st * 16 + w] = s[w];
}
template <int ITERP>
__global__ __launch_bounds__(NT) void k_perm_mfma(uint32_t *out) {
    __shared__ uint32_t tile[NT / 64 * p2m::WAVE_WORDS];
    __shared__ uint64_t ct[p2m::NCONST * 16];
    const p2m::Ctx c = p2m::make_ctx(tile + (threadIdx.x >> 6) * p2m::WAVE_WORDS, ct);
    __syncthreads();
    const uint32_t st = blockIdx.x * NT + threadIdx.x;
    uint32_t s[16];
#pragma unroll
    for (int w = 0; w < 16; w++) s[w] = init_word(st, w) % kb::P;
    for (int it = 0; it < ITERP; it++) p2m::permute(c, s);
#pragma unroll
    for (int w = 0; w < 16; w++) out[(uint64_t)st * 16 + w] = s[w];
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

template <class F>
static double time_ms(F launch, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char **argv) {
    constexpr int ITER = 256;
    const int blocks = argc > 1 ? atoi(argv[1]) : 4096;  // 4096 x 256 = 1M states
    const size_t states = (size_t)blocks * NT;
    uint32_t *o64, *o32, *omf;
    CK(hipMalloc(&o64, states * 64));
    CK(hipMalloc(&o32, states * 64));
    CK(hipMalloc(&omf, states * 64));
    const int reps = 5;
    const double t64 = time_ms([&] { hipLaunchKernelGGL(k_valu64<ITER>, dim3(blocks), dim3(NT), 0, 0, o64); }, reps);
    const double t32 = time_ms([&] { hipLaunchKernelGGL(k_valu32<ITER>, dim3(blocks), dim3(NT), 0, 0, o32); }, reps);
    const double tmf = time_ms([&] { hipLaunchKernelGGL(k_mfma<ITER>, dim3(blocks), dim3(NT), 0, 0, omf); }, reps);
    std::vector<uint32_t> a(states * 16), b(states * 16), c(states * 16);
    CK(hipMemcpy(a.data(), o64, states * 64, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), o32, states * 64, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c.data(), omf, states * 64, hipMemcpyDeviceToHost));
    size_t bad_mf = 0, bad_32 = 0;
    for (size_t i = 0; i < a.size(); i++) {
        bad_mf += a[i] != c[i];
        bad_32 += (a[i] % kb::P) != b[i];
    }
    // slots: one lane-op at the full SIMD-32 rate; 256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz
    const double slots_per_s = 256.0 * 4 * 32 * 2.4e9;
    auto rep = [&](const char *name, double ms) {
        const double layers = (double)states * ITER;
        printf("%-8s %8.3f ms  %7.3f ns/layer/state (device)  %6.1f slot-equivalents per state-layer\n", name, ms,
               ms * 1e6 / layers * 1e0, ms * 1e-3 * slots_per_s / layers);
    };
    rep("valu64", t64);
    rep("valu32", t32);
    rep("mfma", tmf);
    printf("states %zu  iterations %d  mismatches: mfma %zu  valu32 %zu\n", states, ITER, bad_mf, bad_32);
    // whole permutations
    constexpr int ITERP = 16;
    const double pv = time_ms([&] { hipLaunchKernelGGL(k_perm_valu<ITERP>, dim3(blocks), dim3(NT), 0, 0, o64); }, reps);
    const double pm = time_ms([&] { hipLaunchKernelGGL(k_perm_mfma<ITERP>, dim3(blocks), dim3(NT), 0, 0, omf); }, reps);
    CK(hipMemcpy(a.data(), o64, states * 64, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c.data(), omf, states * 64, hipMemcpyDeviceToHost));
    size_t bad_p = 0;
    for (size_t i = 0; i < a.size(); i++) bad_p += a[i] != c[i];
    const double perms = (double)states * ITERP;
    printf("permute  valu %8.3f ms  %.4e perms/s  %6.0f slot-equivalents/perm\n", pv, perms / (pv * 1e-3),
           pv * 1e-3 * slots_per_s / perms);
    printf("permute  mfma %8.3f ms  %.4e perms/s  %6.0f slot-equivalents/perm  (%.3fx)  mismatches %zu\n", pm,
           perms / (pm * 1e-3), pm * 1e-3 * slots_per_s / perms, pv / pm, bad_p);
    return (bad_mf || bad_32 || bad_p) ? 2 : 0;
}
