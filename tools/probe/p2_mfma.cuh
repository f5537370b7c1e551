// Poseidon2-16 with its external linear layers on the matrix cores (gfx950 v_mfma_i32_16x16x64_i8).
//
// Same permutation and internal representation as p2::permute_lam (p2.cuh): the state at scale LAMBDA,
// lazy Montgomery reductions, round constants injected through the S-box addends.  What changes is where
// the 9 external layers y -> M_E y (M_E = circ(2 M4, M4, M4, M4), ~36 % of the one-lane form's VALU work)
// run.  A wave permutes 64 states together:
//
//   * one-lane layout (the sponge, the partial rounds): lane s holds the 16 words of state s;
//   * MFMA layout (the full rounds): lane L = (n = L & 15, h = L >> 4) holds, for each group g < 4, words
//     4h..4h+3 of state 16g + n.  Those 16 bytes are exactly lane L's B operand of v_mfma_i32_16x16x64_i8
//     (B[k = 16h + j][col n], k <-> (word 4h + j / 4, byte j % 4)), each byte read as a signed limb b - 128
//     (xor 0x80; the offset is the constant K_OFF), and the instruction's C layout (lane L, register r =
//     row 4h + r of column n) is the same "words 4h..4h+3 of state 16g + n" -- consecutive layers need no
//     lane movement.  One MFMA per byte position l, A_l[i][(w, l')] = M_E[i][w] [l' == l]:
//       M_E y = C_0 + 2^8 C_1 + 2^16 C_2 + 2^24 C_3 + K_OFF    exactly (|C_l| <= 35 * 128);
//     16 MFMAs per layer per wave, ~7 VALU slots per word instead of ~15.
//   * the layouts change through a per-wave LDS tile (64 states x 20-word pitch, 16-byte accesses) before
//     the first full round, around the 13 partial rounds (whose internal layer is a row sum: one lane per
//     state keeps it in registers) and after the last full round.
//
// Every lane of the wave must call it (MFMA and the LDS exchange are wave-wide); the outputs are the same
// bits as p2::permute_lam's fold31 (tools/probe/p2_mfma_probe.hip checks them).
#pragma once
#include "../../zkmips_amd/csrc/p2.cuh"

namespace p2m {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr uint64_t K_OFF = 35ull * 128ull * 0x01010101ull;  // sum_w M_E[i][w] * 128 * (1 + 2^8 + 2^16 + 2^24)
constexpr int PITCH = 20;                                   // LDS words per state (16-byte aligned, spread banks)
constexpr int WAVE_WORDS = 64 * PITCH;                       // LDS words per wave for the layout exchange
constexpr int NCONST = 8;                                    // per-word 64-bit constant sets (MFMA layout)

// The per-word constants of the full rounds, indexed [set][word]: set 0 = round 0's explicit constants
// (FT.ext[0]), sets 1..3 = the S-box addends injecting rounds 1..3, set 4 = the partial round 0 addend,
// sets 5..7 = rounds 5..7.
struct ConstTable {
    uint64_t c[NCONST][16];
};
constexpr ConstTable make_consts() {
    ConstTable t{};
    for (int w = 0; w < 16; w++) {
        t.c[0][w] = p2::FT.ext[0][w];
        for (int i = 1; i < 4; i++) t.c[i][w] = p2::INJ.full[i].a[w];
        t.c[4][w] = p2::INJ.part0.a[w];
        for (int i = 5; i < 8; i++) t.c[i][w] = p2::INJ.full[i].a[w];
    }
    return t;
}
__device__ __constant__ inline ConstTable kConsts = make_consts();

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u4;

struct Ctx {
    v4i A[4];          // A_l operands of this lane (row n, k = 16h..16h+15)
    lds_u32 *x;        // this wave's LDS exchange tile (WAVE_WORDS words)
    const lds_u64 *ct; // LDS copy of kConsts (NCONST x 16 x 8 bytes, shared by the workgroup)
    uint32_t lane, n, h;
};

__device__ __forceinline__ int me(int i, int w) {  // M_E = circ(2 M4, M4, M4, M4), M4 = circ(2, 3, 1, 1)
    const int M4[4][4] = {{2, 3, 1, 1}, {1, 2, 3, 1}, {1, 1, 2, 3}, {3, 1, 1, 2}};
    return M4[i & 3][w & 3] * ((i >> 2) == (w >> 2) ? 2 : 1);
}

// the S-box with an injected addend that differs per lane (p2::cube_inj takes a uniform one)
__device__ __forceinline__ uint32_t cube_inj_v(uint32_t r, uint64_t addend) {
    return kb::redc2(kb::mad64(p2::mul_l(r, r), r, addend));
}

// Per-workgroup setup: copy the constant table into LDS (ct: NCONST * 16 uint64 of __shared__ memory) and
// build this lane's operands.  Call from every thread, then __syncthreads() before the first permutation.
__device__ __forceinline__ Ctx make_ctx(uint32_t *wave_tile, uint64_t *ct) {
    Ctx c;
    c.lane = threadIdx.x & 63;
    c.n = c.lane & 15;
    c.h = c.lane >> 4;
    c.x = (lds_u32 *)wave_tile;
    c.ct = (const lds_u64 *)ct;
    for (uint32_t i = threadIdx.x; i < NCONST * 16; i += blockDim.x) ((lds_u64 *)ct)[i] = kConsts.c[i >> 4][i & 15];
#pragma unroll
    for (int l = 0; l < 4; l++) {
        int d[4];
#pragma unroll
        for (int q = 0; q < 4; q++) d[q] = (int)((uint32_t)(me((int)c.n, (int)(4 * c.h + q)) & 0xff) << (8 * l));
        c.A[l] = v4i{d[0], d[1], d[2], d[3]};
    }
    return c;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// one-lane layout (16 words of state `lane`) -> MFMA layout m[g][r] (word 4h + r of state 16g + n)
__device__ __forceinline__ void to_mfma(const Ctx &c, const uint32_t s[16], uint32_t m[4][4]) {
    lds_u4 *row = (lds_u4 *)(c.x + c.lane * PITCH);
#pragma unroll
    for (int q = 0; q < 4; q++) row[q] = u32x4{s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]};
    wave_sync();
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const u32x4 v = *(const lds_u4 *)(c.x + (16 * g + c.n) * PITCH + 4 * c.h);
        m[g][0] = v.x; m[g][1] = v.y; m[g][2] = v.z; m[g][3] = v.w;
    }
    wave_sync();
}

__device__ __forceinline__ void from_mfma(const Ctx &c, const uint32_t m[4][4], uint32_t s[16]) {
#pragma unroll
    for (int g = 0; g < 4; g++)
        *(lds_u4 *)(c.x + (16 * g + c.n) * PITCH + 4 * c.h) = u32x4{m[g][0], m[g][1], m[g][2], m[g][3]};
    wave_sync();
    const lds_u4 *row = (const lds_u4 *)(c.x + c.lane * PITCH);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const u32x4 v = row[q];
        s[4 * q] = v.x; s[4 * q + 1] = v.y; s[4 * q + 2] = v.z; s[4 * q + 3] = v.w;
    }
    wave_sync();
}

// v = M_E y in the MFMA layout (exact 64-bit integers, as p2::external64)
__device__ __forceinline__ void external_m(const Ctx &c, const uint32_t y[4][4], uint64_t v[4][4]) {
    const v4i z = {0, 0, 0, 0};
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const v4i B = {(int)(y[g][0] ^ 0x80808080u), (int)(y[g][1] ^ 0x80808080u), (int)(y[g][2] ^ 0x80808080u),
                       (int)(y[g][3] ^ 0x80808080u)};
        const v4i c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(c.A[0], B, z, 0, 0, 0);
        const v4i c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(c.A[1], B, z, 0, 0, 0);
        const v4i c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(c.A[2], B, z, 0, 0, 0);
        const v4i c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(c.A[3], B, z, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int lo = c0[r] + (c1[r] << 8) + (c2[r] << 16);  // |lo| < 2^29
            v[g][r] = (uint64_t)((int64_t)lo + ((int64_t)c3[r] << 24) + (int64_t)K_OFF);
        }
    }
}

// this lane's four 64-bit constants of set `k` (words 4h..4h+3)
__device__ __forceinline__ void consts(const Ctx &c, int k, uint64_t out[4]) {
    const lds_u64 *p = c.ct + k * 16 + 4 * c.h;
#pragma unroll
    for (int r = 0; r < 4; r++) out[r] = p[r];
}

// p2::permute_lam with the external layers on the matrix cores; returns fold31 of the last layer's
// outputs (what every caller of permute_lam takes next) in the one-lane layout.
__device__ __forceinline__ void permute_lam(const Ctx &c, const uint32_t y_in[16], uint32_t out[16]) {
    using p2::cube_l;
    using p2::fold31;
    using kb::redc2;
    uint32_t y[4][4], r[4][4];
    uint64_t v[4][4], k[4];
    to_mfma(c, y_in, y);
    external_m(c, y, v);
    consts(c, 0, k);
#pragma unroll
    for (int g = 0; g < 4; g++)
#pragma unroll
        for (int q = 0; q < 4; q++) r[g][q] = redc2(v[g][q] + k[q]);
#pragma unroll
    for (int rd = 0; rd < 4; rd++) {  // full rounds 0..3: rounds 1..3 and partial round 0 injected
        consts(c, rd + 1, k);
#pragma unroll
        for (int g = 0; g < 4; g++)
#pragma unroll
            for (int q = 0; q < 4; q++) y[g][q] = cube_inj_v(r[g][q], k[q]);
        external_m(c, y, v);
        if (rd < 3) {
#pragma unroll
            for (int g = 0; g < 4; g++)
#pragma unroll
                for (int q = 0; q < 4; q++) r[g][q] = redc2(v[g][q]);
        }
    }
    // the partial rounds' entry values: s_j = fold31(v_j) for j >= 1, r0 = redc2(v_0) (word 0: h = 0, q = 0)
#pragma unroll
    for (int g = 0; g < 4; g++) {
        y[g][0] = c.h == 0 ? redc2(v[g][0]) : fold31(v[g][0]);
#pragma unroll
        for (int q = 1; q < 4; q++) y[g][q] = fold31(v[g][q]);
    }
    uint32_t sj[16];
    from_mfma(c, y, sj);
    uint32_t r0 = sj[0];
    uint32_t rr[16];
#pragma unroll
    for (int kk = 0; kk < 13; kk++) {  // p2::permute_lam's partial rounds, one lane per state
        const uint32_t y0 = cube_l(r0);
        uint64_t rest = sj[1];
#pragma unroll
        for (int j = 2; j < 16; j++) rest = kb::add_w(rest, sj[j]);
        const uint64_t acc = kb::add_w(rest, y0);
        const uint64_t e0 = kb::add_w(rest, 2 * kb::P - y0);
        if (kk < 12) {
            r0 = redc2(e0 + kb::kc64(p2::FT.inr[kk + 1]));
            const uint32_t lo = (uint32_t)acc & 0x3fffffffu, hi = (uint32_t)(acc >> 30);
            const uint64_t X = kb::mad64_ks(lo, kb::kc32(p2::R_MOD), kb::prod64_ks(hi, kb::kc32(p2::R_2_30)));
#pragma unroll
            for (int j = 1; j < 16; j++) sj[j] = redc2(kb::mad64_ks(sj[j], kb::kc32(p2::DIAG.v[j]), X));
        } else {
            rr[0] = redc2(e0 + kb::kc64(p2::FT.ext[4][0]));
#pragma unroll
            for (int j = 1; j < 16; j++) {
                const uint32_t t = redc2(kb::mad64_ks(sj[j], kb::kc32(p2::DIAG_C.v[j]), acc + kb::kc64(p2::FT.ext[4][j])));
                rr[j] = kb::umin(t, t - kb::P);
            }
        }
    }
    to_mfma(c, rr, r);
#pragma unroll
    for (int rd = 4; rd < 7; rd++) {  // full rounds 4..6 inject rounds 5..7
        consts(c, rd + 1, k);
#pragma unroll
        for (int g = 0; g < 4; g++)
#pragma unroll
            for (int q = 0; q < 4; q++) y[g][q] = cube_inj_v(r[g][q], k[q]);
        external_m(c, y, v);
#pragma unroll
        for (int g = 0; g < 4; g++)
#pragma unroll
            for (int q = 0; q < 4; q++) r[g][q] = redc2(v[g][q]);
    }
#pragma unroll
    for (int g = 0; g < 4; g++)
#pragma unroll
        for (int q = 0; q < 4; q++) y[g][q] = cube_l(r[g][q]);
    external_m(c, y, v);
#pragma unroll
    for (int g = 0; g < 4; g++)
#pragma unroll
        for (int q = 0; q < 4; q++) y[g][q] = fold31(v[g][q]);
    from_mfma(c, y, out);
}

// p2::permute (Montgomery in and out) on the matrix cores
__device__ __forceinline__ void permute(const Ctx &c, uint32_t s[16]) {
    uint32_t y[16], o[16];
#pragma unroll
    for (int j = 0; j < 16; j++) y[j] = p2::to_lam(s[j]);
    permute_lam(c, y, o);
#pragma unroll
    for (int j = 0; j < 16; j++) s[j] = kb::mul(o[j], p2::K_OUT);
}

}  // namespace p2m
