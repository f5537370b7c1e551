// Poseidon2-16 over KoalaBear in Montgomery form, host + gfx950 device.
//
// Configuration = the reference's poseidon2_init (crates/primitives/src/lib.rs:1107-1122):
//   initial external linear layer; 4 full rounds (RC rows 0..3); 13 partial rounds (RC rows
//   4..16, column 0); 4 full rounds (RC rows 17..20); S-box x^3.
//   External layer: M4 blocks + column sums (crates/core/machine/src/operations/poseidon2/air.rs:31-56).
//   Internal layer: s_i <- V_i s_i + sum(s), V = [-2,1,2,1/2,3,4,-1/2,-3,-4,1/2^8,1/8,1/2^24,
//                   -1/2^8,-1/8,-1/16,-1/2^24] (air.rs:12-29).
#pragma once
#include "kb_lazy.cuh"

namespace p2 {

#include "p2_rc.inc"

constexpr uint32_t cx_to_mont(uint32_t x) { return (uint32_t)((((uint64_t)(x % kb::P)) << 32) % kb::P); }
constexpr uint32_t cx_mulmod(uint32_t a, uint32_t b) { return (uint32_t)((uint64_t)a * b % kb::P); }
constexpr uint32_t cx_pow(uint32_t a, uint64_t e) {
    uint64_t r = 1, b = a % kb::P;
    for (; e; e >>= 1, b = b * b % kb::P)
        if (e & 1) r = r * b % kb::P;
    return (uint32_t)r;
}
constexpr uint32_t cx_inv(uint32_t a) { return cx_pow(a, kb::P - 2); }
constexpr uint32_t cx_neg(uint32_t x) { return x ? kb::P - x : 0; }
constexpr uint32_t cx_inv2k(int k) { return cx_inv(cx_pow(2, (uint64_t)k)); }  // 2^-k mod p

// Internal-layer diagonal V (canonical), air.rs:12-29
struct DiagTable {
    uint32_t v[16];
};
constexpr DiagTable make_diag_canon() {
    return DiagTable{{cx_neg(2), 1, 2, cx_inv2k(1), 3, 4, cx_neg(cx_inv2k(1)), cx_neg(3), cx_neg(4), cx_inv2k(8),
                      cx_inv2k(3), cx_inv2k(24), cx_neg(cx_inv2k(8)), cx_neg(cx_inv2k(3)), cx_neg(cx_inv2k(4)),
                      cx_neg(cx_inv2k(24))}};
}
constexpr DiagTable make_diag() {  // Montgomery form (R V_i)
    DiagTable d = make_diag_canon();
    for (int i = 0; i < 16; i++) d.v[i] = cx_to_mont(d.v[i]);
    return d;
}
constexpr DiagTable DIAG_C = make_diag_canon();
constexpr DiagTable DIAG = make_diag();

struct RcTable {
    uint32_t ext[8][16];  // full rounds 0..7 (Montgomery)
    uint32_t inr[13];     // partial rounds
};
constexpr RcTable make_rc() {
    RcTable t{};
    for (int r = 0; r < 4; r++)
        for (int i = 0; i < 16; i++) t.ext[r][i] = cx_to_mont(kP2RoundConstCanon[r][i]);
    for (int r = 0; r < 13; r++) t.inr[r] = cx_to_mont(kP2RoundConstCanon[4 + r][0]);
    for (int r = 4; r < 8; r++)
        for (int i = 0; i < 16; i++) t.ext[r][i] = cx_to_mont(kP2RoundConstCanon[r + 13][i]);
    return t;
}
constexpr RcTable RC = make_rc();

// ---------------------------------------------------------------------------------------------
// One-thread permutation: scaled state, 64-bit linear layers, lazy Montgomery reductions.
//
// The state is carried at the scale LAMBDA = 2^80 mod p (a stored value v stands for v / LAMBDA)
// instead of the Montgomery scale R = 2^32.  Because LAMBDA^2 = R^5 a full round closes on itself:
//   r  = redc(v + LAMBDA rc)   scale LAMBDA / R   (one 4-slot Montgomery reduction, kb::redc2)
//   y  = r^3 / R^2             scale LAMBDA       (two Montgomery products)
//   v' = M_E y                 scale LAMBDA       (64-bit integer adds, no reductions at all)
// The internal layer s_i <- V_i s_i + sum is one v_mad_u64_u32 + one lazy reduction per element,
// redc(s_i (R V_i) + X) with X = R sum (mod p), and element 0's next S-box input is taken straight
// from the partial sum.  Every 32-bit intermediate stays in (0, 2P) (bounds in the comments);
// input and output are canonical Montgomery values in [0, P).
using kb::add_w;
using kb::add_w2;
using kb::kc32;
using kb::kc64;
using kb::mad64;
using kb::mad64_add;
using kb::mad64_ks;
using kb::prod64;
using kb::prod64_ks;
using kb::redc2;

KB_HD uint32_t mul_l(uint32_t a, uint32_t b) { return redc2(prod64(a, b)); }  // a b < P 2^32 -> [0, 2P)
// r < P + 2^10: r^2 < P 2^32 -> sq < 2P; sq r < 2P (P + 2^10) < P 2^32 -> result in [0, 2P)
KB_HD uint32_t cube_l(uint32_t r) { return mul_l(mul_l(r, r), r); }
// 32-bit representative of v < 2^38 (2^31 = 2^24 - 1 mod p): lo + hi (2^24 - 1) < 2^31 + hi 2^24
KB_HD uint32_t fold31(uint64_t v) {
    const uint32_t hi = (uint32_t)(v >> 31), lo = (uint32_t)v & 0x7fffffffu;
    return lo + (hi << 24) - hi;
}

constexpr uint32_t LAMBDA = cx_pow(2, 80);  // LAMBDA^2 = 2^160 = R^5
constexpr uint32_t K_IN = LAMBDA;           // mont(x R, K_IN) = x LAMBDA
constexpr uint32_t K_OUT = cx_inv2k(16);    // mont(x LAMBDA, R^2 / LAMBDA) = x R
constexpr uint32_t R_MOD = cx_pow(2, 32);   // X = R lo + (R 2^30) hi for sum = hi 2^30 + lo
constexpr uint32_t R_2_30 = cx_pow(2, 62);

struct FastTable {
    uint64_t ext[8][16];  // LAMBDA rc (full rounds)
    uint64_t inr[13];     // LAMBDA rc (partial rounds, element 0)
};
constexpr FastTable make_fast() {
    FastTable t{};
    for (int r = 0; r < 4; r++)
        for (int i = 0; i < 16; i++) t.ext[r][i] = cx_mulmod(LAMBDA, kP2RoundConstCanon[r][i] % kb::P);
    for (int r = 0; r < 13; r++) t.inr[r] = cx_mulmod(LAMBDA, kP2RoundConstCanon[4 + r][0] % kb::P);
    for (int r = 4; r < 8; r++)
        for (int i = 0; i < 16; i++) t.ext[r][i] = cx_mulmod(LAMBDA, kP2RoundConstCanon[r + 13][i] % kb::P);
    return t;
}
constexpr FastTable FT = make_fast();

// Round-constant injection.  The S-box output y_j = redc(sq r + A_j) takes an arbitrary addend
// A_j = K_j (K_j < P keeps t < P 2^32), which adds K_j / R to y_j for free.  Choosing
// K = R M_E^{-1} (LAMBDA rc') makes the next external layer emit v + LAMBDA rc' directly, so the
// next round's S-box input is just redc(v).
// M_E = (I_4 + J_4) (x) M4, M_E^{-1} = (I_4 - J_4 / 5) (x) M4^{-1}; M4 as in external64 below.
struct Inj {
    uint64_t a[16];
};
constexpr uint32_t cx_sub(uint32_t a, uint32_t b) { return a >= b ? a - b : a + kb::P - b; }
constexpr uint32_t cx_add(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a + b) % kb::P); }
constexpr Inj make_inj(const uint32_t c_canon[16]) {  // c = rc' (canonical) per element
    // M4^{-1} by Gauss-Jordan mod p
    uint32_t m[4][8] = {{2, 3, 1, 1, 1, 0, 0, 0}, {1, 2, 3, 1, 0, 1, 0, 0}, {1, 1, 2, 3, 0, 0, 1, 0},
                        {3, 1, 1, 2, 0, 0, 0, 1}};
    for (int col = 0; col < 4; col++) {
        int piv = col;
        while (m[piv][col] == 0) piv++;
        for (int k = 0; k < 8; k++) { const uint32_t t = m[col][k]; m[col][k] = m[piv][k]; m[piv][k] = t; }
        const uint32_t iv = cx_inv(m[col][col]);
        for (int k = 0; k < 8; k++) m[col][k] = cx_mulmod(m[col][k], iv);
        for (int r = 0; r < 4; r++)
            if (r != col && m[r][col]) {
                const uint32_t f = m[r][col];
                for (int k = 0; k < 8; k++) m[r][k] = cx_sub(m[r][k], cx_mulmod(f, m[col][k]));
            }
    }
    uint32_t u[16] = {}, tot[4] = {};
    for (int b = 0; b < 4; b++)
        for (int i = 0; i < 4; i++) {
            uint32_t acc = 0;
            for (int k = 0; k < 4; k++) acc = cx_add(acc, cx_mulmod(m[i][4 + k], cx_mulmod(LAMBDA, c_canon[4 * b + k] % kb::P)));
            u[4 * b + i] = acc;
            tot[i] = cx_add(tot[i], acc);
        }
    const uint32_t inv5 = cx_inv(5);
    Inj r{};
    for (int j = 0; j < 16; j++) {
        const uint32_t d = cx_sub(u[j], cx_mulmod(inv5, tot[j & 3]));
        r.a[j] = cx_mulmod(d, R_MOD);
    }
    return r;
}
struct InjTable {
    Inj full[8];  // full[i]: injects full round i's constants (i = 1..3, 5..7; 0 and 4 unused)
    Inj part0;    // injects partial round 0's constant (element 0 only)
};
constexpr InjTable make_inj_table() {
    InjTable t{};
    for (int i = 1; i < 8; i++) {
        if (i == 4) continue;
        const int row = i < 4 ? i : i + 13;
        t.full[i] = make_inj(kP2RoundConstCanon[row]);
    }
    uint32_t c[16] = {};
    c[0] = kP2RoundConstCanon[4][0];
    t.part0 = make_inj(c);
    return t;
}
constexpr InjTable INJ = make_inj_table();

// cube with injected addend (see Inj); r < P + 2^10 -> (0, 2P)
KB_HD uint32_t cube_inj(uint32_t r, uint64_t addend) { return redc2(mad64_add(mul_l(r, r), r, addend)); }

// External layer on y < 2P: circ(2 M4, M4, M4, M4) y, outputs < 35 * 2P < 2^37.
KB_HD void external64(const uint32_t y[16], uint64_t v[16]) {
#pragma unroll
    for (int j = 0; j < 16; j += 4) {
        const uint64_t t01 = (uint64_t)y[j] + y[j + 1], t23 = (uint64_t)y[j + 2] + y[j + 3];
        const uint64_t t0123 = t01 + t23;
        const uint64_t t01123 = add_w(t0123, y[j + 1]), t01233 = add_w(t0123, y[j + 3]);
        v[j] = t01123 + t01;
        v[j + 1] = add_w2(t01123, y[j + 2]);
        v[j + 2] = t01233 + t23;
        v[j + 3] = add_w2(t01233, y[j]);
    }
    uint64_t sums[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        sums[k] = (v[k] + v[4 + k]) + (v[8 + k] + v[12 + k]);
    }
#pragma unroll
    for (int j = 0; j < 16; j++) v[j] += sums[j & 3];
}

// Core permutation on the internal representation: y (scale LAMBDA, each < 2P) -> v, the last
// external layer's 64-bit outputs (scale LAMBDA, < 70P); fold31(v) is again a valid y.
KB_HD void permute_lam(const uint32_t y_in[16], uint64_t v[16]) {
    uint32_t r[16], y[16];
    external64(y_in, v);
#pragma unroll
    for (int j = 0; j < 16; j++) r[j] = redc2(v[j] + kc64(FT.ext[0][j]));  // round 0: explicit constants
    // full rounds 0..2: constants of rounds 1..3 injected by the S-box
#pragma unroll
    for (int rd = 0; rd < 3; rd++) {
#pragma unroll
        for (int j = 0; j < 16; j++) y[j] = cube_inj(r[j], kc64(INJ.full[rd + 1].a[j]));
        external64(y, v);
#pragma unroll
        for (int j = 0; j < 16; j++) r[j] = redc2(v[j]);  // v < 70P: r < P + 35
    }
    // full round 3 injects partial round 0's constant (element 0 only)
#pragma unroll
    for (int j = 0; j < 16; j++) y[j] = cube_inj(r[j], kc64(INJ.part0.a[j]));
    external64(y, v);
    // partial rounds.  s_j (j >= 1) < 2P at scale LAMBDA; r0 = element 0's S-box input.
    uint32_t sj[16];
#pragma unroll
    for (int j = 1; j < 16; j++) sj[j] = fold31(v[j]);  // v < 70P -> < 2^31 + 70 * 2^24 < 2P
    uint32_t r0 = redc2(v[0]);
#pragma unroll
    for (int k = 0; k < 13; k++) {
        const uint32_t y0 = cube_l(r0);  // (0, 2P)
        uint64_t rest = sj[1];
#pragma unroll
        for (int j = 2; j < 16; j++) rest = add_w(rest, sj[j]);  // < 30P
        const uint64_t acc = add_w(rest, y0);                     // < 32P < 2^36
        // element 0: V_0 = -2, so x0' = sum_{j>=1} x_j - x0; next S-box input directly
        // (t < 33P, so r0 < P + 17)
        const uint64_t e0 = add_w(rest, 2 * kb::P - y0);
        if (k < 12) {
            r0 = redc2(e0 + kc64(FT.inr[k + 1]));
            // X = R acc (mod p), X < 2^30 R_MOD + 64 P < P (2^32 - 2P); with s_j < 2P and
            // DIAG < P the sum below stays under 2P 2^32, so the outputs are in (0, 2P)
            const uint32_t lo = (uint32_t)acc & 0x3fffffffu, hi = (uint32_t)(acc >> 30);
            const uint64_t X = mad64_ks(lo, kc32(R_MOD), prod64_ks(hi, kc32(R_2_30)));
#pragma unroll
            for (int j = 1; j < 16; j++) sj[j] = redc2(mad64_ks(sj[j], kc32(DIAG.v[j]), X));
        } else {
            // last partial round: produce the S-box inputs of full round 4 (scale LAMBDA / R):
            // redc(V_j s_j + acc + LAMBDA rc) with canonical V_j, < 2P -> one conditional subtract
            r[0] = redc2(e0 + kc64(FT.ext[4][0]));
#pragma unroll
            for (int j = 1; j < 16; j++) {
                const uint32_t t = redc2(mad64_ks(sj[j], kc32(DIAG_C.v[j]), acc + kc64(FT.ext[4][j])));
                r[j] = kb::umin(t, t - kb::P);
            }
        }
    }
    // full rounds 4..6 inject rounds 5..7; round 7 plain
#pragma unroll
    for (int rd = 4; rd < 7; rd++) {
#pragma unroll
        for (int j = 0; j < 16; j++) y[j] = cube_inj(r[j], kc64(INJ.full[rd + 1].a[j]));
        external64(y, v);
#pragma unroll
        for (int j = 0; j < 16; j++) r[j] = redc2(v[j]);
    }
#pragma unroll
    for (int j = 0; j < 16; j++) y[j] = cube_l(r[j]);
    external64(y, v);
}

// Montgomery (< P) <-> internal representation
KB_HD uint32_t to_lam(uint32_t x) { return mul_l(x, K_IN); }                 // (0, 2P), scale LAMBDA
KB_HD uint32_t from_lam(uint64_t v) { return kb::mul(fold31(v), K_OUT); }  // fold31 * K_OUT < P 2^32

KB_HD void permute(uint32_t s[16]) {
    uint32_t y[16];
    uint64_t v[16];
#pragma unroll
    for (int j = 0; j < 16; j++) y[j] = to_lam(s[j]);
    permute_lam(y, v);
#pragma unroll
    for (int j = 0; j < 16; j++) s[j] = from_lam(v[j]);
}

// PaddingFreeSponge<_,16,8,8> (overwrite mode) with the state kept in the internal
// representation between permutations: absorbing a chunk converts only the 8 new inputs, and the
// carried elements are folded (fold31) instead of converted out and back in.
struct Sponge {
    uint32_t y[16];  // scale LAMBDA, < 2P
    uint64_t v[16];  // last permutation's output layer
    KB_HD void init() {
#pragma unroll
        for (int j = 0; j < 16; j++) y[j] = 0;
    }
    // absorb a full chunk of 8 Montgomery inputs and permute
    KB_HD void absorb8(const uint32_t in[8]) {
#pragma unroll
        for (int j = 0; j < 8; j++) y[j] = to_lam(in[j]);
        permute_lam(y, v);
#pragma unroll
        for (int j = 0; j < 16; j++) y[j] = fold31(v[j]);
    }
    // absorb rate inputs already in the internal representation
    KB_HD void absorb_y(const uint32_t yin[8]) {
#pragma unroll
        for (int j = 0; j < 8; j++) y[j] = yin[j];
        permute_lam(y, v);
#pragma unroll
        for (int j = 0; j < 16; j++) y[j] = fold31(v[j]);
    }
    KB_HD void digest(uint32_t out[8]) const {
#pragma unroll
        for (int j = 0; j < 8; j++) out[j] = kb::mul(y[j], K_OUT);  // y = fold31(v) < 2^32
    }
};

// Sponge hash of n Montgomery elements ld(0..n-1) (PaddingFreeSponge, overwrite mode: a partial
// last chunk leaves the rest of the rate as the previous permutation wrote it; n = 0 -> zeros).
// The next chunk is loaded before the current one is permuted, so global-load latency overlaps
// the permutation.
template <class Load>
KB_HD void sponge_hash(int n, const Load &ld, uint32_t out[8]) {
    Sponge sp;
    sp.init();
    if (n <= 0) {
        sp.digest(out);
        return;
    }
    // loads are unconditional (index clamped to n - 1): a conditional load is a branch, and the
    // copy at its join point would force the wait before the permutation
    auto ldc = [&](int k) { return ld(k < n ? k : n - 1); };
    uint32_t nxt[8];
#pragma unroll
    for (int k = 0; k < 8; k++) nxt[k] = ldc(k);
    int base = 0;
    for (; base + 8 <= n; base += 8) {
        uint32_t in[8];
#pragma unroll
        for (int k = 0; k < 8; k++) in[k] = nxt[k];
#pragma unroll
        for (int k = 0; k < 8; k++) nxt[k] = ldc(base + 8 + k);
#ifdef __HIP_DEVICE_COMPILE__
        __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the permutation
#endif
        sp.absorb8(in);
    }
    if (base < n) {
        uint32_t yin[8];
#pragma unroll
        for (int k = 0; k < 8; k++) yin[k] = base + k < n ? to_lam(nxt[k]) : sp.y[k];
        sp.absorb_y(yin);
    }
    sp.digest(out);
}

// TruncatedPermutation<_,2,8,16>: perm(l || r)[0..8]
KB_HD void compress(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) {
    uint32_t s[16];
#pragma unroll
    for (int i = 0; i < 8; i++) { s[i] = l[i]; s[8 + i] = r[i]; }
    permute(s);
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = s[i];
}

}  // namespace p2

// Latency-optimised permutation: one state spread over a 16-lane row of the wavefront (lane l
// holds s_l, 4 states per wave).  The linear layers become cross-lane DPP adds, so one
// permutation is a ~5x shorter dependent chain than the one-thread form; it costs ~3x more lane
// work, so it is used only where few permutations are in flight (tree tops, small levels,
// transcript).  Every lane of the wave must execute it (DPP reads neighbour lanes).
namespace p2x16 {
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
constexpr int QP(int a, int b, int c, int d) { return a | (b << 2) | (c << 4) | (d << 6); }
constexpr int ROR(int k) { return 0x120 + k; }
constexpr int BCAST0 = 0x150;  // row_newbcast:0 (lane 0 of each 16-lane row to the whole row)

// external layer: M4 = circ(2,3,1,1) per 4-lane block (n_j = quad_sum + x_j + 2 x_{j+1}),
// then the column sums over the four blocks (lanes j, j+4, j+8, j+12)
__device__ __forceinline__ uint32_t external(uint32_t x) {
    using namespace kb;
    const uint32_t q = add(x, dpp<QP(1, 0, 3, 2)>(x));
    const uint32_t S = add(q, dpp<QP(2, 3, 0, 1)>(q));
    const uint32_t n = add(add(S, x), dbl(dpp<QP(1, 2, 3, 0)>(x)));
    uint32_t c = add(n, dpp<ROR(4)>(n));
    c = add(c, dpp<ROR(8)>(c));
    return add(n, c);
}

__device__ __constant__ inline p2::RcTable kRc = p2::RC;
__device__ __constant__ inline p2::DiagTable kDiag = p2::DIAG;

// per-lane round constants (full rounds) and internal diagonal entry; l = lane within the row
struct Lane {
    uint32_t rc[8];
    uint32_t dg;
    int l;
};
__device__ __forceinline__ Lane lane_consts(int l) {
    Lane c;
#pragma unroll
    for (int r = 0; r < 8; r++) c.rc[r] = kRc.ext[r][l];
    c.dg = kDiag.v[l];
    c.l = l;
    return c;
}

__device__ __forceinline__ uint32_t permute(uint32_t x, const Lane &c) {
    using namespace kb;
    x = external(x);
#pragma unroll
    for (int r = 0; r < 4; r++) x = external(cube(add(x, c.rc[r])));
#pragma unroll
    for (int r = 0; r < 13; r++) {
        // the row sum of the lanes other than 0 does not wait for lane 0's s-box: it runs beside the
        // cube, and lane 0's s-box output joins it by one broadcast (row_newbcast:0)
        const uint32_t y = cube(add(x, p2::RC.inr[r]));
        uint32_t s = (c.l == 0) ? 0u : x;
        s = add(s, dpp<ROR(1)>(s));
        s = add(s, dpp<ROR(2)>(s));
        s = add(s, dpp<ROR(4)>(s));
        s = add(s, dpp<ROR(8)>(s));
        s = add(s, dpp<BCAST0>(y));
        x = add(mul((c.l == 0) ? y : x, c.dg), s);
    }
#pragma unroll
    for (int r = 4; r < 8; r++) x = external(cube(add(x, c.rc[r])));
    return x;
}
}  // namespace p2x16
