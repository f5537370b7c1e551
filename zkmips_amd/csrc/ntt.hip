// Coset LDE for KoalaBear on gfx950: column-major, LDS-tiled multi-pass radix-2 NTT.
//
// Semantics (TwoAdicFriPcs::commit = coset_lde_batch + bit_reverse_rows; call sites
// crates/stark/src/prover.rs:277,403,497; row i <-> point shift * w_{2n}^{rev(i)}, pinned by
// crates/recursion/circuit/src/fri.rs:134-150).
//
// Algorithm per column of height N = 2^L, blowup 2:
//   1. iNTT as DIF (natural evaluations in -> bit-reversed coefficients), in place.
//   2. The blowup-2 LDE in bit-reversed order is [bitrev(E0) | bitrev(E1)] with
//      E0 = NTT_N(c_k s^k / N) and E1 = NTT_N(c_k (s w_2N)^k / N): one contiguous DIT pass
//      applies both twists to the bit-reversed coefficients and starts both transforms.
//   3. DIT passes (bit-reversed in -> natural out); the last pass writes every output element
//      to its bit-reversed row, so the LDE is produced without a separate permutation pass.
// Passes: the lowest <= 13 bits in one contiguous LDS tile (8192 elements), the remaining bits
// in strided passes of <= 9 bits over 32/64-column-wide tiles (128/256 B coalesced rows); the
// inverse's last pass, the twists and the forward's first pass are one fused kernel, so a 2^22
// column costs 3 HBM passes.  Butterflies run in radix-8 register groups (stage_group).
#include "internal.hpp"
#include "prof.hpp"

namespace zkm {

using namespace kb;

static constexpr int NT = 256;          // threads per workgroup

// ------------------------------------------------------------------ layout conversion
__global__ void k_to_col_major(const uint32_t *__restrict__ in, uint64_t h, uint64_t w, int mont_in,
                               uint32_t *__restrict__ out) {
    __shared__ uint32_t tile[64][65];
    uint64_t r0 = (uint64_t)blockIdx.x * 64, c0 = (uint64_t)blockIdx.y * 64;
    int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
    for (int i = ty; i < 64; i += 4) {
        uint64_t r = r0 + i, c = c0 + tx;
        uint32_t v = 0;
        if (r < h && c < w) {
            v = in[r * w + c];
            v = mont_in ? v : to_mont(v);
        }
        tile[i][tx] = v;
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) {
        uint64_t c = c0 + i, r = r0 + tx;
        if (r < h && c < w) out[c * h + r] = tile[tx][i];
    }
}

__global__ void k_from_col_major(const uint32_t *__restrict__ in, uint64_t h, uint64_t w,
                                 uint32_t *__restrict__ out) {
    __shared__ uint32_t tile[64][65];
    uint64_t r0 = (uint64_t)blockIdx.x * 64, c0 = (uint64_t)blockIdx.y * 64;
    int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int i = ty; i < 64; i += 4) {
        uint64_t c = c0 + i, r = r0 + tx;
        tile[i][tx] = (r < h && c < w) ? from_mont(in[c * h + r]) : 0u;
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) {
        uint64_t r = r0 + i, c = c0 + tx;
        if (r < h && c < w) out[r * w + c] = tile[tx][i];
    }
}

// Narrow matrices (w <= 128): a block takes 64 whole rows, so its read is one contiguous span of
// 64 w words (the 64x64-tile kernel reads 4 w-byte rows in 256-byte pieces and, for w = 67, spends
// a second tile column on 3 words per row); each column then leaves as one 256-byte segment.
// The tile is sized to the matrix (w x 65 words of dynamic LDS, 17.4 KB for w = 67): a fixed 128-column tile
// (33 KB) held a CU to four blocks' loads in flight.
static constexpr int TW_ROWS = 64, TW_MAXW = 128;
__global__ __launch_bounds__(NT) void k_to_col_major_rows(const uint32_t *__restrict__ in, uint64_t h, uint32_t w,
                                                          int mont_in, uint32_t *__restrict__ out) {
    extern __shared__ uint32_t tile[];  // [c][r], pitch 65: conflict-free both ways
    const uint64_t nblk = (h + TW_ROWS - 1) / TW_ROWS;
    for (uint64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {  // grid-stride: a capped grid for host sources
    if (blk != blockIdx.x) __syncthreads();  // the previous block's tile has been written out
    const uint64_t r0 = blk * TW_ROWS;
    const uint32_t nr = (uint32_t)(h - r0 < TW_ROWS ? h - r0 : TW_ROWS);
    const uint32_t n = nr * w;
    const uint32_t *src = in + r0 * w;
    constexpr int PER = TW_MAXW * TW_ROWS / NT;  // 32 elements per thread at most
    uint32_t v[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {  // all loads issued before the first LDS store
        const uint32_t i = threadIdx.x + k * NT;
        v[k] = i < n ? src[i] : 0u;
    }
    const float rw = 1.0f / (float)w;  // i / w by a float reciprocal, corrected (i < 2^13)
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const uint32_t i = threadIdx.x + k * NT;
        if (i < n) {
            uint32_t r = (uint32_t)((float)i * rw);
            if (r * w > i) r--;
            else if ((r + 1) * w <= i) r++;
            const uint32_t c = i - r * w;
            tile[c * (TW_ROWS + 1) + r] = mont_in ? v[k] : to_mont(v[k]);
        }
    }
    __syncthreads();
#pragma unroll 8
    for (uint32_t i = threadIdx.x; i < w * TW_ROWS; i += NT) {
        const uint32_t c = i / TW_ROWS, r = i % TW_ROWS;
        if (r < nr) out[(uint64_t)c * h + r0 + r] = tile[c * (TW_ROWS + 1) + r];
    }
    }
}

void launch_to_col_major(const uint32_t *d_in, uint64_t h, uint64_t w, bool mont_in, uint32_t *d_out, hipStream_t s,
                         unsigned max_grid) {
    if (!h || !w) return;
    if (w <= TW_MAXW) {
        uint64_t g = (h + TW_ROWS - 1) / TW_ROWS;
        if (max_grid && g > max_grid) g = max_grid;
        hipLaunchKernelGGL(k_to_col_major_rows, dim3((unsigned)g), dim3(NT), (unsigned)(w * (TW_ROWS + 1) * 4), s,
                           d_in, h, (uint32_t)w, (int)mont_in, d_out);
        HIP_CHECK(hipGetLastError());
        return;
    }
    dim3 g((unsigned)((h + 63) / 64), (unsigned)((w + 63) / 64));
    hipLaunchKernelGGL(k_to_col_major, g, dim3(NT), 0, s, d_in, h, w, (int)mont_in, d_out);
    HIP_CHECK(hipGetLastError());
}
void launch_from_col_major(const uint32_t *d_in, uint64_t h, uint64_t w, uint32_t *d_out, hipStream_t s) {
    if (!h || !w) return;
    dim3 g((unsigned)((h + 63) / 64), (unsigned)((w + 63) / 64));
    hipLaunchKernelGGL(k_from_col_major, g, dim3(NT), 0, s, d_in, h, w, d_out);
    HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------ twiddles
// tw[h + j] = w_{2h}^j for h = 2^k, 0 <= j < h (w = forward or inverse root).
__global__ void k_build_twiddles(uint32_t *tw, uint32_t *twi, int log_max, const uint32_t *roots,
                                 const uint32_t *iroots) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) { tw[0] = 0; twi[0] = 0; return; }
    if (i >= (1ull << log_max)) return;
    int k = 63 - __builtin_clzll(i);  // h = 2^k
    uint64_t j = i - (1ull << k);
    tw[i] = pow(roots[k + 1], j);
    twi[i] = pow(iroots[k + 1], j);
}

// rows for layouts SE = 2, 32, 512 (offsets 0, 2, 34 rows), one row per (SE, off < SE):
// k = 0: w_{2SE}^off; k = 1,2: w_{4SE}^{off + SE m}; k = 3..6: w_{8SE}^..; k = 7..14: w_{16SE}^..
static constexpr uint32_t TT_WORDS = (2 + 32 + 512) * 16;
__device__ __forceinline__ uint32_t tt_row(int SE) { return SE == 2 ? 0u : SE == 32 ? 2u : 34u; }
__global__ void k_build_tile_tw(const uint32_t *tw, const uint32_t *twi, uint32_t *tt, uint32_t *tti) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= TT_WORDS) return;
    const uint32_t row = i >> 4, k = i & 15;
    const uint32_t SE = row < 2 ? 2 : row < 34 ? 32 : 512;
    const uint32_t off = row - (SE == 2 ? 0 : SE == 32 ? 2 : 34);
    if (k == 15) { tt[i] = 0; tti[i] = 0; return; }
    const uint32_t st = k == 0 ? 0 : k < 3 ? 1 : k < 7 ? 2 : 3;
    const uint32_t m = k - ((1u << st) - 1);
    const uint32_t idx = (SE << st) + off + SE * m;
    tt[i] = tw[idx];
    tti[i] = twi[idx];
}

void build_twiddles(Ctx &c, int log_max) {
    size_t n = 1ull << log_max;
    HIP_CHECK(hipMalloc((void **)&c.tw_fwd, n * 4));
    HIP_CHECK(hipMalloc((void **)&c.tw_inv, n * 4));
    uint32_t roots[32], iroots[32];
    for (int k = 0; k <= TWO_ADICITY; k++) { roots[k] = two_adic_gen(k); iroots[k] = inv(roots[k]); }
    uint32_t *d_r;
    HIP_CHECK(hipMalloc((void **)&d_r, 64 * 4));
    HIP_CHECK(hipMemcpy(d_r, roots, 32 * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_r + 32, iroots, 32 * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_build_twiddles, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, 0, c.tw_fwd, c.tw_inv,
                       log_max, d_r, d_r + 32);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipFree(d_r));
    c.tw_log = log_max;
    // per-thread twiddle rows of the 8192-point register tiles (t13::net16)
    HIP_CHECK(hipMalloc((void **)&c.tt_fwd, 2 * TT_WORDS * 4));
    c.tt_inv = c.tt_fwd + TT_WORDS;
    hipLaunchKernelGGL(k_build_tile_tw, dim3((TT_WORDS + NT - 1) / NT), dim3(NT), 0, 0, c.tw_fwd, c.tw_inv, c.tt_fwd,
                       c.tt_inv);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipDeviceSynchronize());
}

// ------------------------------------------------------------------ tile stage engine
// A tile lives in LDS as x[r * LD + t] (R rows, T columns, row pitch LD).  Row r, column t holds
// global index base + r*S + c0 + t, so the butterfly of a stage with half-size h = hr*S at lower
// row r uses w_{2h}^{(r mod hr)*S + c0 + t} = tw[h + (r mod hr)*S + c0 + t] (all indices < 2^24).
// Stages are processed G <= 3 at a time: each thread holds the 2^G elements a group of G stages
// touches in registers, so a tile makes one LDS round trip per 3 stages instead of per stage.
// LDS address of tile element (row r, column t).  Strided tiles (SWS >= 0) XOR-swizzle the
// column with row bits SWS..SWS+4, so that the bit-reversed row walk of MODE_BITREV_OUT (32 lanes
// on rows 2^SWS apart) hits 32 distinct banks; row-major walks stay conflict-free.
template <int LD, int SWS>
__device__ __forceinline__ int tile_at(int r, int t) {
    if constexpr (SWS < 0) return r * LD + t;
    else return r * LD + (t ^ ((r >> SWS) & 31));
}

template <int G, int T, int LD, bool DIT, int SWS, int NTH>
__device__ __forceinline__ void stage_group(uint32_t *x, int R, int lc, const uint32_t *__restrict__ tw, uint32_t S,
                                            uint32_t c0) {
    constexpr int E = 1 << G;
    const int hrc = 1 << lc;
    const int ngroups = (R * T) >> G;
    for (int g = threadIdx.x; g < ngroups; g += NTH) {
        const int t = g & (T - 1);
        const int q = g / T;
        const int rlow = q & (hrc - 1);
        const int r0 = ((q >> lc) << (lc + G)) | rlow;
        uint32_t v[E];
#pragma unroll
        for (int k = 0; k < E; k++) v[k] = x[tile_at<LD, SWS>(r0 + k * hrc, t)];
        const uint32_t jb = (uint32_t)rlow * S + c0 + (uint32_t)t;
        const uint32_t step = (uint32_t)hrc * S;
        if (DIT) {
#pragma unroll
            for (int b = 0; b < G; b++) {
                const uint32_t h = step << b;
#pragma unroll
                for (int k = 0; k < E; k++) {
                    if (k & (1 << b)) continue;
                    const uint32_t w = tw[h + jb + (uint32_t)(k & ((1 << b) - 1)) * step];
                    const uint32_t u = v[k], y = mul(v[k + (1 << b)], w);
                    v[k] = add(u, y);
                    v[k + (1 << b)] = sub(u, y);
                }
            }
        } else {
#pragma unroll
            for (int b = G - 1; b >= 0; b--) {
                const uint32_t h = step << b;
#pragma unroll
                for (int k = 0; k < E; k++) {
                    if (k & (1 << b)) continue;
                    const uint32_t w = tw[h + jb + (uint32_t)(k & ((1 << b) - 1)) * step];
                    const uint32_t u = v[k], y = v[k + (1 << b)];
                    v[k] = add(u, y);
                    v[k + (1 << b)] = mul(sub(u, y), w);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < E; k++) x[tile_at<LD, SWS>(r0 + k * hrc, t)] = v[k];
    }
    __syncthreads();
}

// All LOGR stages of a tile: DIT bottom-up (half-sizes 1,2,4,...), DIF top-down.
template <int LOGR, int T, int LD, bool DIT, int SWS, int NTH>
__device__ __forceinline__ void tile_stages(uint32_t *x, const uint32_t *__restrict__ tw, uint32_t S, uint32_t c0) {
    constexpr int R = 1 << LOGR;
    if (DIT) {
        int lc = 0;
        for (; lc + 3 <= LOGR; lc += 3) stage_group<3, T, LD, true, SWS, NTH>(x, R, lc, tw, S, c0);
        if (LOGR - lc == 2) stage_group<2, T, LD, true, SWS, NTH>(x, R, lc, tw, S, c0);
        else if (LOGR - lc == 1) stage_group<1, T, LD, true, SWS, NTH>(x, R, lc, tw, S, c0);
    } else {
        int rem = LOGR;
        for (; rem >= 3; rem -= 3) stage_group<3, T, LD, false, SWS, NTH>(x, R, rem - 3, tw, S, c0);
        if (rem == 2) stage_group<2, T, LD, false, SWS, NTH>(x, R, 0, tw, S, c0);
        else if (rem == 1) stage_group<1, T, LD, false, SWS, NTH>(x, R, 0, tw, S, c0);
    }
}

// the LDE's intermediate stores (strided MODE_PLAIN passes and the fused tile's output, read again by the next
// pass) keep the default policy, so that 8-column batches of a 2^22 trace find part of them in the Infinity
// Cache: 2^22 x 64 LDE 3.49 -> 3.43 ms, shard resident 26.46 -> 26.04 ms (profiles/r05_lde_mall_ab.txt);
// -DZKM_LDE_MID_AUX=2 makes them non-temporal like the final passes' stores
#ifndef ZKM_LDE_MID_AUX
#define ZKM_LDE_MID_AUX 0
#endif

struct ColMap {
    // virtual column v -> offset (v / nsub) * col_stride + (v % nsub) * sub_stride
    uint64_t col_stride, sub_stride;
    uint32_t nsub;
    __device__ __forceinline__ uint64_t off(uint32_t v) const {
        return (uint64_t)(v / nsub) * col_stride + (uint64_t)(v % nsub) * sub_stride;
    }
};

struct Twist {
    const uint32_t *lo0, *hi0, *lo1, *hi1;
    // 8192-tile form (k_lde_fused13s): f_e(rev_L(b 2^13 + i)) = g_e[b] * u_e[t][j] for element j of
    // thread t in layout L2 (i = lay_idx<2>(t, j)); u_e: 512 x 16, g_e: 2^(L-13) entries
    const uint32_t *u0, *g0, *u1, *g1;
    __device__ __forceinline__ uint32_t f(int e, uint32_t k) const {
        return e ? mul(hi1[k >> 12], lo1[k & 4095]) : mul(hi0[k >> 12], lo0[k & 4095]);
    }
};

// Strided-pass output modes: MODE_BITREV_OUT (last DIT pass, R*S == N): natural n = r*S + c goes to row rev_L(n);
// MODE_TWIST_OUT (last DIT pass of an inverse transform): natural coefficient n goes to both LDE halves multiplied by
// the coset twists f_0(n), f_1(n).
enum PassMode { MODE_PLAIN = 0, MODE_BITREV_OUT = 1, MODE_TWIST_OUT = 2 };

// Contiguous pass over blocks of R consecutive elements (bit-reversed-input pipeline):
//   MODE_PLAIN: stages only; MODE_TWIST_OUT: DIT (inverse) then twisted writes to both halves.
template <int LOGR, bool DIT, int NTH>
__global__ __launch_bounds__(NTH) void k_ntt_contig(const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md,
                                                   const uint32_t *__restrict__ tw, int mode, Twist tws,
                                                   uint64_t dst_half) {
    constexpr int R = 1 << LOGR;
    __shared__ uint32_t x[R];
    const uint32_t base = blockIdx.x * (uint32_t)R;
    const uint32_t *sp = src + ms.off(blockIdx.y) + base;
    for (int i = threadIdx.x; i < R; i += NTH) x[i] = sp[i];
    __syncthreads();
    tile_stages<LOGR, 1, 1, DIT, -1, NTH>(x, tw, 1, 0);
    uint32_t *dp = dst + md.off(blockIdx.y);
    if (mode == MODE_TWIST_OUT) {
        for (int i = threadIdx.x; i < R; i += NTH) {
            const uint32_t n = base + i;
            dp[n] = mul(x[i], tws.f(0, n));
            dp[dst_half + n] = mul(x[i], tws.f(1, n));
        }
    } else {
        for (int i = threadIdx.x; i < R; i += NTH) dp[base + i] = x[i];
    }
}

// Fused middle of the natural-input LDE: the inverse NTT's last (contiguous, DIF) pass, the two
// coset twists, and the first (contiguous, DIT) pass of both forward transforms, on one tile.
// The DIF output tile (bit-reversed coefficients) is exactly the DIT input tile, so the
// coefficients never round-trip through HBM.  bitrev_out: the whole transform fits the tile.
template <int LOGR, int NTH>
__global__ __launch_bounds__(NTH) void k_lde_fused(const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md, int L,
                                                  const uint32_t *__restrict__ tw_inv,
                                                  const uint32_t *__restrict__ tw_fwd, Twist tws, uint64_t dst_half,
                                                  int bitrev_out) {
    constexpr int R = 1 << LOGR;
    __shared__ uint32_t a[R];
    __shared__ uint32_t x[R];
    const uint32_t base = blockIdx.x * (uint32_t)R;
    const uint32_t *sp = src + ms.off(blockIdx.y) + base;
    for (int i = threadIdx.x; i < R; i += NTH) a[i] = sp[i];
    __syncthreads();
    tile_stages<LOGR, 1, 1, false, -1, NTH>(a, tw_inv, 1, 0);
    uint32_t *dcol = dst + md.off(blockIdx.y);
    for (int e = 0; e < 2; e++) {
        for (int i = threadIdx.x; i < R; i += NTH) x[i] = mul(a[i], tws.f(e, rev_bits(base + i, L)));
        __syncthreads();
        tile_stages<LOGR, 1, 1, true, -1, NTH>(x, tw_fwd, 1, 0);
        uint32_t *dp = dcol + (uint64_t)e * dst_half;
        if (!bitrev_out) {
            for (int i = threadIdx.x; i < R; i += NTH) dp[base + i] = x[i];
        } else {
            for (int i = threadIdx.x; i < R; i += NTH) dp[i] = x[rev_bits((uint32_t)i, LOGR)];
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ 8192-point register tiles
// One workgroup of 512 threads holds an 8192-element tile in registers, 16 elements per thread,
// in one of three layouts (index of element j of thread t):
//   L512: t + 512 j                       stages h = 512..4096 in registers
//   L32 : (t >> 5) * 512 + (t & 31) + 32 j  stages h = 32..256
//   L2  : (t >> 1) * 32  + (t & 1)  + 2 j   stages h = 2..16; h = 1 pairs lanes t, t^1 (DPP)
// Layout changes go through a 34 KB LDS tile whose rows are padded (sw13) so that every layout's
// ds_read_b32 / ds_write_b32 is conflict-free within each 32-lane half.
// Butterflies: DIF x' = x + y, y' = (x - y) w;  DIT t = y w, x' = x + t, y' = x - t;
// w = w_{2h}^{i mod h} from tw[h + (i mod h)].
namespace t13 {
constexpr int NTH = 512;

// padded LDS word address: row pitch 34 per 32 words.  For every layout, element j's address is a
// per-thread base plus a constant (foldable into the ds_* immediate offset), and each 32-lane
// half of a wave hits 32 distinct banks: L512 and L32 walk consecutive words; L2 lanes 2m + b
// land on bank b + 2m + 2j.
__device__ __forceinline__ uint32_t sw13(uint32_t idx) { return idx + 2 * (idx >> 5); }
constexpr uint32_t LDS13 = 8192 + 2 * 256;

template <int SE>
__device__ __forceinline__ uint32_t lay_idx(uint32_t t, uint32_t j) {
    if constexpr (SE == 512) return t + 512 * j;
    else if constexpr (SE == 32) return (t >> 5) * 512 + (t & 31) + 32 * j;
    else return (t >> 1) * 32 + (t & 1) + 2 * j;
}
template <int SE>
__device__ __forceinline__ uint32_t lay_off(uint32_t t) {  // (index of element 0) mod SE
    if constexpr (SE == 512) return (uint32_t)t;
    else if constexpr (SE == 32) return (uint32_t)(t & 31);
    else return (uint32_t)(t & 1);
}

// the four in-register stages of a layout with element stride SE
template <bool DIT, int SE>
__device__ __forceinline__ void net16(uint32_t v[16], uint32_t off, const uint32_t *__restrict__ tt) {
    // this thread's 15 twiddles, contiguous (k_build_tile_tw)
    uint32_t w16[16];
    const uint4 *row = (const uint4 *)(tt + (tt_row(SE) + off) * 16);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint4 r = row[q];
        w16[4 * q] = r.x; w16[4 * q + 1] = r.y; w16[4 * q + 2] = r.z; w16[4 * q + 3] = r.w;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int st = DIT ? q : 3 - q;  // DIT: h = SE, 2SE, 4SE, 8SE; DIF: reverse
        const int span = 1 << st;
#pragma unroll
        for (int m = 0; m < span; m++) {
            const uint32_t w = w16[span - 1 + m];
#pragma unroll
            for (int j = m; j < 16; j += 2 * span) {
                const uint32_t x = v[j], y = v[j + span];
                if (DIT) {
                    const uint32_t tt = mul(y, w);  // y may be lazy (< 2P): y w < P 2^32
                    if (q < 3 && ((j >> (st + 1)) & 1)) {
                        // both outputs are the multiplied operand of the next stage: leave them
                        // unreduced in [0, 2P)
                        v[j] = x + tt;
                        v[j + span] = x + (P - tt);
                    } else {
                        v[j] = add(x, tt);
                        v[j + span] = sub(x, tt);
                    }
                } else {
                    v[j] = add(x, y);
                    v[j + span] = mul(x + (P - y), w);  // (0, 2P) operand: no reduction before the product
                }
            }
        }
    }
}

// h = 1 stage (w = 1 for both DIF and DIT): lanes t (even) and t^1 (odd) exchange by DPP
__device__ __forceinline__ void stage_h1(uint32_t v[16], bool odd) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint32_t nb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[j], 0xB1 /*quad_perm [1,0,3,2]*/, 0xF,
                                                                  0xF, false);
        const uint32_t neg_or_v = odd ? P - v[j] : v[j];  // odd lane: nb - v = nb + (P - v)
        v[j] = add(nb, neg_or_v);
    }
}

// sw13(lay_idx<SE>(t, j)) written as a per-thread base plus a constant stride (544, 34 or 2 words): element j's
// LDS address is the base plus an immediate offset, one base register per layout, which the compiler does not
// derive from sw13's shift by itself
template <int SE>
__device__ __forceinline__ uint32_t lds_base(uint32_t t) {
    if constexpr (SE == 512) return t + 2 * (t >> 5);
    else if constexpr (SE == 32) return (t >> 5) * 544 + (t & 31);
    else return (t >> 1) * 34 + (t & 1);
}
template <int SE> constexpr uint32_t LDS_STRIDE = SE == 512 ? 544 : SE == 32 ? 34 : 2;
template <int SE>
__device__ __forceinline__ void to_lds(uint32_t *x, const uint32_t v[16], uint32_t t) {
    uint32_t *p = x + lds_base<SE>(t);
#pragma unroll
    for (int j = 0; j < 16; j++) p[LDS_STRIDE<SE> * j] = v[j];
}
template <int SE>
__device__ __forceinline__ void from_lds(const uint32_t *x, uint32_t v[16], uint32_t t) {
    const uint32_t *p = x + lds_base<SE>(t);
#pragma unroll
    for (int j = 0; j < 16; j++) v[j] = p[LDS_STRIDE<SE> * j];
}

// Exchange ordering between the layouts.  L512 spreads a wave's elements over the whole tile, but L32
// and L2 of wave w both hold exactly tile elements [1024 w, 1024 w + 1024) (a wave is threads 64 w ..
// 64 w + 63: L32 rows t >> 5 in {2w, 2w + 1}, L2 groups t >> 1 in [32 w, 32 w + 32)), so the L32 <-> L2
// exchanges only touch the wave's own LDS words: a DS instruction stream of one wave executes in
// order, and the compiler only has to keep the accesses in program order -- no workgroup barrier.
// WL = false keeps workgroup barriers there instead.
template <bool WL>
__device__ __forceinline__ void own_sync() {
    if constexpr (WL) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

// DIF over all 13 stages: v in L512 (natural) -> v in L2 (bit-reversed within the tile)
template <bool WL = false>
__device__ __forceinline__ void dif13(uint32_t v[16], uint32_t *x, uint32_t t, const uint32_t *__restrict__ tw) {
    net16<false, 512>(v, lay_off<512>(t), tw);
    to_lds<512>(x, v, t);
    __syncthreads();
    from_lds<32>(x, v, t);
    net16<false, 32>(v, lay_off<32>(t), tw);
    own_sync<WL>();
    to_lds<32>(x, v, t);
    own_sync<WL>();
    from_lds<2>(x, v, t);
    net16<false, 2>(v, lay_off<2>(t), tw);
    stage_h1(v, t & 1);
    own_sync<WL>();  // LDS free for the next user (WL: its next writes are this wave's own L2 / L32 words)
}

}  // namespace t13

// TILED: source and destination tile-major (k_ntt_s9b TILE): element e of 8192-run b (b < 512) at
// (e / 32) * 16384 + b * 32 + e % 32 -- the strided passes on either side then move contiguous 64 KB tiles,
// and this VALU-bound kernel takes the 128-B segments instead
__device__ __forceinline__ uint32_t tiled13(uint32_t b, uint32_t t, uint32_t j) {
    return ((t >> 5) + 16 * j) * 16384u + b * 32u + (t & 31);
}

// Fused middle of the natural-input LDE for transforms larger than one tile (k_lde_fused13s): the iNTT's last 13
// (DIF) stages, both coset twists and the forward transforms' first 13 (DIT) stages.  The coefficients stay in
// registers while each coset is twisted, transformed and stored in turn through ONE 34.8 KB LDS tile: 64 VGPRs,
// four workgroups (32 waves) per CU.  Against round 5's two-coset form (both cosets in registers at once, twice
// the LDS; deleted after its A/B, git history keeps it): per 8-column batch of a 2^22 LDE 202 vs 208 us, LDE
// 2^22 x 67 -0.8 % (profiles/r05_t13_seq_ab.txt); the tile is at ~0.74 of the VALU issue rate.
namespace t13 {
// net16 with each stage's twiddles loaded just before the stage (at most 8 live instead of 15)
template <bool DIT, int SE>
__device__ __forceinline__ void net16s(uint32_t v[16], uint32_t off, const uint32_t *__restrict__ tt) {
    const uint32_t *row = tt + (tt_row(SE) + off) * 16;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int st = DIT ? q : 3 - q;
        const int span = 1 << st;
        uint32_t w[8];
#pragma unroll
        for (int m = 0; m < span; m++) w[m] = row[span - 1 + m];
#pragma unroll
        for (int m = 0; m < span; m++) {
#pragma unroll
            for (int j = m; j < 16; j += 2 * span) {
                // at most four butterflies' products in flight (the 80-register budget; other waves hide the latency)
                if (((j >> (st + 1)) * span + m) % 4 == 0) __builtin_amdgcn_sched_barrier(0);
                const uint32_t a = v[j], b = v[j + span];
                if (DIT) {
                    const uint32_t tt = mul(b, w[m]);
                    if (q < 3 && ((j >> (st + 1)) & 1)) {
                        v[j] = a + tt;
                        v[j + span] = a + (P - tt);
                    } else {
                        v[j] = add(a, tt);
                        v[j + span] = sub(a, tt);
                    }
                } else {
                    v[j] = add(a, b);
                    v[j + span] = mul(a + (P - b), w[m]);
                }
            }
        }
    }
}
template <bool WL>
__device__ __forceinline__ void dit13(uint32_t v[16], uint32_t *x, uint32_t t, const uint32_t *__restrict__ tw) {
    stage_h1(v, t & 1);
    net16s<true, 2>(v, lay_off<2>(t), tw);
    to_lds<2>(x, v, t);
    own_sync<WL>();
    from_lds<32>(x, v, t);
    net16s<true, 32>(v, lay_off<32>(t), tw);
    own_sync<WL>();
    to_lds<32>(x, v, t);
    __syncthreads();
    from_lds<512>(x, v, t);
    net16s<true, 512>(v, lay_off<512>(t), tw);
}
}  // namespace t13

// ------------------------------------------------------------------ 512-row strided register tiles
// One workgroup of 1024 threads: 512 rows (stride S) x 32 consecutive columns, 16 elements per
// thread as two radix-8 networks.  Lane -> column (t = tid & 31), so every global access moves
// whole 128-B row segments and every row-major LDS access is conflict-free; the columns are
// XOR-swizzled by row bits 4..8 so that the bit-reversed column walk of the BITREV output is too.
// Layouts (u = tid >> 5, network n in {0,1}, element k < 8, g = 2u + n):
//   LH: row (u + 32n) + 64k          stages h_r = 64, 128, 256 rows
//   LM: row (g >> 3) * 64 + (g & 7) + 8k   h_r = 8, 16, 32
//   LL: row 8g + k                   h_r = 1, 2, 4
// The butterfly at rows (r, r + h_r) of the transform uses w_{2h}^{(r mod h_r) S + c0 + t}, h = h_r S.
namespace s9 {
constexpr int NTH = 1024;
enum { LH = 0, LM = 1, LL = 2 };

__device__ __forceinline__ uint32_t at(uint32_t r, uint32_t t) { return r * 32 + (t ^ ((r >> 4) & 31)); }

template <int LAY>
__device__ __forceinline__ uint32_t row0(uint32_t u, int n) {
    const uint32_t g = 2 * u + n;
    if constexpr (LAY == LH) return u + 32 * n;
    else if constexpr (LAY == LM) return (g >> 3) * 64 + (g & 7);
    else return 8 * g;
}
template <int LAY> constexpr uint32_t RS = LAY == LH ? 64 : LAY == LM ? 8 : 1;

// three stages of one network; off = row0 mod RS
template <bool DIT, int LAY>
__device__ __forceinline__ void net8(uint32_t *v, uint32_t off, uint32_t S, uint32_t ct,
                                     const uint32_t *__restrict__ tw) {
    constexpr uint32_t rs = RS<LAY>;
#pragma unroll
    for (int q = 0; q < 3; q++) {
        const int st = DIT ? q : 2 - q;
        const int span = 1 << st;
        const uint32_t h = (rs << st) * S;
#pragma unroll
        for (int m = 0; m < span; m++) {
            const uint32_t w = tw[h + (off + rs * m) * S + ct];
#pragma unroll
            for (int k = m; k < 8; k += 2 * span) {
                const uint32_t a = v[k], b = v[k + span];
                if (DIT) {
                    const uint32_t tt = mul(b, w);
                    if (q < 2 && ((k >> (st + 1)) & 1)) {  // next stage multiplies both: lazy [0, 2P)
                        v[k] = a + tt;
                        v[k + span] = a + (P - tt);
                    } else {
                        v[k] = add(a, tt);
                        v[k + span] = sub(a, tt);
                    }
                } else {
                    v[k] = add(a, b);
                    v[k + span] = mul(a + (P - b), w);
                }
            }
        }
    }
}

template <bool DIT, int LAY>
__device__ __forceinline__ void nets(uint32_t v[16], uint32_t u, uint32_t S, uint32_t ct,
                                     const uint32_t *__restrict__ tw) {
#pragma unroll
    for (int n = 0; n < 2; n++) net8<DIT, LAY>(v + 8 * n, row0<LAY>(u, n) % RS<LAY>, S, ct, tw);
}
template <int LAY>
__device__ __forceinline__ void to_lds(uint32_t *x, const uint32_t v[16], uint32_t u, uint32_t t) {
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[at(row0<LAY>(u, n) + RS<LAY> * k, t)] = v[8 * n + k];
}
template <int LAY>
__device__ __forceinline__ void from_lds(const uint32_t *x, uint32_t v[16], uint32_t u, uint32_t t) {
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int k = 0; k < 8; k++) v[8 * n + k] = x[at(row0<LAY>(u, n) + RS<LAY> * k, t)];
}
}  // namespace s9

// 9 strided stages (rows at stride S = 2^logS) of a transform, natural order in and out, or (DIT)
// with the MODE_BITREV_OUT / MODE_TWIST_OUT writes (natural n = r S + c to row rev_L(n); twisted into both halves).
template <bool DIT, int MODE>
__global__ __launch_bounds__(s9::NTH, 4) void k_ntt_s9(const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md,
                                                       int logS, const uint32_t *__restrict__ tw, Twist tws,
                                                       uint64_t dst_half) {
    using namespace s9;
    __shared__ uint32_t x[512 * 32];
    const uint32_t S = 1u << logS;
    const uint32_t groups = S >> 5;
    const uint32_t outer = blockIdx.x / groups;
    const uint32_t c0 = (blockIdx.x % groups) * 32;
    const uint32_t base = outer * 512u * S;
    const uint32_t t = threadIdx.x & 31, u = threadIdx.x >> 5;
    const uint32_t ct = c0 + t;
    const uint32_t *sp = src + ms.off(blockIdx.y) + base + ct;
    uint32_t *dp = dst + md.off(blockIdx.y);
    uint32_t v[16];
    if (DIT) {
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int k = 0; k < 8; k++) v[8 * n + k] = sp[(row0<LL>(u, n) + k) * S];
        nets<true, LL>(v, u, S, ct, tw);
        to_lds<LL>(x, v, u, t);
        __syncthreads();
        from_lds<LM>(x, v, u, t);
        nets<true, LM>(v, u, S, ct, tw);
        __syncthreads();
        to_lds<LM>(x, v, u, t);
        __syncthreads();
        from_lds<LH>(x, v, u, t);
        nets<true, LH>(v, u, S, ct, tw);
        if (MODE == MODE_PLAIN) {
#pragma unroll
            for (int n = 0; n < 2; n++)
#pragma unroll
                for (int k = 0; k < 8; k++) dp[base + (row0<LH>(u, n) + 64 * k) * S + ct] = v[8 * n + k];
        } else if (MODE == MODE_TWIST_OUT) {
#pragma unroll
            for (int n = 0; n < 2; n++)
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t i = base + (row0<LH>(u, n) + 64 * k) * S + ct;
                    dp[i] = mul(v[8 * n + k], tws.f(0, i));
                    dp[dst_half + i] = mul(v[8 * n + k], tws.f(1, i));
                }
        } else {  // BITREV_OUT: natural n = r S + c -> row rev_L(n) = rev_logS(c) * 512 + rev_9(r)
            __syncthreads();
            to_lds<LH>(x, v, u, t);
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t idx = (uint32_t)i * NTH + threadIdx.x;
                const uint32_t tc = idx >> 9, q = idx & 511;
                dp[(uint64_t)rev_bits(c0 + tc, logS) * 512 + q] = x[at(rev_bits(q, 9), tc)];
            }
        }
    } else {
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int k = 0; k < 8; k++) v[8 * n + k] = sp[(row0<LH>(u, n) + 64 * k) * S];
        nets<false, LH>(v, u, S, ct, tw);
        to_lds<LH>(x, v, u, t);
        __syncthreads();
        from_lds<LM>(x, v, u, t);
        nets<false, LM>(v, u, S, ct, tw);
        __syncthreads();
        to_lds<LM>(x, v, u, t);
        __syncthreads();
        from_lds<LL>(x, v, u, t);
        nets<false, LL>(v, u, S, ct, tw);
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int k = 0; k < 8; k++) dp[base + (row0<LL>(u, n) + k) * S + ct] = v[8 * n + k];
    }
}

// LOGR = 6..8 strided stages as register tiles of R = 2^LOGR rows x 32 columns, 2R threads x two 8-element
// networks: the k_ntt_s9 design for the passes of the 2^19 and 2^21 LDEs (13-stage tile + 6 / 8) and of the
// recursion shards' heights.  The LDS-staged strided kernel these replaced (deleted in round 6 with k_ntt_rg) ran at about half the bytes per second
// of the 9-stage kernels (2^21 x 67 LDE 2.55 -> 2.01 ms, profiles/r05_lde_s8_ab.txt).  Layouts (u = tid >> 5,
// network n in {0,1}, g = 2u + n < R/8, element k < 8), three stages per layout except where noted:
//   LOGR 8: LH row g + 32k (h_r 32..128) | LM row (g>>2)*32 + (g&3) + 4k (4..16) | LL row 8g + k (1, 2)
//   LOGR 7: LH row g + 16k (16..64)      | LM row (g>>1)*16 + (g&1) + 2k (2..8)  | LL row 8g + k (1)
//   LOGR 6: LH row g + 8k (8..32)        |                                        | LL row 8g + k (1..4)
//   LOGR 5: LH row g + 4k (4..16)        |                                        | LL row 8g + k (1, 2)
// (LOGR 5 is one wave per workgroup: the 2^18 LDE's pass and both of the 2^23 LDE's; 2^18 -9 %, profiles/r05_lde_s5_ab.txt)
namespace sr {
enum { LH = 0, LM = 1, LL = 2 };
template <int LOGR>
__device__ __forceinline__ uint32_t at(uint32_t r, uint32_t t) {
    // columns XOR-swizzled by row bits LOGR-5..LOGR-1: a half-wave's 32 lanes touch one row (any swizzle is
    // conflict-free), and the bit-reversed output walk's rows base + 2^(LOGR-5) m (m < 32) land on 32 banks
    return r * 32 + (t ^ ((r >> (LOGR - 5)) & 31));
}
template <int LOGR, int LAY> constexpr uint32_t RS = LAY == LH ? (1u << (LOGR - 3)) : LAY == LL ? 1u : (LOGR == 8 ? 4u : 2u);
template <int LOGR, int LAY>
constexpr int NST = LAY != LL ? 3 : LOGR == 8 ? 2 : LOGR == 7 ? 1 : LOGR == 5 ? 2 : 3;  // 8 = 3+3+2, 7 = 3+3+1, 6 = 3+3, 5 = 3+2
template <int LOGR, int LAY>
__device__ __forceinline__ uint32_t row0(uint32_t u, int n) {
    const uint32_t g = 2 * u + n;
    if constexpr (LAY == LH) return g;
    else if constexpr (LAY == LM) return LOGR == 8 ? (g >> 2) * 32 + (g & 3) : (g >> 1) * 16 + (g & 1);
    else return 8 * g;
}

// NST stages of one 8-element network (as s9::net8; fewer stages: independent groups of 2^NST elements)
template <int LOGR, bool DIT, int LAY>
__device__ __forceinline__ void net8(uint32_t *v, uint32_t off, uint32_t S, uint32_t ct,
                                     const uint32_t *__restrict__ tw) {
    constexpr uint32_t rs = RS<LOGR, LAY>;
    constexpr int ns = NST<LOGR, LAY>;
#pragma unroll
    for (int q = 0; q < ns; q++) {
        const int st = DIT ? q : ns - 1 - q;
        const int span = 1 << st;
        const uint32_t h = (rs << st) * S;
#pragma unroll
        for (int m = 0; m < span; m++) {
            const uint32_t w = tw[h + (off + rs * m) * S + ct];
#pragma unroll
            for (int k = m; k < 8; k += 2 * span) {
                const uint32_t a = v[k], b = v[k + span];
                if (DIT) {
                    const uint32_t tt = mul(b, w);
                    if (q < ns - 1 && ((k >> (st + 1)) & 1)) {  // next stage multiplies both: lazy [0, 2P)
                        v[k] = a + tt;
                        v[k + span] = a + (P - tt);
                    } else {
                        v[k] = add(a, tt);
                        v[k + span] = sub(a, tt);
                    }
                } else {
                    v[k] = add(a, b);
                    v[k + span] = mul(a + (P - b), w);
                }
            }
        }
    }
}
template <int LOGR, bool DIT, int LAY>
__device__ __forceinline__ void nets(uint32_t v[16], uint32_t u, uint32_t S, uint32_t ct,
                                     const uint32_t *__restrict__ tw) {
#pragma unroll
    for (int n = 0; n < 2; n++) net8<LOGR, DIT, LAY>(v + 8 * n, row0<LOGR, LAY>(u, n) % RS<LOGR, LAY>, S, ct, tw);
}
template <int LOGR, int LAY>
__device__ __forceinline__ void to_lds(uint32_t *x, const uint32_t v[16], uint32_t u, uint32_t t) {
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[at<LOGR>(row0<LOGR, LAY>(u, n) + RS<LOGR, LAY> * k, t)] = v[8 * n + k];
}
template <int LOGR, int LAY>
__device__ __forceinline__ void from_lds(const uint32_t *x, uint32_t v[16], uint32_t u, uint32_t t) {
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int k = 0; k < 8; k++) v[8 * n + k] = x[at<LOGR>(row0<LOGR, LAY>(u, n) + RS<LOGR, LAY> * k, t)];
}
}  // namespace sr

template <int LOGR, bool DIT, int MODE>
__global__ __launch_bounds__(2 << LOGR) void k_ntt_sr(const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md,
                                                       int logS, const uint32_t *__restrict__ tw, Twist tws,
                                                       uint64_t dst_half) {
    using namespace sr;
    constexpr uint32_t R = 1u << LOGR, NTH = 2 * R;
    constexpr bool MID = LOGR > 6;  // a middle layout (two LDS exchanges) or only LH and LL (one)
    __shared__ uint32_t x[R * 32];
    const uint32_t S = 1u << logS;
    const uint32_t groups = S >> 5;
    const uint32_t outer = blockIdx.x / groups;
    const uint32_t c0 = (blockIdx.x % groups) * 32;
    const uint32_t base = outer * R * S;
    const uint32_t t = threadIdx.x & 31, u = threadIdx.x >> 5;
    const uint32_t ct = c0 + t;
    const uint32_t *sp = src + ms.off(blockIdx.y) + base + ct;
    uint32_t *dp = dst + md.off(blockIdx.y);
    constexpr uint32_t HS = RS<LOGR, LH>;  // LH row stride
    uint32_t v[16];
    if (DIT) {
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int k = 0; k < 8; k++) v[8 * n + k] = sp[(row0<LOGR, LL>(u, n) + k) * S];
        nets<LOGR, true, LL>(v, u, S, ct, tw);
        to_lds<LOGR, LL>(x, v, u, t);
        __syncthreads();
        if constexpr (MID) {
            from_lds<LOGR, LM>(x, v, u, t);
            nets<LOGR, true, LM>(v, u, S, ct, tw);
            __syncthreads();
            to_lds<LOGR, LM>(x, v, u, t);
            __syncthreads();
        }
        from_lds<LOGR, LH>(x, v, u, t);
        nets<LOGR, true, LH>(v, u, S, ct, tw);
        if (MODE == MODE_PLAIN) {
#pragma unroll
            for (int n = 0; n < 2; n++)
#pragma unroll
                for (int k = 0; k < 8; k++) dp[base + (row0<LOGR, LH>(u, n) + HS * k) * S + ct] = v[8 * n + k];
        } else if (MODE == MODE_TWIST_OUT) {
#pragma unroll
            for (int n = 0; n < 2; n++)
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t i = base + (row0<LOGR, LH>(u, n) + HS * k) * S + ct;
                    dp[i] = mul(v[8 * n + k], tws.f(0, i));
                    dp[dst_half + i] = mul(v[8 * n + k], tws.f(1, i));
                }
        } else {  // BITREV_OUT: natural n = r S + c -> row rev_L(n) = rev_logS(c) * R + rev_LOGR(r)
            __syncthreads();
            to_lds<LOGR, LH>(x, v, u, t);
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t idx = (uint32_t)i * NTH + threadIdx.x;
                const uint32_t tc = idx >> LOGR, q = idx & (R - 1);
                __builtin_nontemporal_store(x[at<LOGR>(rev_bits(q, LOGR), tc)],
                                            &dp[(uint64_t)rev_bits(c0 + tc, logS) * R + q]);
            }
        }
    } else {
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int k = 0; k < 8; k++) v[8 * n + k] = sp[(row0<LOGR, LH>(u, n) + HS * k) * S];
        nets<LOGR, false, LH>(v, u, S, ct, tw);
        to_lds<LOGR, LH>(x, v, u, t);
        __syncthreads();
        if constexpr (MID) {
            from_lds<LOGR, LM>(x, v, u, t);
            nets<LOGR, false, LM>(v, u, S, ct, tw);
            __syncthreads();
            to_lds<LOGR, LM>(x, v, u, t);
            __syncthreads();
        }
        from_lds<LOGR, LL>(x, v, u, t);
        nets<LOGR, false, LL>(v, u, S, ct, tw);
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int k = 0; k < 8; k++) dp[base + (row0<LOGR, LL>(u, n) + k) * S + ct] = v[8 * n + k];
    }
}

// LOGR = 1..4 strided stages (the short passes of the recursion shards' LDEs: 2^14..2^17 = the 13-stage tile + 1..4)
// with one column per thread and all R = 2^LOGR rows in its registers: no LDS and no barrier; every load and store
// instruction of a wave moves 256 consecutive bytes of one row, and the stage twiddles w_{2h}^{m S + c} are as
// coalesced.  The bit-reversed-output pass writes each thread's R outputs as one contiguous run (16-byte stores).
template <int LOGR, bool DIT, int MODE>
__global__ __launch_bounds__(256) void k_ntt_rg(const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md, int logS,
                                                const uint32_t *__restrict__ tw, Twist tws, uint64_t dst_half) {
    constexpr uint32_t R = 1u << LOGR;
    const uint32_t S = 1u << logS;
    const uint32_t groups = S >> 8;  // 256-column groups per block of R S rows
    const uint32_t outer = blockIdx.x / groups;
    const uint32_t c = (blockIdx.x % groups) * 256 + threadIdx.x;
    const uint32_t base = outer * R * S;
    const uint32_t *sp = src + ms.off(blockIdx.y) + base + c;
    uint32_t *dp = dst + md.off(blockIdx.y);
    uint32_t v[R];
#pragma unroll
    for (uint32_t r = 0; r < R; r++) v[r] = sp[r * S];
#pragma unroll
    for (int q = 0; q < LOGR; q++) {
        const int st = DIT ? q : LOGR - 1 - q;  // DIT: h = S, 2S, ...; DIF: reverse
        const uint32_t span = 1u << st;
#pragma unroll
        for (uint32_t m = 0; m < span; m++) {
            const uint32_t w = tw[(span + m) * S + c];  // w_{2h}^{m S + c}, h = span S
#pragma unroll
            for (uint32_t k = m; k < R; k += 2 * span) {
                const uint32_t a = v[k], b = v[k + span];
                if (DIT) {
                    const uint32_t tt = mul(b, w);
                    v[k] = add(a, tt);
                    v[k + span] = sub(a, tt);
                } else {
                    v[k] = add(a, b);
                    v[k + span] = mul(a + (P - b), w);  // (0, 2P) operand: no reduction before the product
                }
            }
        }
    }
    if (MODE == MODE_BITREV_OUT) {  // R S == N: natural n = r S + c -> row rev_logS(c) R + rev_LOGR(r), R words per thread
        uint32_t *o = dp + (uint64_t)rev_bits(c, logS) * R;
        if constexpr (R >= 4) {
#pragma unroll
            for (uint32_t j = 0; j < R; j += 4)
                reinterpret_cast<uint4 *>(o)[j / 4] = make_uint4(v[rev_bits(j, LOGR)], v[rev_bits(j + 1, LOGR)],
                                                                 v[rev_bits(j + 2, LOGR)], v[rev_bits(j + 3, LOGR)]);
        } else {
#pragma unroll
            for (uint32_t j = 0; j < R; j++) o[j] = v[rev_bits(j, LOGR)];
        }
        return;
    }
#pragma unroll
    for (uint32_t r = 0; r < R; r++) {
        const uint32_t i = base + r * S + c;
        if (MODE == MODE_TWIST_OUT) {
            dp[i] = mul(v[r], tws.f(0, i));
            dp[dst_half + i] = mul(v[r], tws.f(1, i));
        } else {
            dp[i] = v[r];
        }
    }
}

// Same tiles and networks as k_ntt_s9, addressed through buffer descriptors: every global access
// (data, twiddles, stores) is one per-thread 32-bit voffset fixed for the kernel plus a
// wave-uniform soffset (k S words, twiddle stage bases) computed on the scalar unit, so the
// address arithmetic leaves the VALU (k_ntt_s9 spent ~40 % of its VALU issue on 64-bit address
// math).  LDS tiles are XOR-swizzled only where the bit-reversed output walk needs it, so the
// other layouts' LDS addresses are a base plus immediate offsets.
namespace s9 {
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mkrs(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint32_t bld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}
// cache-policy bits of the strided passes' final stores: non-temporal (nt).  Their output is the LDE, read much
// later by the leaf hashing: LDE 2^22 x 64 3.66-3.67 vs 3.71-3.72 ms with the default policy when every pass stored
// nt (profiles/r05_ntt_nt_store_ab.txt); -DZKM_NTT_STORE_AUX=0 restores it.  Intermediate stores: bst_mid.
#ifndef ZKM_NTT_STORE_AUX
#define ZKM_NTT_STORE_AUX 2
#endif
__device__ __forceinline__ void bst(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, soff, ZKM_NTT_STORE_AUX);
}
__device__ __forceinline__ void bst_mid(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, soff, ZKM_LDE_MID_AUX);
}
template <bool SWZ>
__device__ __forceinline__ uint32_t atb(uint32_t r, uint32_t t) {
    if constexpr (SWZ) return r * 32 + (t ^ ((r >> 4) & 31));
    else return r * 32 + t;
}

// The same network with its twiddles generated in registers from ONE loaded value.  Stage st of the network
// (half-size h = rs 2^st S rows) uses w_{st,m} = w_{2h}^{(off + rs m) S + ct} = w_{st,0} * w_{2^(st+1)}^m, and
// w_{st,0} = w_{st+1,0}^2 (the same exponent, a root of half the order); so only w_{2,0} is read and the other
// six twiddles cost two squarings and four products by the constants w_4^1, w_8^1..3 of the table's direction
// (the strided passes spent 35 of 51 vector-memory instructions per wave on twiddle loads with the VALU ~9 %
// busy, profiles/r04_lde_pmc.txt).
struct TwC {
    uint32_t w4, w8[3];  // w_4^1 = tw[3], w_8^m = tw[4 + m]
};
__device__ __forceinline__ TwC twc(const uint32_t *__restrict__ tw) {
    return TwC{tw[3], {tw[5], tw[6], tw[7]}};
}
struct Tw8 {
    uint32_t w[3][4];  // w[st][m], m < 2^st
};
__device__ __forceinline__ Tw8 tw8(uint32_t wtop, const TwC &c) {
    Tw8 r;
    r.w[2][0] = wtop;
    r.w[1][0] = mul(wtop, wtop);
    r.w[0][0] = mul(r.w[1][0], r.w[1][0]);
    r.w[1][1] = mul(r.w[1][0], c.w4);
#pragma unroll
    for (int m = 1; m < 4; m++) r.w[2][m] = mul(wtop, c.w8[m - 1]);
    return r;
}
template <bool DIT>
__device__ __forceinline__ void net8r(uint32_t *v, const Tw8 &W) {
#pragma unroll
    for (int q = 0; q < 3; q++) {
        const int st = DIT ? q : 2 - q;
        const int span = 1 << st;
#pragma unroll
        for (int m = 0; m < span; m++) {
            const uint32_t w = W.w[st][m];
#pragma unroll
            for (int k = m; k < 8; k += 2 * span) {
                const uint32_t a = v[k], b = v[k + span];
                if (DIT) {
                    const uint32_t tt = mul(b, w);
                    if (q < 2 && ((k >> (st + 1)) & 1)) {
                        v[k] = a + tt;
                        v[k + span] = a + (P - tt);
                    } else {
                        v[k] = add(a, tt);
                        v[k + span] = sub(a, tt);
                    }
                } else {
                    v[k] = add(a, b);
                    v[k + span] = mul(a + (P - b), w);
                }
            }
        }
    }
}
// one network's stages, twiddles generated from w_{2,0}, which sits at voff + soff0 + 4 rs S words (the form that
// loaded all seven per network lost its A/B: 3.94 vs 3.93 ms for the 2^22 x 67 LDE, round 5)
template <bool DIT, int LAY>
__device__ __forceinline__ void net8x(uint32_t *v, __amdgpu_buffer_rsrc_t rtw, uint32_t voff, uint32_t soff0,
                                      uint32_t S4, const TwC &c) {
    net8r<DIT>(v, tw8(bld(rtw, voff, soff0 + 4 * RS<LAY> * S4), c));
}

template <int LAY, bool SWZ>
__device__ __forceinline__ void to_ldsb(uint32_t *x, const uint32_t v[16], uint32_t u, uint32_t t) {
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[atb<SWZ>(row0<LAY>(u, n) + RS<LAY> * k, t)] = v[8 * n + k];
}
template <int LAY, bool SWZ>
__device__ __forceinline__ void from_ldsb(const uint32_t *x, uint32_t v[16], uint32_t u, uint32_t t) {
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int k = 0; k < 8; k++) v[8 * n + k] = x[atb<SWZ>(row0<LAY>(u, n) + RS<LAY> * k, t)];
}
}  // namespace s9

// TILE (bit 0: source, bit 1: destination; only for the one-pass case 512 x S = the column): that side is
// tile-major -- the tile's 512 rows x 32 columns contiguous (64 KB, row pitch 32 words) at tile index
// c0 / 32 -- instead of row-major with pitch S (the LDE's intermediates at 2^22, lde_natural).
template <bool DIT, int MODE, int TILE = 0>
__global__ __launch_bounds__(s9::NTH, 4) void k_ntt_s9b(const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md,
                                                        int logS, const uint32_t *__restrict__ tw,
                                                        uint32_t tw_words, uint32_t nv, int remap) {
    using namespace s9;
    constexpr bool SWZ = DIT && MODE == MODE_BITREV_OUT;
    constexpr bool TS = TILE & 1, TD = (TILE & 2) != 0;
    __shared__ uint32_t x[512 * 32];
    const uint32_t S = 1u << logS, S4 = S * 4;
    // XCD-aware order: workgroup i runs on XCD i mod 8, so XCD x takes the contiguous range
    // [x total/8, (x+1) total/8) of (tile, column) pairs, columns fastest: the columns of one tile
    // run back to back on one XCD and read the tile's twiddles from its L2 instead of HBM
    const uint32_t total = gridDim.x, lin = blockIdx.x;
    const uint32_t vid = (total & 7) ? lin : (lin & 7) * (total >> 3) + (lin >> 3);
    const uint32_t ntile = total / nv;
    const uint32_t col = remap ? vid % nv : lin / ntile, tile = remap ? vid / nv : lin % ntile;
    const uint32_t outer = tile >> (logS - 5);
    const uint32_t c0 = (tile & ((S >> 5) - 1)) * 32;
    const uint32_t base = outer * 512u * S;
    const uint32_t t = threadIdx.x & 31, u = threadIdx.x >> 5;
    const uint32_t ct = c0 + t;
    const uint64_t tbase = (uint64_t)(c0 >> 5) * (512u * 32u);  // tile-major: the tile's 64 KB
    const auto rsrc = TS ? mkrs(src + ms.off(col) + tbase, 512u * 128u) : mkrs(src + ms.off(col) + base, 512u * S4);
    const auto rtw = mkrs(tw, tw_words * 4);
    const TwC twk = twc(tw);
    const uint32_t vLL = ct * 4;                    // twiddle offsets per layout / network
    const uint32_t vLM0 = (((2 * u) & 7) * S + ct) * 4, vLM1 = (((2 * u + 1) & 7) * S + ct) * 4;
    const uint32_t vLH = (u * S + ct) * 4;          // also rows u + 32 n + 64 k of the tile
    const uint32_t vL16 = (16 * u * S + ct) * 4;    // rows 16 u + 8 n + k of the tile
    // data offsets of the source / destination side (row pitch S words, or 32 when tile-major)
    const uint32_t sP4 = TS ? 128u : S4, dP4 = TD ? 128u : S4;
    const uint32_t sLH = TS ? (u * 32 + t) * 4 : vLH, sL16 = TS ? (16 * u * 32 + t) * 4 : vL16;
    const uint32_t dLH = TD ? (u * 32 + t) * 4 : vLH, dL16 = TD ? (16 * u * 32 + t) * 4 : vL16;
    uint32_t v[16];
    if (DIT) {
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int k = 0; k < 8; k++) v[8 * n + k] = bld(rsrc, sL16, (uint32_t)(8 * n + k) * sP4);
        {  // both networks of LL share their twiddles (off = 0)
            const Tw8 W = tw8(bld(rtw, vLL, 4 * S4), twk);
            net8r<true>(v, W);
            net8r<true>(v + 8, W);
        }
        to_ldsb<LL, false>(x, v, u, t);
        __syncthreads();
        from_ldsb<LM, false>(x, v, u, t);
        net8x<true, LM>(v, rtw, vLM0, 0, S4, twk);
        net8x<true, LM>(v + 8, rtw, vLM1, 0, S4, twk);
        __syncthreads();
        to_ldsb<LM, false>(x, v, u, t);
        __syncthreads();
        from_ldsb<LH, false>(x, v, u, t);
        net8x<true, LH>(v, rtw, vLH, 0, S4, twk);
        net8x<true, LH>(v + 8, rtw, vLH, 32 * S4, S4, twk);
        if (MODE == MODE_PLAIN) {
            const auto rdst = TD ? mkrs(dst + md.off(col) + tbase, 512u * 128u) : mkrs(dst + md.off(col) + base, 512u * S4);
#pragma unroll
            for (int n = 0; n < 2; n++)
#pragma unroll
                for (int k = 0; k < 8; k++) bst_mid(v[8 * n + k], rdst, dLH, (uint32_t)(32 * n + 64 * k) * dP4);
        } else {  // BITREV_OUT: natural n = r S + c -> row rev_L(n) = rev_logS(c) * 512 + rev_9(r)
            __syncthreads();
            to_ldsb<LH, SWZ>(x, v, u, t);
            __syncthreads();
            const auto rdst = mkrs(dst + md.off(col), 512u * S4);
            const uint32_t q = threadIdx.x & 511, hb = threadIdx.x >> 9, rq = rev_bits(q, 9);
            const uint32_t vo = (((rev_bits(c0, logS) + (hb << (logS - 1))) << 9) + q) * 4;
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t tc = 2 * i + hb;
                const uint32_t so = (rev_bits((uint32_t)(2 * i), 5) << (logS - 5)) << 11;  // rows x 512 words x 4 B
                bst(x[atb<SWZ>(rq, tc)], rdst, vo, so);
            }
        }
    } else {
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int k = 0; k < 8; k++) v[8 * n + k] = bld(rsrc, sLH, (uint32_t)(32 * n + 64 * k) * sP4);
        net8x<false, LH>(v, rtw, vLH, 0, S4, twk);
        net8x<false, LH>(v + 8, rtw, vLH, 32 * S4, S4, twk);
        to_ldsb<LH, false>(x, v, u, t);
        __syncthreads();
        from_ldsb<LM, false>(x, v, u, t);
        net8x<false, LM>(v, rtw, vLM0, 0, S4, twk);
        net8x<false, LM>(v + 8, rtw, vLM1, 0, S4, twk);
        __syncthreads();
        to_ldsb<LM, false>(x, v, u, t);
        __syncthreads();
        from_ldsb<LL, false>(x, v, u, t);
        {  // both networks of LL share their twiddles (off = 0)
            const Tw8 W = tw8(bld(rtw, vLL, 4 * S4), twk);
            net8r<false>(v, W);
            net8r<false>(v + 8, W);
        }
        const auto rdst = TD ? mkrs(dst + md.off(col) + tbase, 512u * 128u) : mkrs(dst + md.off(col) + base, 512u * S4);
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int k = 0; k < 8; k++) bst_mid(v[8 * n + k], rdst, dL16, (uint32_t)(8 * n + k) * dP4);
    }
}

// 10 strided stages (the 2^23 LDE = 2^13 tile x 2^10 strided: three HBM passes instead of five with two 5-stage
// passes each way).  One workgroup of 1024 threads: 1024 rows (stride S) x 16 consecutive columns, 16 elements
// per thread, 64 KB of LDS (two workgroups per CU, as k_ntt_s9b).  Lane -> column (t = tid & 15: 64-B row
// segments), u = tid >> 4 < 64.  Layouts (network n in {0,1}, g = 2u + n < 128):
//   LH: one 16-point network, rows u + 64k (k < 16)           stages h_r = 64, 128, 256, 512 rows
//   LM: two 8-point networks, rows (g >> 3) 64 + (g & 7) + 8k  h_r = 8, 16, 32
//   LL: two 8-point networks, rows 8g + k                      h_r = 1, 2, 4
// Twiddles as k_ntt_s9b: one load per network (its top twiddle), the rest generated (squarings and products by
// w_4, w_8^m, w_16^m).  LDS: row r at physical row r ^ (r1 ^ r4 ^ r9) (bit i of r: ri), so the two rows a
// 32-lane half touches (in LH rows differing in bit 0, LM in bit 1, LL in bit 4, the bit-reversed output walk in
// bit 9) sit in opposite 16-bank halves; the output walk also XORs the column with row bits 5..8.
namespace s10 {
constexpr int NTH = 1024;
template <bool SWZ>
__device__ __forceinline__ uint32_t at(uint32_t r, uint32_t t) {
    const uint32_t p = r ^ (((r >> 1) ^ (r >> 4) ^ (r >> 9)) & 1u);
    if constexpr (SWZ) return p * 16 + (t ^ ((r >> 5) & 15));
    else return p * 16 + t;
}
struct Tw16 {
    uint32_t w[4][8];  // w[st][m], m < 2^st
};
struct TwC16 {
    uint32_t w4, w8[3], w16[7];
};
__device__ __forceinline__ TwC16 twc16(const uint32_t *__restrict__ tw) {
    TwC16 c;
    c.w4 = tw[3];
#pragma unroll
    for (int m = 1; m < 4; m++) c.w8[m - 1] = tw[4 + m];
#pragma unroll
    for (int m = 1; m < 8; m++) c.w16[m - 1] = tw[8 + m];
    return c;
}
// w_{st,0} = w_{st+1,0}^2 and w_{st,m} = w_{st,0} w_{2^(st+1)}^m (the top twiddle w_{3,0} loaded)
__device__ __forceinline__ Tw16 tw16(uint32_t wtop, const TwC16 &c) {
    Tw16 r;
    r.w[3][0] = wtop;
    r.w[2][0] = mul(wtop, wtop);
    r.w[1][0] = mul(r.w[2][0], r.w[2][0]);
    r.w[0][0] = mul(r.w[1][0], r.w[1][0]);
    r.w[1][1] = mul(r.w[1][0], c.w4);
#pragma unroll
    for (int m = 1; m < 4; m++) r.w[2][m] = mul(r.w[2][0], c.w8[m - 1]);
#pragma unroll
    for (int m = 1; m < 8; m++) r.w[3][m] = mul(wtop, c.w16[m - 1]);
    return r;
}
template <bool DIT>
__device__ __forceinline__ void net16r(uint32_t *v, const Tw16 &W) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int st = DIT ? q : 3 - q;
        const int span = 1 << st;
#pragma unroll
        for (int m = 0; m < span; m++) {
            const uint32_t w = W.w[st][m];
#pragma unroll
            for (int k = m; k < 16; k += 2 * span) {
                const uint32_t a = v[k], b = v[k + span];
                if (DIT) {
                    const uint32_t tt = mul(b, w);
                    if (q < 3 && ((k >> (st + 1)) & 1)) {  // next stage multiplies both: lazy [0, 2P)
                        v[k] = a + tt;
                        v[k + span] = a + (P - tt);
                    } else {
                        v[k] = add(a, tt);
                        v[k + span] = sub(a, tt);
                    }
                } else {
                    v[k] = add(a, b);
                    v[k + span] = mul(a + (P - b), w);
                }
            }
        }
    }
}
// element k of network n of a layout: its tile row
enum { LH = 0, LM = 1, LL = 2 };
template <int LAY>
__device__ __forceinline__ uint32_t row(uint32_t u, int n, int k) {
    const uint32_t g = 2 * u + n;
    if constexpr (LAY == LH) return u + 64 * (8 * n + k);  // (n, k) = element 8n + k of the 16-point network
    else if constexpr (LAY == LM) return (g >> 3) * 64 + (g & 7) + 8 * k;
    else return 8 * g + k;
}
template <int LAY, bool SWZ>
__device__ __forceinline__ void to_lds(uint32_t *x, const uint32_t v[16], uint32_t u, uint32_t t) {
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[at<SWZ>(row<LAY>(u, n, k), t)] = v[8 * n + k];
}
template <int LAY>
__device__ __forceinline__ void from_lds(const uint32_t *x, uint32_t v[16], uint32_t u, uint32_t t) {
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int k = 0; k < 8; k++) v[8 * n + k] = x[at<false>(row<LAY>(u, n, k), t)];
}
}  // namespace s10

template <bool DIT, int MODE>
__global__ __launch_bounds__(s10::NTH, 4) void k_ntt_s10(const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md,
                                                         int logS, const uint32_t *__restrict__ tw, uint32_t tw_words,
                                                         uint32_t nv, Twist tws, uint64_t dst_half) {
    using namespace s10;
    using s9::bld;
    using s9::mkrs;
    using s9::TwC;
    using s9::Tw8;
    __shared__ uint32_t x[1024 * 16];
    const uint32_t S = 1u << logS, S4 = S * 4;
    // XCD-aware order (k_ntt_s9b): the columns of one tile back to back on one XCD
    const uint32_t total = gridDim.x, lin = blockIdx.x;
    const uint32_t vid = (total & 7) ? lin : (lin & 7) * (total >> 3) + (lin >> 3);
    const uint32_t col = vid % nv, tile = vid / nv;
    const uint32_t outer = tile >> (logS - 4);
    const uint32_t c0 = (tile & ((S >> 4) - 1)) * 16;
    const uint32_t base = outer * 1024u * S;
    const uint32_t t = threadIdx.x & 15, u = threadIdx.x >> 4;
    const uint32_t ct = c0 + t;
    const auto rsrc = mkrs(src + ms.off(col) + base, 1024u * S4);
    const auto rtw = mkrs(tw, tw_words * 4);
    const TwC twk = s9::twc(tw);
    const TwC16 tw16c = twc16(tw);
    // top-twiddle offsets: LH w_{1024 S}^{u S + ct} (index 512 S + u S + ct), LM w_{64 S}^{(g & 7) S + ct}, LL
    // w_{8 S}^{ct}; data: LH rows u + 64 k, LL rows 16 u + 8 n + k
    const uint32_t vLH = (u * S + ct) * 4, vL16 = (16 * u * S + ct) * 4, vLL = ct * 4;
    const uint32_t vLM0 = (((2 * u) & 7) * S + ct) * 4, vLM1 = (((2 * u + 1) & 7) * S + ct) * 4;
    uint32_t v[16];
    if (DIT) {
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int k = 0; k < 8; k++) v[8 * n + k] = bld(rsrc, vL16, (uint32_t)(8 * n + k) * S4);
        {  // both networks of LL share their twiddles (off = 0)
            const Tw8 W = s9::tw8(bld(rtw, vLL, 4 * S4), twk);
            s9::net8r<true>(v, W);
            s9::net8r<true>(v + 8, W);
        }
        to_lds<LL, false>(x, v, u, t);
        __syncthreads();
        from_lds<LM>(x, v, u, t);
        s9::net8r<true>(v, s9::tw8(bld(rtw, vLM0, 32 * S4), twk));
        s9::net8r<true>(v + 8, s9::tw8(bld(rtw, vLM1, 32 * S4), twk));
        __syncthreads();
        to_lds<LM, false>(x, v, u, t);
        __syncthreads();
        from_lds<LH>(x, v, u, t);
        net16r<true>(v, tw16(bld(rtw, vLH, 512 * S4), tw16c));
        if (MODE == MODE_PLAIN) {
            const auto rdst = mkrs(dst + md.off(col) + base, 1024u * S4);
#pragma unroll
            for (int k = 0; k < 16; k++) s9::bst_mid(v[k], rdst, vLH, (uint32_t)(64 * k) * S4);
        } else if (MODE == MODE_TWIST_OUT) {  // the inverse's last pass: coefficient n to both LDE halves, twisted
            uint32_t *dp = dst + md.off(col);
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const uint32_t i = base + (u + 64 * (uint32_t)k) * S + ct;
                dp[i] = mul(v[k], tws.f(0, i));
                dp[dst_half + i] = mul(v[k], tws.f(1, i));
            }
        } else {  // BITREV_OUT: natural n = r S + c -> row rev_L(n) = rev_logS(c) * 1024 + rev_10(r)
            __syncthreads();
            to_lds<LH, true>(x, v, u, t);
            __syncthreads();
            const auto rdst = mkrs(dst + md.off(col), 1024u * S4);
            const uint32_t q = threadIdx.x, rq = rev_bits(q, 10);
            const uint32_t vo = ((rev_bits(c0, logS) << 10) + q) * 4;
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const uint32_t so = (rev_bits((uint32_t)i, 4) << (logS - 4)) << 12;  // rows x 1024 words x 4 B
                s9::bst(x[at<true>(rq, (uint32_t)i)], rdst, vo, so);
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = bld(rsrc, vLH, (uint32_t)(64 * k) * S4);
        net16r<false>(v, tw16(bld(rtw, vLH, 512 * S4), tw16c));
        to_lds<LH, false>(x, v, u, t);
        __syncthreads();
        from_lds<LM>(x, v, u, t);
        s9::net8r<false>(v, s9::tw8(bld(rtw, vLM0, 32 * S4), twk));
        s9::net8r<false>(v + 8, s9::tw8(bld(rtw, vLM1, 32 * S4), twk));
        __syncthreads();
        to_lds<LM, false>(x, v, u, t);
        __syncthreads();
        from_lds<LL>(x, v, u, t);
        {
            const Tw8 W = s9::tw8(bld(rtw, vLL, 4 * S4), twk);
            s9::net8r<false>(v, W);
            s9::net8r<false>(v + 8, W);
        }
        const auto rdst = mkrs(dst + md.off(col) + base, 1024u * S4);
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int k = 0; k < 8; k++) s9::bst_mid(v[8 * n + k], rdst, vL16, (uint32_t)(8 * n + k) * S4);
    }
}

template <bool TILED>
__global__ __launch_bounds__(t13::NTH, 6) void k_lde_fused13s(const uint32_t *src, uint32_t *dst, ColMap ms,
                                                             ColMap md, int L, const uint32_t *__restrict__ tt_inv,
                                                             const uint32_t *__restrict__ tt_fwd, Twist tws,
                                                             uint64_t dst_half) {
    using namespace t13;
    __shared__ uint32_t x[LDS13];
    const uint32_t t = threadIdx.x;
    const uint32_t N = 1u << L;
    // element j of thread t: word voff / 4 + j * SJ of the column (TILED: tiled13; else lay_idx<512> + base)
    const uint32_t voff = TILED ? (((t >> 5) * 16384u) + blockIdx.x * 32u + (t & 31)) * 4u : (blockIdx.x * 8192u + t) * 4u;
    constexpr uint32_t SJ4 = TILED ? 16u * 16384u * 4u : 512u * 4u;
    const auto rs = s9::mkrs(src + ms.off(blockIdx.y), N * 4u);
    uint32_t c[16];
#pragma unroll
    for (int j = 0; j < 16; j++) c[j] = s9::bld(rs, voff, (uint32_t)j * SJ4);
    dif13<true>(c, x, t, tt_inv);
    const auto rd = s9::mkrs(dst + md.off(blockIdx.y), (uint32_t)((dst_half + N) * 4u));
#pragma unroll 1
    for (int e = 0; e < 2; e++) {
        uint32_t v[16];
        {
            const uint32_t g = e ? tws.g1[blockIdx.x] : tws.g0[blockIdx.x];
            const uint4 *u = (const uint4 *)((e ? tws.u1 : tws.u0) + t * 16);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint4 a = u[q];
                const uint32_t au[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
                for (int r = 0; r < 4; r++) v[4 * q + r] = mul(mul_lazy(c[4 * q + r], g), au[r]);
            }
        }
        if (e) __syncthreads();  // the first coset's cross-wave L512 reads are done before this one's LDS writes
        dit13<true>(v, x, t, tt_fwd);
        const uint32_t so = e ? (uint32_t)(dst_half * 4u) : 0u;
#pragma unroll
        for (int j = 0; j < 16; j++) s9::bst_mid(v[j], rd, voff, so + (uint32_t)j * SJ4);
    }
}

// ------------------------------------------------------------------ dispatch
static constexpr int LOGC = 13;  // contiguous tile: 8192 elements
static constexpr int LOGS = 9;   // strided radix per pass (512 rows x 32 columns)

// columns per tile: k_ntt_s10 16, k_ntt_s9* / k_ntt_sr 32 (their swizzle spans 32 columns), k_ntt_rg 256 (a column per thread)
static int strided_T(int logR) { return logR == 10 ? 16 : logR >= 5 ? 32 : 256; }

template <bool DIT>
static void run_strided(int logR, const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md, uint32_t nv, int L,
                        int logS, const uint32_t *tw, int mode, hipStream_t s, Twist tws = Twist{},
                        uint64_t dst_half = 0, uint32_t tw_words = 0, int tile = 0) {
    const int T = strided_T(logR);
    ARG_CHECK((1 << logS) >= T, "strided pass narrower than its tile");
    ARG_CHECK(!tile || (logR == 9 && logS + 9 == L && tw_words && mode != MODE_TWIST_OUT),
              "tile-major sides need the one-pass 512-row strided kernel");
    dim3 g((unsigned)(((1ull << L) >> logR) / T), nv);
    if (logR == 10) {  // 1024-row x 16-column register tiles (k_ntt_s10): the LDEs of 2^23
        ARG_CHECK(tw_words && !tile, "the 10-stage pass: row-major sides");
        const dim3 g1(g.x * nv);
        if (!DIT)
            hipLaunchKernelGGL((k_ntt_s10<false, MODE_PLAIN>), g1, dim3(s10::NTH), 0, s, src, dst, ms, md, logS, tw,
                               tw_words, nv, tws, dst_half);
        else if (mode == MODE_PLAIN)
            hipLaunchKernelGGL((k_ntt_s10<true, MODE_PLAIN>), g1, dim3(s10::NTH), 0, s, src, dst, ms, md, logS, tw,
                               tw_words, nv, tws, dst_half);
        else if (mode == MODE_TWIST_OUT)
            hipLaunchKernelGGL((k_ntt_s10<true, MODE_TWIST_OUT>), g1, dim3(s10::NTH), 0, s, src, dst, ms, md, logS, tw,
                               tw_words, nv, tws, dst_half);
        else
            hipLaunchKernelGGL((k_ntt_s10<true, MODE_BITREV_OUT>), g1, dim3(s10::NTH), 0, s, src, dst, ms, md, logS,
                               tw, tw_words, nv, tws, dst_half);
        HIP_CHECK(hipGetLastError());
        return;
    }
    if (logR == 9 && tw_words && mode != MODE_TWIST_OUT) {
        // buffer-addressed register tiles (k_ntt_s9b), one grid dimension: (tile, column) remapped in the
        // kernel; tile-major source (bit 0) and / or destination (bit 1)
        const dim3 g1(g.x * nv);
#define S9B(TL)                                                                                                   \
    if (!DIT)                                                                                                     \
        hipLaunchKernelGGL((k_ntt_s9b<false, MODE_PLAIN, TL>), g1, dim3(s9::NTH), 0, s, src, dst, ms, md, logS, tw, \
                           tw_words, nv, 1);                                                                      \
    else if (mode == MODE_PLAIN)                                                                                  \
        hipLaunchKernelGGL((k_ntt_s9b<true, MODE_PLAIN, TL>), g1, dim3(s9::NTH), 0, s, src, dst, ms, md, logS, tw,  \
                           tw_words, nv, 1);                                                                      \
    else                                                                                                          \
        hipLaunchKernelGGL((k_ntt_s9b<true, MODE_BITREV_OUT, TL>), g1, dim3(s9::NTH), 0, s, src, dst, ms, md, logS, \
                           tw, tw_words, nv, 1);
        if (tile == 1) { S9B(1) } else if (tile == 2) { S9B(2) } else if (tile == 3) { S9B(3) } else { S9B(0) }
#undef S9B
        HIP_CHECK(hipGetLastError());
        return;
    }
    if (logR == 9) {  // register-tile kernel (T = 32), flat addressing: the twisted-output pass
        if (!DIT)
            hipLaunchKernelGGL((k_ntt_s9<false, MODE_PLAIN>), g, dim3(s9::NTH), 0, s, src, dst, ms, md, logS, tw, tws,
                               dst_half);
        else if (mode == MODE_PLAIN)
            hipLaunchKernelGGL((k_ntt_s9<true, MODE_PLAIN>), g, dim3(s9::NTH), 0, s, src, dst, ms, md, logS, tw, tws,
                               dst_half);
        else if (mode == MODE_TWIST_OUT)
            hipLaunchKernelGGL((k_ntt_s9<true, MODE_TWIST_OUT>), g, dim3(s9::NTH), 0, s, src, dst, ms, md, logS, tw,
                               tws, dst_half);
        else
            hipLaunchKernelGGL((k_ntt_s9<true, MODE_BITREV_OUT>), g, dim3(s9::NTH), 0, s, src, dst, ms, md, logS, tw,
                               tws, dst_half);
        HIP_CHECK(hipGetLastError());
        return;
    }
    if (logR >= 5 && logR <= 8) {  // register tiles of 2^logR rows x 32 columns (k_ntt_sr)
#define SRL(LR)                                                                                                   \
    if (!DIT)                                                                                                     \
        hipLaunchKernelGGL((k_ntt_sr<LR, false, MODE_PLAIN>), g, dim3(2 << LR), 0, s, src, dst, ms, md, logS, tw, tws, \
                           dst_half);                                                                             \
    else if (mode == MODE_PLAIN)                                                                                  \
        hipLaunchKernelGGL((k_ntt_sr<LR, true, MODE_PLAIN>), g, dim3(2 << LR), 0, s, src, dst, ms, md, logS, tw, tws,  \
                           dst_half);                                                                             \
    else if (mode == MODE_TWIST_OUT)                                                                              \
        hipLaunchKernelGGL((k_ntt_sr<LR, true, MODE_TWIST_OUT>), g, dim3(2 << LR), 0, s, src, dst, ms, md, logS, tw,   \
                           tws, dst_half);                                                                        \
    else                                                                                                          \
        hipLaunchKernelGGL((k_ntt_sr<LR, true, MODE_BITREV_OUT>), g, dim3(2 << LR), 0, s, src, dst, ms, md, logS, tw,  \
                           tws, dst_half);
        if (logR == 8) { SRL(8) } else if (logR == 7) { SRL(7) } else if (logR == 6) { SRL(6) } else { SRL(5) }
#undef SRL
        HIP_CHECK(hipGetLastError());
        return;
    }
    if (logR >= 1 && logR <= 4) {  // one column per thread (k_ntt_rg)
        const dim3 gr((unsigned)(((1ull << L) >> logR) >> 8), nv);
#define RGL(LR)                                                                                                   \
    if (!DIT)                                                                                                     \
        hipLaunchKernelGGL((k_ntt_rg<LR, false, MODE_PLAIN>), gr, dim3(256), 0, s, src, dst, ms, md, logS, tw, tws, \
                           dst_half);                                                                             \
    else if (mode == MODE_PLAIN)                                                                                  \
        hipLaunchKernelGGL((k_ntt_rg<LR, true, MODE_PLAIN>), gr, dim3(256), 0, s, src, dst, ms, md, logS, tw, tws,  \
                           dst_half);                                                                             \
    else if (mode == MODE_TWIST_OUT)                                                                              \
        hipLaunchKernelGGL((k_ntt_rg<LR, true, MODE_TWIST_OUT>), gr, dim3(256), 0, s, src, dst, ms, md, logS, tw,   \
                           tws, dst_half);                                                                        \
    else                                                                                                          \
        hipLaunchKernelGGL((k_ntt_rg<LR, true, MODE_BITREV_OUT>), gr, dim3(256), 0, s, src, dst, ms, md, logS, tw,  \
                           tws, dst_half);
        if (logR == 4) { RGL(4) } else if (logR == 3) { RGL(3) } else if (logR == 2) { RGL(2) } else { RGL(1) }
#undef RGL
        HIP_CHECK(hipGetLastError());
        return;
    }
throw ArgError("bad strided radix");
}

template <bool DIT>
static void run_contig(int logR, const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md, uint32_t nv, int L,
                       const uint32_t *tw, int mode, Twist tws, uint64_t dst_half, hipStream_t s) {
    dim3 g((unsigned)((1ull << L) >> logR), nv);
#define CCASE(k)                                                                                                 \
    case k:                                                                                                      \
        hipLaunchKernelGGL((k_ntt_contig<k, DIT, NT>), g, dim3(NT), 0, s, src, dst, ms, md, tw, mode, tws, dst_half); \
        break;
    switch (logR) {
        CCASE(1) CCASE(2) CCASE(3) CCASE(4) CCASE(5) CCASE(6) CCASE(7) CCASE(8) CCASE(9) CCASE(10) CCASE(11) CCASE(12)
        CCASE(13)
        default: throw ArgError("bad contiguous radix");
    }
#undef CCASE
    HIP_CHECK(hipGetLastError());
}

static void run_fused(int logR, const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md, uint32_t nv, int L,
                      const uint32_t *tw_inv, const uint32_t *tw_fwd, Twist tws, uint64_t dst_half, int bitrev_out,
                      hipStream_t s) {
    dim3 g((unsigned)((1ull << L) >> logR), nv);
#define FCASE(k)                                                                                                    \
    case k:                                                                                                         \
        hipLaunchKernelGGL((k_lde_fused<k, NT>), g, dim3(NT), 0, s, src, dst, ms, md, L, tw_inv, tw_fwd, tws,    \
                               dst_half, bitrev_out);                                                               \
        break;
    switch (logR) {
        FCASE(1) FCASE(2) FCASE(3) FCASE(4) FCASE(5) FCASE(6) FCASE(7) FCASE(8) FCASE(9) FCASE(10) FCASE(11) FCASE(12)
        FCASE(13)
        default: throw ArgError("bad fused radix");
    }
#undef FCASE
    HIP_CHECK(hipGetLastError());
}

// strided pass radices for the bits above the contiguous tile (top to bottom, i.e. DIF order): the 13-stage tile and
// the rest in balanced passes of at most 9 stages (a 9-stage pass first with an 11-stage tile was the faster 2^20
// plan only while that height's 7-stage pass was LDS-staged: profiles/r05_lde_plan_ab.txt, r05_lde_s8_ab.txt).
// allow10: 10 remaining stages as one k_ntt_s10 pass (the LDEs of 2^23: three HBM passes, not five)
static std::vector<int> strided_plan(int L, int &logC, bool allow10 = false) {
    logC = L < LOGC ? L : LOGC;
    int rem = L - logC;
    if (allow10 && rem == 10) return {10};
    std::vector<int> p;
    int np = (rem + LOGS - 1) / LOGS;
    for (int i = 0; i < np; i++) {
        int b = rem / (np - i);
        p.push_back(b);
        rem -= b;
    }
    return p;
}

// Twist tables f0(k) = shift^k / N, f1(k) = (shift w_2N)^k / N, k = hi*4096 + lo; cached per
// (N, shift) in the context (a handful of distinct pairs per machine), built once on the host.
static uint32_t host_rev(uint32_t x, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; i++) { r = (r << 1) | (x & 1u); x >>= 1; }
    return r;
}

static Twist get_twist(Ctx &c, uint64_t N, int L, uint32_t shift, hipStream_t s) {
    const int nhi = (int)((N + 4095) / 4096);
    const int ng = L > 13 ? 1 << (L - 13) : 0;
    const size_t per = 4096 + nhi + (ng ? 8192 + ng : 0);  // per coset
    auto make = [&](const uint32_t *p) {
        Twist t{p, p + 4096, p + per, p + per + 4096, nullptr, nullptr, nullptr, nullptr};
        if (ng) {
            t.u0 = p + 4096 + nhi;
            t.g0 = t.u0 + 8192;
            t.u1 = p + per + 4096 + nhi;
            t.g1 = t.u1 + 8192;
        }
        return t;
    };
    std::lock_guard<std::mutex> g(c.mu);
    for (auto &kv : c.twists)
        if (kv.first.first == L && kv.first.second == shift) return make(kv.second.p);
    std::vector<uint32_t> tt(2 * per);
    const uint32_t ninv = inv(to_mont((uint32_t)(N % P)));
    uint32_t sh[2] = {shift, mul(shift, two_adic_gen(L + 1))};
    for (int e = 0; e < 2; e++) {
        uint32_t *lo = tt.data() + e * per, *hi = lo + 4096;
        uint32_t x = ONE;
        for (int i = 0; i < 4096; i++) { lo[i] = x; x = mul(x, sh[e]); }
        uint32_t step = x;  // shift^4096
        uint32_t y = ninv;
        for (int i = 0; i < nhi; i++) { hi[i] = y; y = mul(y, step); }
        if (ng) {
            // u_e = s^(2^(L-13)); tile factor u_e^rev13(i), block factor s^rev_{L-13}(b) / N
            uint32_t *u = hi + nhi, *gg = u + 8192;
            const uint32_t ue = pow(sh[e], 1ull << (L - 13));
            std::vector<uint32_t> upow(8192);
            uint32_t z = ONE;
            for (int i = 0; i < 8192; i++) { upow[i] = z; z = mul(z, ue); }
            for (uint32_t t = 0; t < 512; t++)
                for (uint32_t j = 0; j < 16; j++) {
                    const uint32_t i = (t >> 1) * 32 + (t & 1) + 2 * j;
                    u[t * 16 + j] = upow[host_rev(i, 13)];
                }
            for (int b = 0; b < ng; b++) gg[b] = mul(pow(sh[e], host_rev((uint32_t)b, L - 13)), ninv);
        }
    }
    c.twists.emplace_back(std::make_pair(L, shift), DBuf(tt.size(), s));
    const uint32_t *p = c.twists.back().second.p;
    HIP_CHECK(hipMemcpyAsync((void *)p, tt.data(), tt.size() * 4, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));
    return make(p);
}

// Algorithmic GF operations of one column's blowup-2 coset LDE: iNTT over N,
// N twists, forward NTT over 2N = 3 (N/2) log N + N + 3 N log 2N (mul + add + sub per butterfly).
static double lde_gf_ops(uint64_t N) {
    const double L = (double)ilog2(N);
    return 3.0 * (N / 2.0) * L + (double)N + 3.0 * (double)N * (L + 1.0);
}

// Bit-reversed input evaluations (quotient chunks, produced bit-reversed by k_quotient):
//   DIT iNTT (bit-reversed in -> natural coefficients), twist on the last pass's write into both
//   LDE halves, then DIF in place (natural -> bit-reversed): no permutation pass at all.
void lde_batch_bitrev_in(Ctx &c, const DMat &src, uint32_t shift, DMat &dst, hipStream_t s) {
    ARG_CHECK(dst.height == 2 * src.height && dst.width == src.width, "LDE destination shape");
    lde_batch_bitrev_in_strided(c, src, shift, dst.d, 2 * src.height, s);
}

// dst column c at dst + c * dst_stride (dst_stride >= 2N): blowup 4 writes each half of a 4N-row column
void lde_batch_bitrev_in_strided(Ctx &c, const DMat &src, uint32_t shift, uint32_t *dst_d, uint64_t dst_stride,
                                 hipStream_t s) {
    const uint64_t N = src.height, W = src.width;
    if (!W) return;
    ARG_CHECK(dst_stride >= 2 * N, "LDE destination stride");
    DMat dst{dst_d, 2 * N, W};
    PROF("lde", s, 12.0 * N * W);
    prof_add("lde_gfops", lde_gf_ops(N) * W);
    const int L = ilog2(N);
    ARG_CHECK((1ull << L) == N && L >= 1, "LDE height must be a power of two >= 2");
    ARG_CHECK(L + 1 <= c.tw_log, "LDE larger than the twiddle tables");
    int logC;
    std::vector<int> sp = strided_plan(L, logC, true);
    const Twist tws = get_twist(c, N, L, shift, s);
    const uint32_t nv = (uint32_t)W;
    ColMap m_src{N, 0, 1}, m_dst1{dst_stride, 0, 1}, m_dst2{dst_stride, N, 2};
    if (sp.empty()) {
        run_contig<true>(logC, src.d, dst.d, m_src, m_dst1, nv, L, c.tw_inv, MODE_TWIST_OUT, tws, N, s);
    } else {
        DBuf work(N * W, s);
        run_contig<true>(logC, src.d, work.p, m_src, m_src, nv, L, c.tw_inv, MODE_PLAIN, tws, 0, s);
        int logS = logC;
        for (int i = (int)sp.size() - 1; i >= 0; i--) {
            const bool last = (i == 0);
            run_strided<true>(sp[i], work.p, last ? dst.d : work.p, m_src, last ? m_dst1 : m_src, nv, L, logS,
                              c.tw_inv, last ? MODE_TWIST_OUT : MODE_PLAIN, s, tws, N, 1u << c.tw_log);
            logS += sp[i];
        }
    }
    int logS = L;
    for (size_t i = 0; i < sp.size(); i++) {
        logS -= sp[i];
        run_strided<false>(sp[i], dst.d, dst.d, m_dst2, m_dst2, 2 * nv, L, logS, c.tw_fwd, MODE_PLAIN, s, Twist{}, 0,
                           1u << c.tw_log);
    }
    run_contig<false>(logC, dst.d, dst.d, m_dst2, m_dst2, 2 * nv, L, c.tw_fwd, MODE_PLAIN, Twist{}, 0, s);
}

// Columns per pass batch of the natural-input LDE: 16 (measured 4.62 ms vs 4.67 ms for all 67 columns of a
// 2^22 trace at once), 8 at 2^22 rows (with default-policy intermediate stores part of a batch's
// intermediates stay in the Infinity Cache: 2^22 x 64 3.49 -> 3.43 ms against 16, 3.47 at 4, 3.75 at 2;
// profiles/r05_lde_mall_ab.txt), 2 at 2^23 rows (k_ntt_s10's row-major intermediates: 2^23 x 64 7.24 ms against 7.38
// at 4, 7.78 at 8, 7.83 at 16; profiles/r06_cb23.txt), and up to a 256 MB work buffer for short traces (compress shapes,
// 2^14..2^18 rows: fewer launches; profiles/r03_lde_cb_ab.txt); ZKM_LDE_CB overrides (0 = all).
static uint32_t lde_col_batch(uint64_t N, uint32_t nv) {
    static const long env = [] {
        const char *e = getenv("ZKM_LDE_CB");
        return e ? atol(e) : -1L;
    }();
    uint64_t cb;
    if (env >= 0) cb = env ? (uint64_t)env : nv;
    else cb = N == (1ull << 22) ? 8 : N == (1ull << 23) ? 2 : std::max<uint64_t>(16, (1ull << 25) / N);
    return (uint32_t)std::min<uint64_t>(cb, nv);
}

// Natural-input LDE (traces):  [strided DIF iNTT passes] -> fused {contiguous DIF iNTT, twists,
// contiguous DIT forward x2} -> [strided DIT forward passes, the last writing bit-reversed rows].
void lde_batch(Ctx &c, const DMat &src, uint32_t shift, DMat &dst, hipStream_t s) {
    ARG_CHECK(dst.height == 2 * src.height && dst.width == src.width, "LDE destination shape");
    lde_batch_strided(c, src, shift, dst.d, 2 * src.height, s);
}

// nsh coset shifts (1, or 2 for blowup 4): the strided inverse passes run once per column batch
// into `winv` and each shift's fused + forward passes read it, writing the LDE of shift e at
// dst + e * half_off (column stride dst_stride).
static void lde_natural(Ctx &c, const DMat &src, const uint32_t *shifts, int nsh, uint32_t *dst_d,
                        uint64_t dst_stride, uint64_t half_off, hipStream_t s) {
    const uint64_t N = src.height, W = src.width;
    if (!W) return;
    ARG_CHECK(dst_stride >= (uint64_t)nsh * 2 * N, "LDE destination stride");
    PROF("lde", s, 12.0 * N * W * nsh);
    prof_add("lde_gfops", lde_gf_ops(N) * W * nsh);
    const int L = ilog2(N);
    ARG_CHECK((1ull << L) == N && L >= 1, "LDE height must be a power of two >= 2");
    ARG_CHECK(L + 1 <= c.tw_log, "LDE larger than the twiddle tables");
    int logC;
    std::vector<int> sp = strided_plan(L, logC, true);
    const uint32_t nv = (uint32_t)W;
    ColMap m_src{N, 0, 1}, m_w1{2 * N, 0, 1}, m_w2{2 * N, N, 2}, m_out{dst_stride, N, 2};
    if (sp.empty()) {
        for (int e = 0; e < nsh; e++)
            run_fused(logC, src.d, dst_d + e * half_off, m_src, ColMap{dst_stride, 0, 1}, nv, L, c.tw_inv, c.tw_fwd,
                      get_twist(c, N, L, shifts[e], s), N, 1, s);
        return;
    }
    // Columns go through all passes in batches of `cb`: a batch's work buffer (2N words per
    // column, [E0 | E1]; the iNTT runs in its first half) is written and re-read while it still
    // sits in the 256 MB Infinity Cache, so only the first read and the last write reach HBM.
    const uint32_t cb = lde_col_batch(N, nv);
    DBuf work(2 * N * cb, s);
    DBuf winv(nsh > 1 ? N * cb : 0, s);
    // the intermediates tile-major (the one-strided-pass size, 2^22): the strided passes read / write whole
    // 64 KB tiles, the VALU-bound fused pass takes the 128-B segments: LDE 4.05-4.13 -> 3.92-3.94 ms for 2^22 x 67
    // (profiles/r04_lde_tiled_plain_ab.txt; the pattern alone: profiles/r04_tile_probe.txt)
    const bool tiled = nsh == 1 && logC == 13 && sp.size() == 1 && sp[0] == 9;
    for (uint32_t c0 = 0; c0 < nv; c0 += cb) {
        const uint32_t nb = std::min(cb, nv - c0);
        const uint32_t *in = src.d + (uint64_t)c0 * N;
        // one shift: the inverse passes run in the work buffer's first half (fused in place)
        uint32_t *ibuf = nsh > 1 ? winv.p : work.p;
        const ColMap m_i = nsh > 1 ? m_src : m_w1;
        ColMap min = m_src;
        int logS = L;
        for (size_t i = 0; i < sp.size(); i++) {
            logS -= sp[i];
            run_strided<false>(sp[i], in, ibuf, min, m_i, nb, L, logS, c.tw_inv, MODE_PLAIN, s, Twist{}, 0,
                               1u << c.tw_log, tiled ? 2 : 0);
            in = ibuf;
            min = m_i;
        }
        for (int e = 0; e < nsh; e++) {
            const Twist tws = get_twist(c, N, L, shifts[e], s);
            uint32_t *out = dst_d + (uint64_t)c0 * dst_stride + e * half_off;
            if (logC == 13) {
                auto k = tiled ? k_lde_fused13s<true> : k_lde_fused13s<false>;
                hipLaunchKernelGGL(k, dim3((unsigned)(N >> 13), nb), dim3(t13::NTH), 0, s, ibuf, work.p, m_i, m_w1, L,
                                   c.tt_inv, c.tt_fwd, tws, N);
                HIP_CHECK(hipGetLastError());
            } else {
                run_fused(logC, ibuf, work.p, m_i, m_w1, nb, L, c.tw_inv, c.tw_fwd, tws, N, 0, s);
            }
            logS = logC;
            for (int i = (int)sp.size() - 1; i >= 0; i--) {
                const bool last = (i == 0);
                run_strided<true>(sp[i], work.p, last ? out : work.p, m_w2, last ? m_out : m_w2, 2 * nb, L, logS,
                                  c.tw_fwd, last ? MODE_BITREV_OUT : MODE_PLAIN, s, Twist{}, 0, 1u << c.tw_log,
                                  tiled ? 1 : 0);
                logS += sp[i];
            }
        }
    }
}

void lde_batch_strided(Ctx &c, const DMat &src, uint32_t shift, uint32_t *dst_d, uint64_t dst_stride, hipStream_t s) {
    lde_natural(c, src, &shift, 1, dst_d, dst_stride, 0, s);
}

// Blowup 4 of natural-order evaluations: rows [0, 2N) of every 4N-row column are the blowup-2 LDE
// with shift0, rows [2N, 4N) the one with shift1; the inverse transform is shared.
void lde_batch_blowup4(Ctx &c, const DMat &src, uint32_t shift0, uint32_t shift1, uint32_t *dst_d, hipStream_t s) {
    const uint32_t sh[2] = {shift0, shift1};
    lde_natural(c, src, sh, 2, dst_d, 4 * src.height, 2 * src.height, s);
}

}  // namespace zkm
