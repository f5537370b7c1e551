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

void launch_to_col_major(const uint32_t *d_in, uint64_t h, uint64_t w, bool mont_in, uint32_t *d_out, hipStream_t s) {
    if (!h || !w) return;
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
}

// ------------------------------------------------------------------ tile stage engine
// A tile lives in LDS as x[r * LD + t] (R rows, T columns, row pitch LD).  Row r, column t holds
// global index base + r*S + c0 + t, so the butterfly of a stage with half-size h = hr*S at lower
// row r uses w_{2h}^{(r mod hr)*S + c0 + t} = tw[h + (r mod hr)*S + c0 + t] (all indices < 2^24).
// Stages are processed G <= 3 at a time: each thread holds the 2^G elements a group of G stages
// touches in registers, so a tile makes one LDS round trip per 3 stages instead of per stage.
template <int G, int T, int LD, bool DIT>
__device__ __forceinline__ void stage_group(uint32_t *x, int R, int lc, const uint32_t *__restrict__ tw, uint32_t S,
                                            uint32_t c0) {
    constexpr int E = 1 << G;
    const int hrc = 1 << lc;
    const int ngroups = (R * T) >> G;
    for (int g = threadIdx.x; g < ngroups; g += NT) {
        const int t = g & (T - 1);
        const int q = g / T;
        const int rlow = q & (hrc - 1);
        const int r0 = ((q >> lc) << (lc + G)) | rlow;
        uint32_t v[E];
#pragma unroll
        for (int k = 0; k < E; k++) v[k] = x[(r0 + k * hrc) * LD + t];
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
        for (int k = 0; k < E; k++) x[(r0 + k * hrc) * LD + t] = v[k];
    }
    __syncthreads();
}

// All LOGR stages of a tile: DIT bottom-up (half-sizes 1,2,4,...), DIF top-down.
template <int LOGR, int T, int LD, bool DIT>
__device__ __forceinline__ void tile_stages(uint32_t *x, const uint32_t *__restrict__ tw, uint32_t S, uint32_t c0) {
    constexpr int R = 1 << LOGR;
    if (DIT) {
        int lc = 0;
        for (; lc + 3 <= LOGR; lc += 3) stage_group<3, T, LD, true>(x, R, lc, tw, S, c0);
        if (LOGR - lc == 2) stage_group<2, T, LD, true>(x, R, lc, tw, S, c0);
        else if (LOGR - lc == 1) stage_group<1, T, LD, true>(x, R, lc, tw, S, c0);
    } else {
        int rem = LOGR;
        for (; rem >= 3; rem -= 3) stage_group<3, T, LD, false>(x, R, rem - 3, tw, S, c0);
        if (rem == 2) stage_group<2, T, LD, false>(x, R, 0, tw, S, c0);
        else if (rem == 1) stage_group<1, T, LD, false>(x, R, 0, tw, S, c0);
    }
}

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
    __device__ __forceinline__ uint32_t f(int e, uint32_t k) const {
        return e ? mul(hi1[k >> 12], lo1[k & 4095]) : mul(hi0[k >> 12], lo0[k & 4095]);
    }
};

enum PassMode { MODE_PLAIN = 0, MODE_BITREV_OUT = 1, MODE_TWIST_OUT = 2 };

// Strided pass: rows at stride S = 2^logS inside outer blocks of R*S, tiles of T columns.
//   MODE_BITREV_OUT (last DIT pass, R*S == N): natural n = r*S + c goes to row rev_L(n).
//   MODE_TWIST_OUT  (last DIT pass of an inverse transform): natural coefficient n goes to both
//                   LDE halves multiplied by the coset twists f_0(n), f_1(n).
template <int LOGR, int T, bool DIT>
__global__ __launch_bounds__(NT) void k_ntt_strided(const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md,
                                                    int logS, const uint32_t *__restrict__ tw, int mode, Twist tws,
                                                    uint64_t dst_half) {
    constexpr int R = 1 << LOGR;
    constexpr int LD = T + 1;  // padded rows: conflict-free column walks (bit-reversed write)
    __shared__ uint32_t x[R * LD];
    const uint32_t S = 1u << logS;
    const uint32_t groups = S / T;
    const uint32_t tile = blockIdx.x;
    const uint32_t outer = tile / groups;
    const uint32_t c0 = (tile % groups) * T;
    const uint32_t base = outer * (uint32_t)R * S;
    const uint32_t *sp = src + ms.off(blockIdx.y);
    uint32_t *dp = dst + md.off(blockIdx.y);
    for (int i = threadIdx.x; i < R * T; i += NT) {
        const int r = i / T, t = i & (T - 1);
        x[r * LD + t] = sp[base + (uint32_t)r * S + c0 + t];
    }
    __syncthreads();
    tile_stages<LOGR, T, LD, DIT>(x, tw, S, c0);
    if (mode == MODE_PLAIN) {
        for (int i = threadIdx.x; i < R * T; i += NT) {
            const int r = i / T, t = i & (T - 1);
            dp[base + (uint32_t)r * S + c0 + t] = x[r * LD + t];
        }
    } else if (mode == MODE_TWIST_OUT) {
        for (int i = threadIdx.x; i < R * T; i += NT) {
            const int r = i / T, t = i & (T - 1);
            const uint32_t n = base + (uint32_t)r * S + c0 + t;
            const uint32_t v = x[r * LD + t];
            dp[n] = mul(v, tws.f(0, n));
            dp[dst_half + n] = mul(v, tws.f(1, n));
        }
    } else {
        for (int i = threadIdx.x; i < R * T; i += NT) {
            const int t = i / R, q = i & (R - 1);
            dp[(uint64_t)rev_bits(c0 + t, logS) * R + q] = x[(int)rev_bits((uint32_t)q, LOGR) * LD + t];
        }
    }
}

// Contiguous pass over blocks of R consecutive elements (bit-reversed-input pipeline):
//   MODE_PLAIN: stages only; MODE_TWIST_OUT: DIT (inverse) then twisted writes to both halves.
template <int LOGR, bool DIT>
__global__ __launch_bounds__(NT) void k_ntt_contig(const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md,
                                                   const uint32_t *__restrict__ tw, int mode, Twist tws,
                                                   uint64_t dst_half) {
    constexpr int R = 1 << LOGR;
    __shared__ uint32_t x[R];
    const uint32_t base = blockIdx.x * (uint32_t)R;
    const uint32_t *sp = src + ms.off(blockIdx.y) + base;
    for (int i = threadIdx.x; i < R; i += NT) x[i] = sp[i];
    __syncthreads();
    tile_stages<LOGR, 1, 1, DIT>(x, tw, 1, 0);
    uint32_t *dp = dst + md.off(blockIdx.y);
    if (mode == MODE_TWIST_OUT) {
        for (int i = threadIdx.x; i < R; i += NT) {
            const uint32_t n = base + i;
            dp[n] = mul(x[i], tws.f(0, n));
            dp[dst_half + n] = mul(x[i], tws.f(1, n));
        }
    } else {
        for (int i = threadIdx.x; i < R; i += NT) dp[base + i] = x[i];
    }
}

// Fused middle of the natural-input LDE: the inverse NTT's last (contiguous, DIF) pass, the two
// coset twists, and the first (contiguous, DIT) pass of both forward transforms, on one tile.
// The DIF output tile (bit-reversed coefficients) is exactly the DIT input tile, so the
// coefficients never round-trip through HBM.  bitrev_out: the whole transform fits the tile.
template <int LOGR>
__global__ __launch_bounds__(NT) void k_lde_fused(const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md, int L,
                                                  const uint32_t *__restrict__ tw_inv,
                                                  const uint32_t *__restrict__ tw_fwd, Twist tws, uint64_t dst_half,
                                                  int bitrev_out) {
    constexpr int R = 1 << LOGR;
    __shared__ uint32_t a[R];
    __shared__ uint32_t x[R];
    const uint32_t base = blockIdx.x * (uint32_t)R;
    const uint32_t *sp = src + ms.off(blockIdx.y) + base;
    for (int i = threadIdx.x; i < R; i += NT) a[i] = sp[i];
    __syncthreads();
    tile_stages<LOGR, 1, 1, false>(a, tw_inv, 1, 0);
    uint32_t *dcol = dst + md.off(blockIdx.y);
    for (int e = 0; e < 2; e++) {
        for (int i = threadIdx.x; i < R; i += NT) x[i] = mul(a[i], tws.f(e, rev_bits(base + i, L)));
        __syncthreads();
        tile_stages<LOGR, 1, 1, true>(x, tw_fwd, 1, 0);
        uint32_t *dp = dcol + (uint64_t)e * dst_half;
        if (!bitrev_out) {
            for (int i = threadIdx.x; i < R; i += NT) dp[base + i] = x[i];
        } else {
            for (int i = threadIdx.x; i < R; i += NT) dp[i] = x[rev_bits((uint32_t)i, LOGR)];
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ dispatch
static constexpr int LOGC = 13;  // contiguous tile: 8192 elements
static constexpr int LOGS = 9;   // strided radix per pass (512 rows x 32 columns)

static int strided_T(int logR) { return logR >= 9 ? 32 : 64; }

template <bool DIT>
static void run_strided(int logR, const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md, uint32_t nv, int L,
                        int logS, const uint32_t *tw, int mode, hipStream_t s, Twist tws = Twist{},
                        uint64_t dst_half = 0) {
    const int T = strided_T(logR);
    ARG_CHECK((1 << logS) >= T, "strided pass narrower than its tile");
    dim3 g((unsigned)(((1ull << L) >> logR) / T), nv);
#define SCASE(k, t)                                                                                             \
    case k:                                                                                                     \
        hipLaunchKernelGGL((k_ntt_strided<k, t, DIT>), g, dim3(NT), 0, s, src, dst, ms, md, logS, tw, mode, tws, \
                           dst_half);                                                                           \
        break;
    switch (logR) {
        SCASE(1, 64) SCASE(2, 64) SCASE(3, 64) SCASE(4, 64) SCASE(5, 64) SCASE(6, 64) SCASE(7, 64) SCASE(8, 64)
        SCASE(9, 32)
        default: throw ArgError("bad strided radix");
    }
#undef SCASE
    HIP_CHECK(hipGetLastError());
}

template <bool DIT>
static void run_contig(int logR, const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md, uint32_t nv, int L,
                       const uint32_t *tw, int mode, Twist tws, uint64_t dst_half, hipStream_t s) {
    dim3 g((unsigned)((1ull << L) >> logR), nv);
#define CCASE(k)                                                                                                 \
    case k:                                                                                                      \
        hipLaunchKernelGGL((k_ntt_contig<k, DIT>), g, dim3(NT), 0, s, src, dst, ms, md, tw, mode, tws, dst_half); \
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
        hipLaunchKernelGGL((k_lde_fused<k>), g, dim3(NT), 0, s, src, dst, ms, md, L, tw_inv, tw_fwd, tws, dst_half, \
                           bitrev_out);                                                                             \
        break;
    switch (logR) {
        FCASE(1) FCASE(2) FCASE(3) FCASE(4) FCASE(5) FCASE(6) FCASE(7) FCASE(8) FCASE(9) FCASE(10) FCASE(11) FCASE(12)
        FCASE(13)
        default: throw ArgError("bad fused radix");
    }
#undef FCASE
    HIP_CHECK(hipGetLastError());
}

// strided pass radices for the bits above the contiguous tile (top to bottom, i.e. DIF order)
static std::vector<int> strided_plan(int L, int &logC) {
    logC = L < LOGC ? L : LOGC;
    int rem = L - logC;
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
static Twist get_twist(Ctx &c, uint64_t N, int L, uint32_t shift, hipStream_t s) {
    const int nhi = (int)((N + 4095) / 4096);
    std::lock_guard<std::mutex> g(c.mu);
    for (auto &kv : c.twists)
        if (kv.first.first == L && kv.first.second == shift) {
            const uint32_t *p = kv.second.p;
            return Twist{p, p + 4096, p + 4096 + nhi, p + 2 * 4096 + nhi};
        }
    std::vector<uint32_t> tt(2 * (4096 + nhi));
    const uint32_t ninv = inv(to_mont((uint32_t)(N % P)));
    uint32_t sh[2] = {shift, mul(shift, two_adic_gen(L + 1))};
    for (int e = 0; e < 2; e++) {
        uint32_t *lo = tt.data() + e * (4096 + nhi), *hi = lo + 4096;
        uint32_t x = ONE;
        for (int i = 0; i < 4096; i++) { lo[i] = x; x = mul(x, sh[e]); }
        uint32_t step = x;  // shift^4096
        uint32_t y = ninv;
        for (int i = 0; i < nhi; i++) { hi[i] = y; y = mul(y, step); }
    }
    c.twists.emplace_back(std::make_pair(L, shift), DBuf(tt.size(), s));
    const uint32_t *p = c.twists.back().second.p;
    HIP_CHECK(hipMemcpyAsync((void *)p, tt.data(), tt.size() * 4, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));
    return Twist{p, p + 4096, p + 4096 + nhi, p + 2 * 4096 + nhi};
}

// Bit-reversed input evaluations (quotient chunks, produced bit-reversed by k_quotient):
//   DIT iNTT (bit-reversed in -> natural coefficients), twist on the last pass's write into both
//   LDE halves, then DIF in place (natural -> bit-reversed): no permutation pass at all.
void lde_batch_bitrev_in(Ctx &c, const DMat &src, uint32_t shift, DMat &dst, hipStream_t s) {
    const uint64_t N = src.height, W = src.width;
    if (!W) return;
    PROF("lde", s, 12.0 * N * W);
    const int L = ilog2(N);
    ARG_CHECK((1ull << L) == N && L >= 1, "LDE height must be a power of two >= 2");
    ARG_CHECK(L + 1 <= c.tw_log, "LDE larger than the twiddle tables");
    ARG_CHECK(dst.height == 2 * N && dst.width == W, "LDE destination shape");
    int logC;
    std::vector<int> sp = strided_plan(L, logC);
    const Twist tws = get_twist(c, N, L, shift, s);
    const uint32_t nv = (uint32_t)W;
    ColMap m_src{N, 0, 1}, m_dst1{2 * N, 0, 1}, m_dst2{2 * N, N, 2};
    if (sp.empty()) {
        run_contig<true>(logC, src.d, dst.d, m_src, m_dst1, nv, L, c.tw_inv, MODE_TWIST_OUT, tws, N, s);
    } else {
        DBuf work(N * W, s);
        run_contig<true>(logC, src.d, work.p, m_src, m_src, nv, L, c.tw_inv, MODE_PLAIN, tws, 0, s);
        int logS = logC;
        for (int i = (int)sp.size() - 1; i >= 0; i--) {
            const bool last = (i == 0);
            run_strided<true>(sp[i], work.p, last ? dst.d : work.p, m_src, last ? m_dst1 : m_src, nv, L, logS,
                              c.tw_inv, last ? MODE_TWIST_OUT : MODE_PLAIN, s, tws, N);
            logS += sp[i];
        }
    }
    int logS = L;
    for (size_t i = 0; i < sp.size(); i++) {
        logS -= sp[i];
        run_strided<false>(sp[i], dst.d, dst.d, m_dst2, m_dst2, 2 * nv, L, logS, c.tw_fwd, MODE_PLAIN, s);
    }
    run_contig<false>(logC, dst.d, dst.d, m_dst2, m_dst2, 2 * nv, L, c.tw_fwd, MODE_PLAIN, Twist{}, 0, s);
}

// Natural-input LDE (traces):  [strided DIF iNTT passes] -> fused {contiguous DIF iNTT, twists,
// contiguous DIT forward x2} -> [strided DIT forward passes, the last writing bit-reversed rows].
void lde_batch(Ctx &c, const DMat &src, uint32_t shift, DMat &dst, hipStream_t s) {
    const uint64_t N = src.height, W = src.width;
    if (!W) return;
    PROF("lde", s, 12.0 * N * W);
    const int L = ilog2(N);
    ARG_CHECK((1ull << L) == N && L >= 1, "LDE height must be a power of two >= 2");
    ARG_CHECK(L + 1 <= c.tw_log, "LDE larger than the twiddle tables");
    ARG_CHECK(dst.height == 2 * N && dst.width == W, "LDE destination shape");
    int logC;
    std::vector<int> sp = strided_plan(L, logC);
    const Twist tws = get_twist(c, N, L, shift, s);
    const uint32_t nv = (uint32_t)W;
    ColMap m_src{N, 0, 1}, m_w1{2 * N, 0, 1}, m_w2{2 * N, N, 2};
    if (sp.empty()) {
        run_fused(logC, src.d, dst.d, m_src, m_w1, nv, L, c.tw_inv, c.tw_fwd, tws, N, 1, s);
        return;
    }
    // work buffer: per column 2N ([E0 | E1]); the iNTT runs in its first half
    DBuf work(2 * N * W, s);
    const uint32_t *in = src.d;
    ColMap min = m_src;
    int logS = L;
    for (size_t i = 0; i < sp.size(); i++) {
        logS -= sp[i];
        run_strided<false>(sp[i], in, work.p, min, m_w1, nv, L, logS, c.tw_inv, MODE_PLAIN, s);
        in = work.p;
        min = m_w1;
    }
    run_fused(logC, work.p, work.p, m_w1, m_w1, nv, L, c.tw_inv, c.tw_fwd, tws, N, 0, s);
    logS = logC;
    for (int i = (int)sp.size() - 1; i >= 0; i--) {
        const bool last = (i == 0);
        run_strided<true>(sp[i], work.p, last ? dst.d : work.p, m_w2, last ? m_w2 : m_w2, 2 * nv, L, logS, c.tw_fwd,
                          last ? MODE_BITREV_OUT : MODE_PLAIN, s);
        logS += sp[i];
    }
}

}  // namespace zkm
