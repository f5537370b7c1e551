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
// Passes: the lowest <= 12 bits in one contiguous LDS tile (4096 elements), the remaining bits
// in strided passes of <= 6 bits over 64-column-wide tiles (256 B coalesced rows).
#include "internal.hpp"
#include "prof.hpp"

namespace zkm {

using namespace kb;

static constexpr int NT = 256;          // threads per workgroup
static constexpr int LOGC_MAX = 12;     // contiguous tile: 4096 elements
static constexpr int LOGS_MAX = 6;      // strided tile radix
static constexpr int TS = 64;           // strided tile width (columns of 4 B)

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

// ------------------------------------------------------------------ tile stages
// LDS tile x[r * T + t], R = 2^LOGR rows, T columns.  Global lower index of a butterfly at
// (row r_lo, column t) is n = base + r_lo * S + c0 + t, stage half-size h = hr * S.
template <int LOGR, int T, bool DIT>
__device__ __forceinline__ void tile_stages(uint32_t *x, const uint32_t *__restrict__ tw, uint64_t S, uint64_t c0) {
    constexpr int R = 1 << LOGR;
    constexpr int NB = R * T / 2;
#pragma unroll 1
    for (int st = 0; st < LOGR; st++) {
        const int lhr = DIT ? st : (LOGR - 1 - st);
        const int hr = 1 << lhr;
        const uint64_t h = (uint64_t)hr * S;
        for (int b = threadIdx.x; b < NB; b += NT) {
            const int t = b & (T - 1);
            const int p = b / T;
            const int rlo = ((p >> lhr) << (lhr + 1)) | (p & (hr - 1));
            const uint64_t j = (uint64_t)(p & (hr - 1)) * S + c0 + t;
            const uint32_t w = tw[h + j];
            uint32_t *lo = x + rlo * T + t;
            uint32_t *hi = lo + hr * T;
            uint32_t u = *lo, v = *hi;
            if (DIT) {
                v = mul(v, w);
                *lo = add(u, v);
                *hi = sub(u, v);
            } else {
                *lo = add(u, v);
                *hi = mul(sub(u, v), w);
            }
        }
        __syncthreads();
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

// Strided pass: rows r at stride S within outer blocks of R*S; 64-column tiles.
struct Twist {
    const uint32_t *lo0, *hi0, *lo1, *hi1;
    __device__ __forceinline__ uint32_t f(int e, uint32_t k) const {
        return e ? mul(hi1[k >> 12], lo1[k & 4095]) : mul(hi0[k >> 12], lo0[k & 4095]);
    }
};

template <int LOGR, bool DIT>
__global__ __launch_bounds__(NT) void k_ntt_strided(const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md,
                                                    int L, int logS, const uint32_t *__restrict__ tw, int bitrev_out,
                                                    Twist tws, int twist_out, uint64_t dst_half) {
    constexpr int R = 1 << LOGR;
    constexpr int T = TS;
    __shared__ uint32_t x[R * T];
    const uint64_t S = 1ull << logS;
    const uint64_t groups = S / T;
    const uint64_t tile = blockIdx.x;
    const uint64_t outer = tile / groups;
    const uint64_t c0 = (tile % groups) * T;
    const uint64_t base = outer * (uint64_t)R * S;
    const uint32_t *sp = src + ms.off(blockIdx.y);
    uint32_t *dp = dst + md.off(blockIdx.y);
    for (int i = threadIdx.x; i < R * T; i += NT) {
        const int r = i / T, t = i & (T - 1);
        x[i] = sp[base + (uint64_t)r * S + c0 + t];
    }
    __syncthreads();
    tile_stages<LOGR, T, DIT>(x, tw, S, c0);
    if (twist_out) {
        // natural coefficient index n -> two twisted outputs (E0, E1 halves)
        for (int i = threadIdx.x; i < R * T; i += NT) {
            const int r = i / T, t = i & (T - 1);
            const uint64_t n = base + (uint64_t)r * S + c0 + t;
            dp[n] = mul(x[i], tws.f(0, (uint32_t)n));
            dp[dst_half + n] = mul(x[i], tws.f(1, (uint32_t)n));
        }
    } else if (!bitrev_out) {
        for (int i = threadIdx.x; i < R * T; i += NT) {
            const int r = i / T, t = i & (T - 1);
            dp[base + (uint64_t)r * S + c0 + t] = x[i];
        }
    } else {
        // last pass (outer == 0, R*S == N): natural n = r*S + c -> row rev_L(n) = rev_S(c)*R + rev_R(r)
        for (int i = threadIdx.x; i < R * T; i += NT) {
            const int t = i / R, q = i & (R - 1);
            const uint64_t c = c0 + t;
            const uint32_t r = rev_bits((uint32_t)q, LOGR);
            dp[(uint64_t)rev_bits((uint32_t)c, logS) * R + q] = x[r * T + t];
        }
    }
}

// Contiguous pass over blocks of R consecutive elements.
//   twist != nullptr (DIT only): input = bit-reversed coefficients; for e in {0,1} the tile is
//   multiplied by f_e(k) = hi_e[k >> 12] * lo_e[k & 4095] (k = rev_L(n)) and transformed into
//   dst + md.off(v) + e * dst_half.
//   bitrev_out: single-pass transform (R == N): write natural n to row rev_L(n).
template <int LOGR, bool DIT>
__global__ __launch_bounds__(NT) void k_ntt_contig(const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md,
                                                   int L, const uint32_t *__restrict__ tw, int bitrev_out,
                                                   Twist tws, int use_twist, uint64_t dst_half) {
    constexpr int R = 1 << LOGR;
    __shared__ uint32_t a[R];
    __shared__ uint32_t x[R];
    const uint64_t base = (uint64_t)blockIdx.x * R;
    const uint32_t *sp = src + ms.off(blockIdx.y) + base;
    for (int i = threadIdx.x; i < R; i += NT) a[i] = sp[i];
    __syncthreads();
    if (use_twist == 2) {
        // twist on output: natural coefficient n -> E0 / E1 halves (DIT iNTT of bit-reversed input)
        for (int i = threadIdx.x; i < R; i += NT) x[i] = a[i];
        __syncthreads();
        tile_stages<LOGR, 1, DIT>(x, tw, 1, 0);
        uint32_t *dp = dst + md.off(blockIdx.y);
        for (int i = threadIdx.x; i < R; i += NT) {
            const uint32_t n = (uint32_t)(base + i);
            dp[n] = mul(x[i], tws.f(0, n));
            dp[dst_half + n] = mul(x[i], tws.f(1, n));
        }
        return;
    }
    const int ne = use_twist ? 2 : 1;
    for (int e = 0; e < ne; e++) {
        for (int i = threadIdx.x; i < R; i += NT) {
            uint32_t v = a[i];
            if (use_twist) v = mul(v, tws.f(e, rev_bits((uint32_t)(base + i), L)));
            x[i] = v;
        }
        __syncthreads();
        tile_stages<LOGR, 1, DIT>(x, tw, 1, 0);
        uint32_t *dp = dst + md.off(blockIdx.y) + (uint64_t)e * dst_half;
        if (!bitrev_out) {
            for (int i = threadIdx.x; i < R; i += NT) dp[base + i] = x[i];
        } else {
            for (int i = threadIdx.x; i < R; i += NT) dp[i] = x[rev_bits((uint32_t)i, LOGR)];
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ dispatch
template <bool DIT>
static void run_strided(int logR, const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md, uint32_t nv, int L,
                        int logS, const uint32_t *tw, int bitrev_out, hipStream_t s, Twist tws = Twist{},
                        int twist_out = 0, uint64_t dst_half = 0) {
    uint64_t tiles = (1ull << L) >> (logR + 6);
    dim3 g((unsigned)tiles, nv);
#define SCASE(k) \
    case k: hipLaunchKernelGGL((k_ntt_strided<k, DIT>), g, dim3(NT), 0, s, src, dst, ms, md, L, logS, tw, bitrev_out, tws, twist_out, dst_half); break;
    switch (logR) { SCASE(1) SCASE(2) SCASE(3) SCASE(4) SCASE(5) SCASE(6) default: throw ArgError("bad strided radix"); }
#undef SCASE
    HIP_CHECK(hipGetLastError());
}

template <bool DIT>
static void run_contig(int logR, const uint32_t *src, uint32_t *dst, ColMap ms, ColMap md, uint32_t nv, int L,
                       const uint32_t *tw, int bitrev_out, Twist tws, int use_twist, uint64_t dst_half, hipStream_t s) {
    uint64_t tiles = (1ull << L) >> logR;
    dim3 g((unsigned)tiles, nv);
#define CCASE(k)                                                                                             \
    case k:                                                                                                  \
        hipLaunchKernelGGL((k_ntt_contig<k, DIT>), g, dim3(NT), 0, s, src, dst, ms, md, L, tw, bitrev_out, tws, \
                           use_twist, dst_half);                                                             \
        break;
    switch (logR) {
        CCASE(1) CCASE(2) CCASE(3) CCASE(4) CCASE(5) CCASE(6) CCASE(7) CCASE(8) CCASE(9) CCASE(10) CCASE(11) CCASE(12)
        default: throw ArgError("bad contiguous radix");
    }
#undef CCASE
    HIP_CHECK(hipGetLastError());
}

// strided pass radices for the bits above the contiguous tile (top to bottom, i.e. DIF order)
static std::vector<int> strided_plan(int L, int &logC) {
    logC = L < LOGC_MAX ? L : LOGC_MAX;
    int rem = L - logC;
    std::vector<int> p;
    int np = (rem + LOGS_MAX - 1) / LOGS_MAX;
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
        run_contig<true>(logC, src.d, dst.d, m_src, m_dst1, nv, L, c.tw_inv, 0, tws, 2, N, s);
    } else {
        DBuf work(N * W, s);
        run_contig<true>(logC, src.d, work.p, m_src, m_src, nv, L, c.tw_inv, 0, tws, 0, 0, s);
        int logS = logC;
        for (int i = (int)sp.size() - 1; i >= 0; i--) {
            const bool last = (i == 0);
            run_strided<true>(sp[i], work.p, last ? dst.d : work.p, m_src, last ? m_dst1 : m_src, nv, L, logS,
                              c.tw_inv, 0, s, tws, last ? 1 : 0, N);
            logS += sp[i];
        }
    }
    // forward DIF in place on both halves
    int logS = L;
    for (size_t i = 0; i < sp.size(); i++) {
        logS -= sp[i];
        run_strided<false>(sp[i], dst.d, dst.d, m_dst2, m_dst2, 2 * nv, L, logS, c.tw_fwd, 0, s);
    }
    run_contig<false>(logC, dst.d, dst.d, m_dst2, m_dst2, 2 * nv, L, c.tw_fwd, 0, Twist{}, 0, 0, s);
}

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

    // work buffer: per column 2N ([E0 | E1]); the iNTT runs in its first half
    DBuf work(2 * N * W, s);
    ColMap m_src{N, 0, 1};
    ColMap m_w1{2 * N, 0, 1};       // one virtual column per column, first half
    ColMap m_w2{2 * N, N, 2};       // two virtual columns per column (E0, E1)
    ColMap m_dst2{2 * N, N, 2};     // LDE halves
    const uint32_t nv = (uint32_t)W;

    // 1. iNTT (DIF, inverse twiddles): strided passes top-down, then contiguous
    const uint32_t *in = src.d;
    ColMap min = m_src;
    int logS = L;
    for (size_t i = 0; i < sp.size(); i++) {
        logS -= sp[i];
        run_strided<false>(sp[i], in, work.p, min, m_w1, nv, L, logS, c.tw_inv, 0, s);
        in = work.p;
        min = m_w1;
    }
    run_contig<false>(logC, in, work.p, min, m_w1, nv, L, c.tw_inv, 0, tws, 0, 0, s);

    // 2./3. forward DIT for E0 and E1
    const bool single = sp.empty();
    if (single) {
        // twist + full transform + bit-reversed write straight into the LDE
        run_contig<true>(logC, work.p, dst.d, m_w1, m_w1, nv, L, c.tw_fwd, 1, tws, 1, N, s);
        return;
    }
    run_contig<true>(logC, work.p, work.p, m_w1, m_w1, nv, L, c.tw_fwd, 0, tws, 1, N, s);
    logS = logC;
    for (int i = (int)sp.size() - 1; i >= 0; i--) {
        const bool last = (i == 0);
        run_strided<true>(sp[i], work.p, last ? dst.d : work.p, m_w2, last ? m_dst2 : m_w2, 2 * nv, L, logS, c.tw_fwd,
                          last ? 1 : 0, s);
        logS += sp[i];
    }
}

}  // namespace zkm
