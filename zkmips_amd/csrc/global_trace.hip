// Device trace of the Global chip (crates/core/machine/src/global/mod.rs:77-196): every cross-shard
// lookup message lifted onto the septic curve (GlobalLookupOperation::populate,
// operations/global_lookup.rs:26-90) and the running sum of the points from the zero digest
// (GlobalAccumulationOperation, global_accumulation.rs), i.e. the chip's whole trace and the shard's
// global cumulative sum.  The reference computes the sum with a parallel scan
// (`into_par_iter().scan`, global/mod.rs:162-166); this is the same scan as a three-level device scan.
// The curve group law is associative, so any bracketing gives the host's sequential fold bit for bit.
//
// Septic arithmetic (F_p[z]/(z^7 + 2z - 8), Montgomery form): the same algorithms as the host
// restatement zkmips_amd/csrc/host/septic.cpp (septic_extension.rs: mul :300-316, frobenius
// :575-598, inverse :601-613, sqrt :615-674; septic_curve.rs: curve_formula :101-122, add :53-84,
// lift_x :130-154).  Compute-bound (≈45k lane instructions per lift, ≈10k per point addition): one
// thread per message for the lift, 2048 points per workgroup for the scan.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/zkm_hip.h"
#include "../../include/zkm_tracegen.h"
#include "kb31.cuh"

namespace zkm {
extern thread_local std::string g_last_error;
}
using zkm::g_last_error;

static_assert(sizeof(zkm_global_lookup_event) == 32, "GlobalLookupEvent layout");

namespace zkm::sep {
using namespace kb;

struct S7 {
    uint32_t c[7];
};
struct Pt {  // affine point or infinity, Montgomery coordinates
    S7 x, y;
    uint32_t inf;
};

__device__ __forceinline__ S7 s_zero() {
    S7 r;
#pragma unroll
    for (int i = 0; i < 7; i++) r.c[i] = 0;
    return r;
}
__device__ __forceinline__ S7 s_base(uint32_t a) {
    S7 r = s_zero();
    r.c[0] = a;
    return r;
}
__device__ __forceinline__ bool s_eq(const S7 &a, const S7 &b) {
    bool e = true;
#pragma unroll
    for (int i = 0; i < 7; i++) e &= a.c[i] == b.c[i];
    return e;
}
__device__ __forceinline__ S7 s_add(S7 a, const S7 &b) {
#pragma unroll
    for (int i = 0; i < 7; i++) a.c[i] = add(a.c[i], b.c[i]);
    return a;
}
__device__ __forceinline__ S7 s_sub(S7 a, const S7 &b) {
#pragma unroll
    for (int i = 0; i < 7; i++) a.c[i] = sub(a.c[i], b.c[i]);
    return a;
}
__device__ __forceinline__ S7 s_neg(S7 a) {
#pragma unroll
    for (int i = 0; i < 7; i++) a.c[i] = neg(a.c[i]);
    return a;
}
__device__ __forceinline__ S7 s_scale(S7 a, uint32_t k) {
#pragma unroll
    for (int i = 0; i < 7; i++) a.c[i] = mul(a.c[i], k);
    return a;
}
// schoolbook product, then z^7 = 8 - 2z.  Two 62-bit products share one Montgomery reduction
// (2 p^2 < p 2^32), halving the reductions of the 49 products.
__device__ __noinline__ S7 s_mul(S7 a, S7 b) {
    uint32_t t[13];
#pragma unroll
    for (int k = 0; k < 13; k++) {
        const int lo = k < 7 ? 0 : k - 6, hi = k < 7 ? k : 6;
        uint32_t acc = 0;
        int i = lo;
#pragma unroll
        for (; i + 1 <= hi; i += 2)
            acc = add(acc, redc(prod64(a.c[i], b.c[k - i]) + prod64(a.c[i + 1], b.c[k - i - 1])));
        if (i == hi) acc = add(acc, redc(prod64(a.c[i], b.c[k - i])));
        t[k] = acc;
    }
#pragma unroll
    for (int i = 12; i >= 7; i--) {
        t[i - 7] = add(t[i - 7], dbl(dbl(dbl(t[i]))));
        t[i - 6] = sub(t[i - 6], dbl(t[i]));
    }
    S7 r;
#pragma unroll
    for (int i = 0; i < 7; i++) r.c[i] = t[i];
    return r;
}
__device__ __forceinline__ S7 s_sq(S7 a) { return s_mul(a, a); }

// Frobenius maps x -> x^{p^k} (k = 1, 2, 3, 5) as 7x7 F_p-matrices (columns z^{i p^k}), filled once
// per call by k_septic_init.
struct Frob {
    S7 col[7];
};
__device__ Frob g_frob[4];  // p, p^2, p^3, p^5

__device__ __noinline__ S7 frob_apply(const Frob *f, S7 a) {
    S7 r = s_zero();
#pragma unroll
    for (int i = 0; i < 7; i++) r = s_add(r, s_scale(f->col[i], a.c[i]));
    return r;
}
__device__ S7 s_pow(S7 a, uint64_t e) {
    S7 r = s_base(ONE);
    while (e) {
        if (e & 1) r = s_mul(r, a);
        a = s_sq(a);
        e >>= 1;
    }
    return r;
}

__global__ void k_septic_init() {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    S7 z = s_zero();
    z.c[1] = ONE;
    const S7 zp = s_pow(z, P);
    S7 acc = s_base(ONE);
    for (int i = 0; i < 7; i++) {
        g_frob[0].col[i] = acc;
        acc = s_mul(acc, zp);
    }
    for (int i = 0; i < 7; i++) g_frob[1].col[i] = frob_apply(&g_frob[0], g_frob[0].col[i]);
    for (int i = 0; i < 7; i++) g_frob[2].col[i] = frob_apply(&g_frob[0], g_frob[1].col[i]);
    for (int i = 0; i < 7; i++) g_frob[3].col[i] = frob_apply(&g_frob[1], g_frob[2].col[i]);
}

__device__ __forceinline__ S7 s_pow_r_1(const S7 &a) {  // a^{p + p^2 + ... + p^6}
    const S7 b = s_mul(frob_apply(&g_frob[0], a), frob_apply(&g_frob[1], a));
    const S7 b2 = frob_apply(&g_frob[1], b), b4 = frob_apply(&g_frob[1], b2);
    return s_mul(s_mul(b, b2), b4);
}
__device__ __forceinline__ S7 s_inv(const S7 &a) {
    const S7 r1 = s_pow_r_1(a);
    return s_scale(r1, inv(s_mul(r1, a).c[0]));
}

// Tonelli-Shanks in F_p (p - 1 = 127 * 2^24; 3 is a non-residue), Montgomery form
__device__ bool sqrt_p(uint32_t n, uint32_t &out) {
    if (n == 0) {
        out = 0;
        return true;
    }
    if (kb::pow(n, (P - 1) / 2) != ONE) return false;
    // kb::pow spelled out: an unqualified pow(uint32_t, int) would pick <cmath>'s floating-point template
    uint32_t M = 24, c = kb::pow(to_mont(3), 127), t = kb::pow(n, 127), R = kb::pow(n, 64);
    for (int guard = 0; t != ONE && guard < 32; guard++) {  // at most 24 rounds; the caps only bound a bug
        uint32_t i = 0, tt = t;
        while (tt != ONE && i < 32) {
            tt = sqr(tt);
            i++;
        }
        uint32_t b = c;
        for (uint32_t k = 0; k + i + 1 < M; k++) b = sqr(b);
        M = i;
        c = sqr(b);
        t = mul(t, c);
        R = mul(R, b);
    }
    out = R;
    return true;
}

// a is a square in F_{p^7} (odd degree) iff its norm N(a) = a^{1 + p + ... + p^6} is a square in F_p;
// the host's s_sqrt fails exactly when sqrt_p(N(a)^-1) does.  Returns N(a) in *nrm.
__device__ __forceinline__ bool s_is_square(const S7 &a, uint32_t *nrm) {
    if (s_eq(a, s_zero()) || s_eq(a, s_base(ONE))) {
        *nrm = ONE;
        return true;
    }
    *nrm = s_mul(s_pow_r_1(a), a).c[0];
    return kb::pow(*nrm, (P - 1) / 2) == ONE;
}

// sqrt(a) = a * (a^{(p+1)/2})^{p + p^3 + p^5} * sqrt(N(a))^-1, for a square a with norm nrm
__device__ S7 s_sqrt_known(const S7 &a, uint32_t nrm) {
    if (s_eq(a, s_zero()) || s_eq(a, s_base(ONE))) return a;
    uint32_t r = 0;
    sqrt_p(inv(nrm), r);
    const S7 h = s_pow(a, ((uint64_t)P + 1) / 2);
    const S7 d = s_mul(s_mul(frob_apply(&g_frob[0], h), frob_apply(&g_frob[2], h)), frob_apply(&g_frob[3], h));
    return s_scale(s_mul(d, a), r);
}

__device__ __forceinline__ S7 curve_formula(const S7 &x) {  // x^3 + 3z x - 3
    S7 z3 = s_zero();
    z3.c[1] = to_mont(3);
    return s_sub(s_add(s_mul(s_sq(x), x), s_mul(x, z3)), s_base(to_mont(3)));
}

__device__ Pt add_complete(const Pt &a, const Pt &b) {
    if (a.inf) return b;
    if (b.inf) return a;
    Pt r;
    r.inf = 0;
    S7 slope;
    if (!s_eq(a.x, b.x)) {
        slope = s_mul(s_sub(b.y, a.y), s_inv(s_sub(b.x, a.x)));
    } else if (s_eq(a.y, b.y)) {  // doubling
        S7 num = s_scale(s_sq(a.x), to_mont(3));
        num.c[1] = add(num.c[1], to_mont(3));
        slope = s_mul(num, s_inv(s_add(a.y, a.y)));
    } else {
        r.x = s_zero();
        r.y = s_zero();
        r.inf = 1;
        return r;
    }
    r.x = s_sub(s_sub(s_sq(slope), a.x), b.x);
    r.y = s_sub(s_mul(slope, s_sub(a.x, r.x)), a.y);
    return r;
}

__device__ __forceinline__ Pt load_pt(const uint32_t *p) {
    Pt r;
#pragma unroll
    for (int i = 0; i < 7; i++) {
        r.x.c[i] = p[i];
        r.y.c[i] = p[7 + i];
    }
    r.inf = p[14];
    return r;
}
__device__ __forceinline__ void store_pt(uint32_t *p, const Pt &a) {
#pragma unroll
    for (int i = 0; i < 7; i++) {
        p[i] = a.x.c[i];
        p[7 + i] = a.y.c[i];
    }
    p[14] = a.inf;
}
constexpr int PW = 15;  // words per stored point

// septic_digest.rs:8-22 (CURVE_CUMULATIVE_SUM_START), septic_curve.rs:17-24 (dummy point), canonical
__constant__ uint32_t START[14] = {637514027u, 1595065213u, 1998064738u, 72333738u,  1211544370u,
                                   822986770u, 1518535784u, 1604177449u, 90440090u,  259343427u,
                                   140470264u, 1162099742u, 941559812u,  1064053343u};
__constant__ uint32_t DUMMY[14] = {1706420302u, 1319108093u, 148224806u,  26874985u,  1766171812u,
                                   1645633948u, 2028659224u, 942390502u,  1239997438u, 458866455u,
                                   1843332012u, 1309764648u, 572807436u,  74267719u};
__device__ __forceinline__ Pt const_pt(const uint32_t *c) {
    Pt r;
#pragma unroll
    for (int i = 0; i < 7; i++) {
        r.x.c[i] = to_mont(c[i]);
        r.y.c[i] = to_mont(c[7 + i]);
    }
    r.inf = 0;
    return r;
}

// GlobalCols (global/mod.rs:48-60; mips_memory.py G_*)
enum { G_MSG = 0, G_KIND = 7, G_OFFSET = 8, G_X = 16, G_Y = 23, G_Y6BITS = 30, G_RCW = 60, G_IS_RECEIVE = 61,
       G_IS_SEND = 62, G_REAL = 63, G_INIT_X = 64, G_SUMCHK = 78, G_CUM_X = 85, G_WIDTH = 99 };
constexpr uint32_t HALF = (P - 1) / 2, HALF_PLUS = (P + 1) / 2;
enum { ERR_NO_LIFT = 1, ERR_INFINITY = 2, ERR_U16 = 4 };

// one thread per message: lift, the lookup half of the row (columns 0..63), the point for the scan
__global__ __launch_bounds__(256) void k_global_lift(const uint32_t *__restrict__ ev, uint64_t n,
                                                     uint32_t *__restrict__ trace, uint32_t *__restrict__ pts,
                                                     uint32_t *byte_mult, uint32_t *err) {
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;; e += (uint64_t)gridDim.x * blockDim.x) {
        const bool live = e < n;
        uint32_t msg0 = 0;
        if (live) {
            const uint32_t *r = ev + 8 * e;  // message[7], then is_receive (byte 0), kind (byte 1)
            const uint32_t is_receive = r[7] & 0xFF, kind = (r[7] >> 8) & 0xFF;
            msg0 = r[0];
            S7 m;
#pragma unroll
            for (int i = 0; i < 7; i++) m.c[i] = to_mont(r[i] % P);
            m.c[0] = add(m.c[0], to_mont((kind << 16) % P));
            // lift_x with the smallest offset whose x has a curve point with y_6 != 0.  The cheap
            // squareness test (the norm's Legendre symbol) runs per offset; the square root, ~6x the
            // cost, runs once per lane after the lanes of a wave have found their offsets, so a wave
            // pays for one root instead of one per offset at which some lane succeeds.
            S7 x, y = s_zero();
            uint32_t off = 0;
            bool ok = false;
            while (off < 256) {
                uint32_t nrm = 0;
                S7 f = s_zero();
                for (; off < 256; off++) {
                    x = m;
                    x.c[6] = add(mul(m.c[6], to_mont(256)), to_mont(off));
                    f = curve_formula(x);
                    if (s_is_square(f, &nrm)) break;
                }
                if (off == 256) break;
                y = s_sqrt_known(f, nrm);
                if (y.c[6] != 0) {  // not the exceptional y_6 = 0: done
                    ok = true;
                    break;
                }
                off++;
            }
            if (!ok) {
                atomicOr(err, (uint32_t)ERR_NO_LIFT);
                off = 0;
                x = s_zero();
                y = s_zero();
            }
            if (from_mont(y.c[6]) > HALF) y = s_neg(y);  // is_send normalisation
            if (!is_receive) y = s_neg(y);
            uint32_t *row = trace + G_WIDTH * e;
#pragma unroll
            for (int i = 0; i < 7; i++) row[G_MSG + i] = r[i];
            row[G_KIND] = kind;
#pragma unroll
            for (int i = 0; i < 8; i++) row[G_OFFSET + i] = (off >> i) & 1;
            S7 xc, yc;
#pragma unroll
            for (int i = 0; i < 7; i++) {
                xc.c[i] = from_mont(x.c[i]);
                yc.c[i] = from_mont(y.c[i]);
                row[G_X + i] = xc.c[i];
                row[G_Y + i] = yc.c[i];
            }
            const uint32_t rcv = is_receive ? yc.c[6] - 1u : yc.c[6] - HALF_PLUS;
            uint32_t top = 0;
#pragma unroll
            for (int i = 0; i < 30; i++) {
                const uint32_t b = (rcv >> i) & 1;
                row[G_Y6BITS + i] = b;
                if (i >= 23) top += b;
            }
            row[G_RCW] = from_mont(inv(to_mont((top + P - 7) % P)));
            row[G_IS_RECEIVE] = is_receive;
            row[G_IS_SEND] = 1 - is_receive;
            row[G_REAL] = 1;
            Pt p;
            p.x = x;
            p.y = y;
            p.inf = 0;
            store_pt(pts + PW * e, p);
            if (msg0 >= 65536) atomicOr(err, (uint32_t)ERR_U16);
        }
        // U16Range(message[0]) (global/mod.rs:93-101): one atomic per wave for a wave-uniform shard
        if (byte_mult) {
            const bool on = live && msg0 < 65536;
            const uint64_t act = __ballot(on);
            if (act) {
                const int leader = __ffsll((unsigned long long)act) - 1;
                const uint32_t lead = __shfl(msg0, leader);
                const uint64_t same = __ballot(on && msg0 == lead);
                if ((int)(threadIdx.x & 63) == leader) atomicAdd(byte_mult + lead * 10u + 8u, (uint32_t)__popcll(same));
                if (on && msg0 != lead) atomicAdd(byte_mult + msg0 * 10u + 8u, 1u);
            }
        }
        if (__ballot(e + (uint64_t)gridDim.x * blockDim.x < n) == 0) break;  // wave-uniform exit
    }
}

// Block-local inclusive scan of 2048 points (256 threads x 8): pts[i] <- local prefix, tot[b] <- block sum
constexpr int SCAN_T = 256, SCAN_K = 8, SCAN_CHUNK = SCAN_T * SCAN_K;
__global__ __launch_bounds__(SCAN_T) void k_scan_local(uint32_t *pts, uint64_t n, uint32_t *tot) {
    __shared__ uint32_t sh[2][SCAN_T * PW];
    const uint32_t t = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_CHUNK + (uint64_t)t * SCAN_K;
    Pt acc;
    acc.x = s_zero();
    acc.y = s_zero();
    acc.inf = 1;
    for (int k = 0; k < SCAN_K; k++)
        if (base + k < n) acc = add_complete(acc, load_pt(pts + PW * (base + k)));
    store_pt(sh[0] + PW * t, acc);
    __syncthreads();
    int cur = 0;
    for (int d = 1; d < SCAN_T; d <<= 1) {  // Hillis-Steele over the 256 thread sums
        Pt v = load_pt(sh[cur] + PW * t);
        if (t >= (uint32_t)d) v = add_complete(load_pt(sh[cur] + PW * (t - d)), v);
        store_pt(sh[cur ^ 1] + PW * t, v);
        __syncthreads();
        cur ^= 1;
    }
    Pt run;
    if (t == 0) {
        run.x = s_zero();
        run.y = s_zero();
        run.inf = 1;
    } else {
        run = load_pt(sh[cur] + PW * (t - 1));
    }
    for (int k = 0; k < SCAN_K; k++)
        if (base + k < n) {
            run = add_complete(run, load_pt(pts + PW * (base + k)));
            store_pt(pts + PW * (base + k), run);
        }
    if (t == SCAN_T - 1) store_pt(tot + PW * blockIdx.x, load_pt(sh[cur] + PW * t));
}

// pts[i] <- carry(block) + pts[i], carry = start (level 0 only) + inclusive prefix of the previous blocks
__global__ __launch_bounds__(SCAN_T) void k_scan_apply(uint32_t *pts, uint64_t n, const uint32_t *tot_incl,
                                                       int with_start) {
    __shared__ uint32_t carry[PW];
    const uint64_t b = blockIdx.x;
    if (threadIdx.x == 0) {
        Pt c;
        c.x = s_zero();
        c.y = s_zero();
        c.inf = 1;
        if (with_start) c = const_pt(START);
        if (b > 0) c = add_complete(c, load_pt(tot_incl + PW * (b - 1)));
        store_pt(carry, c);
    }
    __syncthreads();
    const Pt c = load_pt(carry);
    if (c.inf) return;
    for (uint64_t i = b * SCAN_CHUNK + threadIdx.x; i < n && i < (b + 1) * SCAN_CHUNK; i += SCAN_T)
        store_pt(pts + PW * i, add_complete(c, load_pt(pts + PW * i)));
}

// the accumulation half of every row (columns 64..98) and the padding rows
__global__ __launch_bounds__(256) void k_global_fill(uint32_t *__restrict__ trace, const uint32_t *__restrict__ sums,
                                                     uint64_t n, uint64_t height, uint32_t *final_out,
                                                     uint32_t *err) {
    const Pt dummy = const_pt(DUMMY);
    const Pt fin = n ? load_pt(sums + PW * (n - 1)) : dummy;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < height;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t *row = trace + G_WIDTH * i;
        if (i < n) {
            const Pt init = i ? load_pt(sums + PW * (i - 1)) : const_pt(START);
            const Pt cum = load_pt(sums + PW * i);
            if (cum.inf) atomicOr(err, (uint32_t)ERR_INFINITY);
#pragma unroll
            for (int k = 0; k < 7; k++) {
                row[G_INIT_X + k] = from_mont(init.x.c[k]);
                row[G_INIT_X + 7 + k] = from_mont(init.y.c[k]);
                row[G_SUMCHK + k] = 0;
                row[G_CUM_X + k] = from_mont(cum.x.c[k]);
                row[G_CUM_X + 7 + k] = from_mont(cum.y.c[k]);
            }
        } else {
            // populate_dummy: the dummy point, the final digest carried, its sum checker
            // (x1 + x2 + x3)(x2 - x1)^2 - (y2 - y1)^2 with (p1, p2, p3) = (final, dummy, final)
            const S7 dx = s_sub(dummy.x, fin.x), dy = s_sub(dummy.y, fin.y);
            const S7 chk = s_sub(s_mul(s_add(s_add(fin.x, dummy.x), fin.x), s_sq(dx)), s_sq(dy));
            for (int k = 0; k < G_INIT_X; k++) row[k] = 0;
#pragma unroll
            for (int k = 0; k < 7; k++) {
                row[G_X + k] = DUMMY[k];
                row[G_Y + k] = DUMMY[7 + k];
                row[G_INIT_X + k] = from_mont(fin.x.c[k]);
                row[G_INIT_X + 7 + k] = from_mont(fin.y.c[k]);
                row[G_SUMCHK + k] = from_mont(chk.c[k]);
                row[G_CUM_X + k] = from_mont(fin.x.c[k]);
                row[G_CUM_X + 7 + k] = from_mont(fin.y.c[k]);
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && final_out) {
#pragma unroll
        for (int k = 0; k < 7; k++) {
            final_out[k] = from_mont(fin.x.c[k]);
            final_out[7 + k] = from_mont(fin.y.c[k]);
        }
    }
}

}  // namespace zkm::sep

using namespace zkm::sep;

namespace {
#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            g_last_error = std::string("zkm_global_events_to_trace: ") + hipGetErrorString(e_); \
            return ZKM_ERR_HIP;                                                            \
        }                                                                                  \
    } while (0)

// inclusive scan of `n` points at d_pts (PW words each), in place; `with_start` adds the starting digest
int scan_points(uint32_t *d_pts, uint64_t n, int with_start, hipStream_t s) {
    if (n == 0) return ZKM_OK;
    const uint64_t blocks = (n + SCAN_CHUNK - 1) / SCAN_CHUNK;
    uint32_t *d_tot = nullptr;
    HIPCHK(hipMallocAsync((void **)&d_tot, (size_t)blocks * PW * 4, s));
    hipLaunchKernelGGL(k_scan_local, dim3((uint32_t)blocks), dim3(SCAN_T), 0, s, d_pts, n, d_tot);
    HIPCHK(hipGetLastError());
    int rc = ZKM_OK;
    if (blocks > 1) rc = scan_points(d_tot, blocks, 0, s);
    if (rc == ZKM_OK && (blocks > 1 || with_start)) {
        hipLaunchKernelGGL(k_scan_apply, dim3((uint32_t)blocks), dim3(SCAN_T), 0, s, d_pts, n, d_tot, with_start);
        rc = hipGetLastError() == hipSuccess ? ZKM_OK : ZKM_ERR_HIP;
    }
    HIPCHK(hipFreeAsync(d_tot, s));
    return rc;
}
}  // namespace

extern "C" int zkm_global_events_to_trace(const zkm_global_lookup_event *events, uint64_t n, uint32_t *trace,
                                          uint64_t height, uint32_t *byte_mult, uint32_t *final_digest,
                                          void *stream) {
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1))) {
        g_last_error = "zkm_global_events_to_trace: bad arguments (need n <= height, height a power of two >= 16)";
        return ZKM_ERR_ARG;
    }
    hipStream_t s = (hipStream_t)stream;
    uint32_t *d_pts = nullptr, *d_err = nullptr;
    // one exit path: every failure after the first allocation drains the stream (nothing queued may
    // still write into `err` or the buffers) and frees what was allocated
    int rc = ZKM_OK;
    uint32_t err = 0;
    auto fail = [&](hipError_t e) {
        if (e != hipSuccess && rc == ZKM_OK) {
            g_last_error = std::string("zkm_global_events_to_trace: ") + hipGetErrorString(e);
            rc = ZKM_ERR_HIP;
        }
        return rc != ZKM_OK;
    };
    if (!fail(hipMallocAsync((void **)&d_pts, (size_t)(n ? n : 1) * PW * 4, s)) &&
        !fail(hipMallocAsync((void **)&d_err, 4, s)) && !fail(hipMemsetAsync(d_err, 0, 4, s))) {
        hipLaunchKernelGGL(k_septic_init, dim3(1), dim3(64), 0, s);
        if (!fail(hipGetLastError()) && n) {
            const uint64_t want = (n + 255) / 256;
            const uint32_t grid = (uint32_t)(want < 4096 ? want : 4096);
            hipLaunchKernelGGL(k_global_lift, dim3(grid), dim3(256), 0, s, (const uint32_t *)events, n, trace, d_pts,
                               byte_mult, d_err);
            fail(hipGetLastError());
        }
        if (rc == ZKM_OK) rc = scan_points(d_pts, n, 1, s);
        if (rc == ZKM_OK) {
            const uint64_t want = (height + 255) / 256;
            const uint32_t grid = (uint32_t)(want < 4096 ? want : 4096);
            hipLaunchKernelGGL(k_global_fill, dim3(grid), dim3(256), 0, s, trace, d_pts, n, height, final_digest, d_err);
            if (!fail(hipGetLastError())) fail(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, s));
        }
    }
    if (d_pts) fail(hipFreeAsync(d_pts, s));  // stream-ordered: after every queued use
    if (d_err) fail(hipFreeAsync(d_err, s));
    if (fail(hipStreamSynchronize(s))) return rc;  // before `err` is read or leaves scope
    if (rc != ZKM_OK) return rc;
    if (err) {
        g_last_error = std::string("zkm_global_events_to_trace: ") +
                       ((err & ERR_NO_LIFT) ? "a message has no curve point within 256 offsets; " : "") +
                       ((err & ERR_INFINITY) ? "the running global sum reached the point at infinity; " : "") +
                       ((err & ERR_U16) ? "message[0] (the shard) is not a 16-bit value" : "");
        return ZKM_ERR_UNSATISFIED;
    }
    return ZKM_OK;
}
