// Device kernels of MachineProver::open (crates/stark/src/prover.rs:298-653) on gfx950.
//
//  k_perm_rows / scan : generate_permutation_trace (crates/stark/src/permutation.rs:102-196)
//  k_quotient         : quotient_values + Chip::eval (crates/stark/src/quotient.rs:19-171,
//                       chip.rs:259-271, permutation.rs:205-347, folder.rs:79-102)
//  k_inv_points       : batch inverses of (z - s w^i) (barycentric weights, FRI denominators)
//  k_open_dot         : opened values p(z) = (z'^N - 1)/N sum_j y_j w_j  (TwoAdicFriPcs::open)
//  k_fri_reduce       : reduced openings per LDE height (semantics: recursion/circuit/src/fri.rs:97-209)
//  k_fri_fold / leaves: commit phase (fri.rs:247-361 semantics; Plonky3 fold_even_odd)
//  k_pow              : proof-of-work grind (challenger.rs:209-221 check_witness)
//  k_gather           : query openings (rows + Merkle paths)
// All data is column-major Montgomery; EF values are 4 consecutive words.
#include "internal.hpp"
#include "open_kernels.hpp"
#include "p2.cuh"
#include "fri_chal.cuh"

namespace zkm {

using namespace kb;
static constexpr int NT = 256;

__device__ __forceinline__ ef ld_ef(const uint32_t *p) {
    uint4 v = *(const uint4 *)p;
    return ef{{v.x, v.y, v.z, v.w}};
}
__device__ __forceinline__ void st_ef(uint32_t *p, const ef &e) { *(uint4 *)p = make_uint4(e.c[0], e.c[1], e.c[2], e.c[3]); }

// w_M^j for j in [0, M): tw[M/2 + j] for j < M/2, negated above.
__device__ __forceinline__ uint32_t root_pow(const uint32_t *__restrict__ tw, uint64_t M, uint64_t j) {
    if (M == 1) return ONE;
    const uint64_t h = M >> 1;
    return j < h ? tw[h + j] : neg(tw[h + (j - h)]);
}

// value of a VirtualPairCol at one row; advances vp past it
__device__ __forceinline__ uint32_t apply_vpc(const uint32_t *__restrict__ &vp, const uint32_t *__restrict__ main,
                                              const uint32_t *__restrict__ prep, uint64_t ldm, uint64_t row) {
    uint32_t nt = vp[0];
    uint32_t acc = 0;
    for (uint32_t i = 0; i < nt; i++) {
        uint32_t col = vp[1 + 2 * i], w = vp[2 + 2 * i];
        uint32_t v = (col & 0x80000000u) ? main[(uint64_t)(col & 0x7fffffffu) * ldm + row] : prep[(uint64_t)col * ldm + row];
        acc = add(acc, mul(v, w));
    }
    acc = add(acc, vp[1 + 2 * nt]);
    vp += 2 + 2 * nt;
    return acc;
}

// ------------------------------------------------------------------ permutation trace
__global__ __launch_bounds__(NT) void k_perm_rows(PermArgs a) {
    const uint64_t r = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (r >= a.n) return;
    const uint32_t *prog = a.prog;
    const uint32_t nloc = prog[2];
    const uint32_t *table = prog + prog[3];
    ef total = ef_zero();
    for (int b = 0; b < a.nb; b++) {
        ef num = ef_zero(), den = ef_one();
        for (uint32_t i = b * a.batch; i < nloc && i < (uint32_t)(b + 1) * a.batch; i++) {
            const uint32_t *lk = table + 4 * i;
            ef d = ef_add_base(a.alpha, lk[0]);
            const uint32_t *vp = prog + lk[3];
            for (uint32_t v = 0; v < lk[2]; v++) {
                uint32_t x = apply_vpc(vp, a.main, a.prep, a.n, r);
                d = ef_add(d, ef_mul_base(ld_ef(a.beta_pows + 4 * v), x));
            }
            uint32_t m = apply_vpc(vp, a.main, a.prep, a.n, r);
            if (!lk[1]) m = neg(m);
            // num/den += m/d
            num = ef_add(ef_mul(num, d), ef_mul_base(den, m));
            den = ef_mul(den, d);
        }
        ef s = ef_mul(num, ef_inv(den));
#pragma unroll
        for (int e = 0; e < 4; e++) a.out[(uint64_t)(4 * b + e) * a.n + r] = s.c[e];
        total = ef_add(total, s);
    }
    st_ef(a.rowsum + 4 * r, total);
}

// inclusive scan of EF values: block scan (1024 per block) + block totals + fix-up
__device__ __forceinline__ ef warp_scan_incl(ef v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        ef t;
#pragma unroll
        for (int e = 0; e < 4; e++) t.c[e] = __shfl_up(v.c[e], o, 64);
        if (lane >= o) v = ef_add(v, t);
    }
    return v;
}

// scans 4 consecutive elements per thread; writes inclusive scan to out_cols (4 columns, stride n)
// (or back into `data` when out_cols == nullptr) and the block total to totals[blockIdx]
__global__ __launch_bounds__(NT) void k_scan_block(uint32_t *data, uint64_t n, uint32_t *totals) {
    __shared__ uint32_t wsum[NT / 64][4];
    const uint64_t base = (uint64_t)blockIdx.x * NT * 4 + threadIdx.x * 4;
    ef v[4];
    ef run = ef_zero();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        v[k] = (base + k < n) ? ld_ef(data + 4 * (base + k)) : ef_zero();
        run = ef_add(run, v[k]);
        v[k] = run;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    ef incl = warp_scan_incl(run, lane);
    if (lane == 63)
        for (int e = 0; e < 4; e++) wsum[wid][e] = incl.c[e];
    __syncthreads();
    ef off = ef_sub(incl, run);  // exclusive within wave
    for (int w = 0; w < wid; w++) off = ef_add(off, ef{{wsum[w][0], wsum[w][1], wsum[w][2], wsum[w][3]}});
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (base + k < n) st_ef(data + 4 * (base + k), ef_add(v[k], off));
    if (threadIdx.x == NT - 1) st_ef(totals + 4 * blockIdx.x, ef_add(off, run));
}

// exclusive scan of the block totals by one workgroup: contiguous chunk per thread + LDS scan
__global__ __launch_bounds__(NT) void k_scan_totals(uint32_t *totals, uint64_t nblocks) {
    __shared__ uint32_t sums[NT][4];
    const uint64_t per = (nblocks + NT - 1) / NT;
    const uint64_t b0 = threadIdx.x * per, b1 = b0 + per < nblocks ? b0 + per : nblocks;
    ef run = ef_zero();
    for (uint64_t i = b0; i < b1; i++) run = ef_add(run, ld_ef(totals + 4 * i));
    for (int e = 0; e < 4; e++) sums[threadIdx.x][e] = run.c[e];
    __syncthreads();
    if (threadIdx.x == 0) {
        ef acc = ef_zero();
        for (int t = 0; t < NT; t++) {
            ef v{{sums[t][0], sums[t][1], sums[t][2], sums[t][3]}};
            for (int e = 0; e < 4; e++) sums[t][e] = acc.c[e];
            acc = ef_add(acc, v);
        }
    }
    __syncthreads();
    ef off{{sums[threadIdx.x][0], sums[threadIdx.x][1], sums[threadIdx.x][2], sums[threadIdx.x][3]}};
    for (uint64_t i = b0; i < b1; i++) {
        ef t = ld_ef(totals + 4 * i);
        st_ef(totals + 4 * i, off);
        off = ef_add(off, t);
    }
}

__global__ __launch_bounds__(NT) void k_scan_fix(const uint32_t *data, uint64_t n, const uint32_t *totals,
                                                 uint32_t *out_cols) {
    const uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    ef v = ef_add(ld_ef(data + 4 * i), ld_ef(totals + 4 * (i / (NT * 4))));
#pragma unroll
    for (int e = 0; e < 4; e++) out_cols[(uint64_t)e * n + i] = v.c[e];
}

void launch_perm_trace(const PermArgs &a, hipStream_t s, bool rows_done) {
    if (a.nb < 0) return;
    if (!rows_done) {
        hipLaunchKernelGGL(k_perm_rows, dim3((unsigned)((a.n + NT - 1) / NT)), dim3(NT), 0, s, a);
        HIP_CHECK(hipGetLastError());
    }
    const uint64_t nblk = (a.n + NT * 4 - 1) / (NT * 4);
    DBuf totals(4 * nblk, s);
    hipLaunchKernelGGL(k_scan_block, dim3((unsigned)nblk), dim3(NT), 0, s, a.rowsum, a.n, totals.p);
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_scan_totals, dim3(1), dim3(NT), 0, s, totals.p, nblk);
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_scan_fix, dim3((unsigned)((a.n + NT - 1) / NT)), dim3(NT), 0, s, a.rowsum, a.n, totals.p,
                       a.out + (uint64_t)4 * a.nb * a.n);
    HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------ quotient
static constexpr int QSTACK = 24;

__global__ __launch_bounds__(NT) void k_quotient(QuotArgs a) {
    extern __shared__ uint32_t lds_stack[];  // [wave][depth][64]
    const uint64_t tw_ = (uint64_t)blockIdx.x * NT + threadIdx.x;  // row within the window
    const uint64_t t = a.t0 + tw_;
    const int lane = threadIdx.x & 63;
    uint32_t *stk = lds_stack + (threadIdx.x >> 6) * QSTACK * 64 + lane;
    if (tw_ >= a.slot_rows || t >= a.q) return;  // q is a multiple of 64 (>= 16 rows * 2 ... checked on host)
    uint32_t *slots = a.slots + tw_;
    const uint64_t ldm = a.ld;  // LDE height (column stride)
    const uint64_t rl = t;
    const uint64_t k = rev_bits((uint32_t)t, a.log_q);
    const uint64_t kn = (k + a.step) & (a.q - 1);
    const uint64_t rn = rev_bits((uint32_t)kn, a.log_q);
    // selectors at x = 3 w_Q^k over trace domain H_N (quotient.rs:42; Plonky3 selectors_on_coset)
    const uint32_t x = mul(a.gen, root_pow(a.tw, a.q, k));
    // Z_H(x) = x^n - 1 = 3^n w_{Q/n}^(k mod Q/n) - 1 (Q/n = 2^log_qd: 1, 2 or 4 values)
    const uint64_t qn = a.q / a.n;
    uint32_t zp = ONE;
    if (qn > 1) {
        const uint64_t zm = k & (qn - 1), zhh = qn >> 1;
        zp = zm < zhh ? a.tw[zhh + zm] : neg(a.tw[zhh + (zm - zhh)]);
    }
    const uint32_t zh = sub(mul(a.gen_pow_n, zp), ONE);
    const uint32_t d_first = sub(x, ONE), d_last = sub(x, a.wn_inv);
    const uint32_t inv_fl = inv(mul(mul(d_first, d_last), zh));  // one inversion for three
    const uint32_t is_first = mul(mul(inv_fl, d_last), mul(zh, zh));
    const uint32_t is_last = mul(mul(inv_fl, d_first), mul(zh, zh));
    const uint32_t is_trans = d_last;
    const uint32_t inv_z = mul(inv_fl, mul(d_first, d_last));

    const uint32_t *main = a.main, *prep = a.prep, *perm = a.perm;
    const uint32_t *prog = a.prog;
    const uint32_t *code = prog + prog[1];
    const uint32_t code_len = prog[0];
    ef acc = ef_zero();
    uint32_t k_c = 0;  // constraint index
    // ---- AIR program (postfix; stack top in a register, the rest in LDS) ----
    int sp = 0;
    uint32_t top = 0;
    bool has = false;
#define PUSH(v)                                   \
    do {                                          \
        if (has) { stk[sp * 64] = top; sp++; }    \
        top = (v);                                \
        has = true;                               \
    } while (0)
    for (uint32_t pc = 0; pc < code_len;) {
        const uint32_t op = code[pc++];
        switch (op) {
        case 1: { uint32_t c = code[pc++]; PUSH(main[(uint64_t)c * ldm + rl]); break; }
        case 2: { uint32_t c = code[pc++]; PUSH(main[(uint64_t)c * ldm + rn]); break; }
        case 3: { uint32_t c = code[pc++]; PUSH(prep[(uint64_t)c * ldm + rl]); break; }
        case 4: { uint32_t c = code[pc++]; PUSH(prep[(uint64_t)c * ldm + rn]); break; }
        case 5: { uint32_t v = code[pc++]; PUSH(v); break; }
        case 6: { uint32_t i = code[pc++]; PUSH(a.pv[i]); break; }
        case 7: PUSH(is_first); break;
        case 8: PUSH(is_last); break;
        case 9: PUSH(is_trans); break;
        case 10: { sp--; top = add(stk[sp * 64], top); break; }
        case 11: { sp--; top = sub(stk[sp * 64], top); break; }
        case 12: { sp--; top = mul(stk[sp * 64], top); break; }
        case 13: top = neg(top); break;
        case 14: {
            acc = ef_add(acc, ef_mul_base(ld_ef(a.pows + 4 * k_c), top));
            k_c++;
            if (sp) { sp--; top = stk[sp * 64]; } else has = false;
            break;
        }
        case 15: {  // LET s: pop into slot s
            slots[(uint64_t)code[pc++] * a.slot_rows] = top;
            if (sp) { sp--; top = stk[sp * 64]; } else has = false;
            break;
        }
        case 16: { uint32_t sl = code[pc++]; PUSH(slots[(uint64_t)sl * a.slot_rows]); break; }
        default: break;
        }
    }
#undef PUSH
    // ---- LogUp constraints (permutation.rs:256-333) ----
    const uint32_t nloc = prog[2];
    if (nloc) {
        const uint32_t *table = prog + prog[3];
        const int nb = a.perm_w - 1;
        ef sum_l = ef_zero(), sum_n = ef_zero();
        for (int b = 0; b < nb; b++) {
            ef prod = ef_one(), num = ef_zero();
            for (uint32_t i = b * a.batch; i < nloc && i < (uint32_t)(b + 1) * a.batch; i++) {
                const uint32_t *lk = table + 4 * i;
                ef rlc = ef_add_base(a.alpha_p, lk[0]);
                const uint32_t *vp = prog + lk[3];
                for (uint32_t v = 0; v < lk[2]; v++) {
                    uint32_t xv = apply_vpc(vp, main, prep, ldm, rl);
                    rlc = ef_add(rlc, ef_mul_base(ld_ef(a.beta_pows + 4 * v), xv));
                }
                uint32_t m = apply_vpc(vp, main, prep, ldm, rl);
                if (!lk[1]) m = neg(m);
                // numerator = sum_i m_i prod_{j != i} rlc_j, built incrementally
                num = ef_add(ef_mul(num, rlc), ef_mul_base(prod, m));
                prod = ef_mul(prod, rlc);
            }
            ef entry, entry_n;
            for (int e = 0; e < 4; e++) {
                entry.c[e] = perm[(uint64_t)(4 * b + e) * ldm + rl];
                entry_n.c[e] = perm[(uint64_t)(4 * b + e) * ldm + rn];
            }
            sum_l = ef_add(sum_l, entry);
            sum_n = ef_add(sum_n, entry_n);
            ef c = ef_sub(ef_mul(prod, entry), num);
            acc = ef_add(acc, ef_mul(ld_ef(a.pows + 4 * k_c), c));
            k_c++;
        }
        ef phi_l, phi_n;
        for (int e = 0; e < 4; e++) {
            phi_l.c[e] = perm[(uint64_t)(4 * nb + e) * ldm + rl];
            phi_n.c[e] = perm[(uint64_t)(4 * nb + e) * ldm + rn];
        }
        ef c0 = ef_mul_base(ef_sub(phi_l, sum_l), is_first);
        acc = ef_add(acc, ef_mul(ld_ef(a.pows + 4 * k_c), c0)); k_c++;
        ef c1 = ef_mul_base(ef_sub(ef_sub(phi_n, phi_l), sum_n), is_trans);
        acc = ef_add(acc, ef_mul(ld_ef(a.pows + 4 * k_c), c1)); k_c++;
        ef c2 = ef_mul_base(ef_sub(phi_l, a.lcs), is_last);
        acc = ef_add(acc, ef_mul(ld_ef(a.pows + 4 * k_c), c2)); k_c++;
    }
    if (a.global) {
        const uint32_t W = a.main_w;
        for (int i = 0; i < 7; i++) {
            uint32_t cx = mul(sub(main[(uint64_t)(W - 14 + i) * ldm + rl], a.gcs[i]), is_last);
            acc = ef_add(acc, ef_mul_base(ld_ef(a.pows + 4 * k_c), cx)); k_c++;
            uint32_t cy = mul(sub(main[(uint64_t)(W - 7 + i) * ldm + rl], a.gcs[7 + i]), is_last);
            acc = ef_add(acc, ef_mul_base(ld_ef(a.pows + 4 * k_c), cy)); k_c++;
        }
    }
    const ef q = ef_mul_base(acc, inv_z);
    // chunk c = k mod 2^lqd (t = rev_Q(k) = rev_lqd(c) n + rev_n(k >> lqd)), stored bit-reversed within
    // the chunk
    const uint64_t c = k & (uint64_t)(a.step - 1);
    const uint64_t pos = t & (a.n - 1);
#pragma unroll
    for (int e = 0; e < 4; e++) a.chunks[c * a.cstride + e * a.n + pos] = q.c[e];
}

void launch_quotient(const QuotArgs &a0, hipStream_t s) {
    const size_t lds = (size_t)(NT / 64) * QSTACK * 64 * 4;
    QuotArgs a = a0;
    if (!a.n_slots) {  // no shared subexpressions: one launch over every row
        a.slot_rows = a.q;
        a.t0 = 0;
        hipLaunchKernelGGL(k_quotient, dim3((unsigned)((a.q + NT - 1) / NT)), dim3(NT), lds, s, a);
        HIP_CHECK(hipGetLastError());
        return;
    }
    // value slots in global scratch (this interpreter is the ZKM_NO_JIT path; the JIT keeps slots in
    // registers): windows of rows so the scratch stays within ~1 GiB
    uint64_t rows = std::min<uint64_t>(a.q, std::max<uint64_t>(NT, (1ull << 28) / (uint64_t)a.n_slots));
    rows = (rows + NT - 1) / NT * NT;
    DBuf scratch((size_t)a.n_slots * rows, s);
    a.slots = scratch.p;
    a.slot_rows = rows;
    for (uint64_t t0 = 0; t0 < a.q; t0 += rows) {
        a.t0 = t0;
        const uint64_t cnt = std::min<uint64_t>(rows, a.q - t0);
        hipLaunchKernelGGL(k_quotient, dim3((unsigned)((cnt + NT - 1) / NT)), dim3(NT), lds, s, a);
        HIP_CHECK(hipGetLastError());
    }
}

// ------------------------------------------------------------------ batch inverses at points
// out[i] = (mul_omega ? w^idx : 1) / (z - s * w_M^idx), idx = bitrev ? rev(i) : i
static constexpr int INV_CHUNK = 8;  // prefix products stay in registers

// out[i] = (optionally w^idx *) 1 / (z - s w_M^idx), idx = i or rev(i): Montgomery's trick over
// INV_CHUNK consecutive i per thread, one extension-field inversion per chunk
__global__ __launch_bounds__(NT) void k_inv_points(ef z, uint32_t s, const uint32_t *__restrict__ tw, uint64_t M,
                                                   int log_m, int bitrev, int mul_omega, uint32_t *out) {
    const uint64_t c = (uint64_t)blockIdx.x * NT + threadIdx.x;
    const uint64_t i0 = c * INV_CHUNK;
    if (i0 >= M) return;  // M is a power of two >= INV_CHUNK or a single partial chunk
    const int cnt = (int)(M - i0 < (uint64_t)INV_CHUNK ? M - i0 : INV_CHUNK);
    uint32_t om[INV_CHUNK];
    ef d[INV_CHUNK], pre[INV_CHUNK];
#pragma unroll
    for (int k = 0; k < INV_CHUNK; k++) {
        if (k < cnt) {
            const uint64_t i = i0 + k;
            om[k] = root_pow(tw, M, bitrev ? rev_bits((uint32_t)i, log_m) : i);
        } else {
            om[k] = ONE;
        }
    }
    ef run = ef_one();
#pragma unroll
    for (int k = 0; k < INV_CHUNK; k++) {
        d[k] = k < cnt ? ef_sub(z, ef_base(mul(s, om[k]))) : ef_one();
        pre[k] = run;
        run = ef_mul(run, d[k]);
    }
    ef iv = ef_inv(run);
#pragma unroll
    for (int k = INV_CHUNK - 1; k >= 0; k--) {
        const ef v = ef_mul(iv, pre[k]);
        iv = ef_mul(iv, d[k]);
        if (k < cnt) st_ef(out + 4 * (i0 + k), mul_omega ? ef_mul_base(v, om[k]) : v);
    }
}

void launch_inv_points(const ef &z, uint32_t s, const uint32_t *tw, uint64_t M, bool bitrev, bool mul_omega,
                       uint32_t *out, hipStream_t st) {
    const uint64_t chunks = (M + INV_CHUNK - 1) / INV_CHUNK;
    hipLaunchKernelGGL(k_inv_points, dim3((unsigned)((chunks + NT - 1) / NT)), dim3(NT), 0, st, z, s, tw, M,
                       ilog2(M), (int)bitrev, (int)mul_omega, out);
    HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------ opening dot products
// out[col * 8 + 4p .. +4] = sum_j y_{j + p} w_j / R  (p = 1 only if with_next)
// A workgroup takes OPEN_SEG consecutive rows and computes their weights w_j = (w^idx) / (z - s w_n^idx)
// into LDS itself (Montgomery's trick over INV_CHUNK rows per thread, one EF inversion per chunk), so no
// weight table is written to or read from HBM; then it walks its slab of columns OPEN_CB at a time over
// those rows.  Each thread takes rows in
// pairs (j, j + NT): per EF component the two products go into one v_mad_u64_u32 chain and one lazy
// Montgomery reduction, accumulated unreduced in 64 bits.  Per (column, segment) partial sums are
// reduced over the segments by k_open_sum.
static constexpr int OPEN_CB = 4;
static constexpr int OPEN_SEG = 2048;  // rows per workgroup: 32 KB of weights in LDS
__device__ __forceinline__ uint64_t pair_acc(uint64_t acc, uint32_t ya, uint32_t wa, uint32_t yb, uint32_t wb) {
    // ya wa + yb wb < 2P^2 < P 2^32 -> [0, 2P)
    return add_w(acc, redc2(mad64(ya, wa, prod64(yb, wb))));
}

static_assert(OPEN_SEG == NT * INV_CHUNK, "one weight chunk per thread");

// rows [j0 + r0, j0 + r0 + cnt) of the weight table of launch_inv_points, into LDS
__device__ __forceinline__ void open_weights(uint4 *wl, const OpenWeights &pw, uint64_t n, uint64_t j0, uint32_t r0,
                                             int cnt) {
    uint32_t om[INV_CHUNK];
    ef d[INV_CHUNK], pre[INV_CHUNK];
#pragma unroll
    for (int k = 0; k < INV_CHUNK; k++) {
        const uint64_t i = j0 + r0 + k;
        om[k] = k < cnt ? root_pow(pw.tw, n, pw.bitrev ? rev_bits((uint32_t)i, pw.log_n) : i) : ONE;
    }
    ef run = ef_one();
#pragma unroll
    for (int k = 0; k < INV_CHUNK; k++) {
        d[k] = k < cnt ? ef_sub(pw.z, ef_base(mul(pw.s, om[k]))) : ef_one();
        pre[k] = run;
        run = ef_mul(run, d[k]);
    }
    ef iv = ef_inv(run);
#pragma unroll
    for (int k = INV_CHUNK - 1; k >= 0; k--) {
        ef v = ef_mul(iv, pre[k]);
        iv = ef_mul(iv, d[k]);
        if (pw.mul_omega) v = ef_mul_base(v, om[k]);
        if (k < cnt) wl[r0 + k] = make_uint4(v.c[0], v.c[1], v.c[2], v.c[3]);
    }
}

__device__ __forceinline__ void open_dot_lds(const uint64_t *__restrict__ cols, uint32_t ncols, uint64_t n,
                                                 OpenWeights pw, int with_next, int nseg, uint32_t slab,
                                                 uint32_t *partial, uint32_t bx, uint32_t by) {
    __shared__ uint4 wl[OPEN_SEG];
    __shared__ uint32_t red[NT / 64][OPEN_CB][8];
    const uint64_t j0 = (uint64_t)bx * OPEN_SEG;
    const uint32_t len = (uint32_t)(n - j0 < (uint64_t)OPEN_SEG ? n - j0 : OPEN_SEG);
    {
        const uint32_t r0 = threadIdx.x * INV_CHUNK;
        if (r0 < len) open_weights(wl, pw, n, j0, r0, (int)(len - r0 < (uint32_t)INV_CHUNK ? len - r0 : INV_CHUNK));
    }
    __syncthreads();
    const uint32_t c_begin = by * slab;
    const uint32_t c_end = c_begin + slab < ncols ? c_begin + slab : ncols;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint32_t cb0 = c_begin; cb0 < c_end; cb0 += OPEN_CB) {
        const int nc = (int)(c_end - cb0 < (uint32_t)OPEN_CB ? c_end - cb0 : OPEN_CB);
        const uint32_t *y[OPEN_CB];
#pragma unroll
        for (int k = 0; k < OPEN_CB; k++) y[k] = (const uint32_t *)cols[cb0 + (k < nc ? k : 0)] + j0;
        uint64_t a0[OPEN_CB][4], a1[OPEN_CB][4];
#pragma unroll
        for (int k = 0; k < OPEN_CB; k++)
#pragma unroll
            for (int e = 0; e < 4; e++) { a0[k][e] = 0; a1[k][e] = 0; }
        for (uint32_t ra = threadIdx.x; ra < len; ra += 2 * NT) {
            const uint32_t rb0 = ra + NT;
            const bool hb = rb0 < len;
            const uint32_t rb = hb ? rb0 : ra;  // a missing second row pairs with weight 0
            const uint4 wa = wl[ra];
            uint4 wb = wl[rb];
            if (!hb) wb = make_uint4(0, 0, 0, 0);
            const uint32_t wav[4] = {wa.x, wa.y, wa.z, wa.w}, wbv[4] = {wb.x, wb.y, wb.z, wb.w};
            uint32_t va[OPEN_CB], vb[OPEN_CB], na[OPEN_CB], nb[OPEN_CB];
#pragma unroll
            for (int k = 0; k < OPEN_CB; k++) {
                va[k] = y[k][ra];
                vb[k] = y[k][rb];
                if (with_next) {  // the next row wraps to row 0 at the end of the column
                    const uint32_t *yk = y[k] - j0;
                    na[k] = yk[(j0 + ra + 1) & (n - 1)];
                    nb[k] = yk[(j0 + rb + 1) & (n - 1)];
                }
            }
#pragma unroll
            for (int k = 0; k < OPEN_CB; k++)
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    a0[k][e] = pair_acc(a0[k][e], va[k], wav[e], vb[k], wbv[e]);
                    if (with_next) a1[k][e] = pair_acc(a1[k][e], na[k], wav[e], nb[k], wbv[e]);
                }
        }
#pragma unroll
        for (int k = 0; k < OPEN_CB; k++) {
            uint32_t r0[4], r1[4];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                r0[e] = acc_mod(a0[k][e]);
                r1[e] = with_next ? acc_mod(a1[k][e]) : 0u;
            }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    r0[e] = add(r0[e], __shfl_xor(r0[e], o, 64));
                    r1[e] = add(r1[e], __shfl_xor(r1[e], o, 64));
                }
            if (lane == 0)
                for (int e = 0; e < 4; e++) { red[wid][k][e] = r0[e]; red[wid][k][4 + e] = r1[e]; }
        }
        __syncthreads();
        if (threadIdx.x < (unsigned)nc * 8) {
            const int k = threadIdx.x >> 3, e = threadIdx.x & 7;
            uint32_t acc = 0;
            for (int q = 0; q < NT / 64; q++) acc = add(acc, red[q][k][e]);
            partial[((uint64_t)(cb0 + k) * nseg + bx) * 8 + e] = acc;
        }
        __syncthreads();  // red is reused by the next column block
    }
}
// Full segments (n a multiple of OPEN_SEG): thread t owns rows 4t..4t+3 and 4(NT + t)..+3 of its segment
// for every column, so it computes those eight weights once (Montgomery's trick over the eight, one EF
// inversion) and keeps them in registers: no LDS weight table, two 16-byte loads per column and thread
// (each a whole 1 KB range per wave), the next row of the last element by a shuffle from the neighbouring
// lane (the wave's last lane loads it).  The per-thread sums of a column block are reduced through LDS
// (eight threads per output word, 32 partial sums each) instead of a 6-step shuffle tree per word.
static constexpr int OPEN_RED_LD = NT + 8;  // padded row: the eight outputs a wave sums sit on distinct banks


// 32-bit representative of a lazy dot-product sum v < 2^34 (four pair_acc terms, each < 2P): v mod 2^31 plus
// (v >> 31)(2^24 - 1), since 2^31 = 2^24 - 1 mod p; < 2^31 + 2^27.  Congruent, not canonical: three VALU
// operations instead of acc_mod's reduction and product, the block sum is reduced once
__device__ __forceinline__ uint32_t fold_acc(uint64_t v) {
    const uint32_t hi = (uint32_t)(v >> 31), lo = (uint32_t)v & 0x7fffffffu;
    return lo + (hi << 24) - hi;
}

// The full-segment kernel (round 4's register-weight form, above) with the next column block's loads issued
// before the current block's products (two register sets used alternately), two columns per block: 116 VGPRs,
// 4 waves per SIMD (0.600-0.606 vs 0.608-0.614 ms per shard with four columns, profiles/r05_open_cb_ab.txt; the
// round-4 kernel without the prefetch and the LDS-weight form for full segments lost their A/Bs and are gone)
template <int CB>
__device__ __forceinline__ void open_dot_pf(const uint64_t *__restrict__ cols, uint32_t ncols, uint64_t n,
                                                      OpenWeights pw, int with_next, int nseg, uint32_t slab,
                                                      uint32_t *partial, uint32_t bx, uint32_t by) {
    __shared__ uint32_t red[CB * 8][OPEN_RED_LD];
    constexpr int TPW = NT / (CB * 8);  // reduction threads per output word
    const uint64_t j0 = (uint64_t)bx * OPEN_SEG;
    const uint32_t t = threadIdx.x, lane = t & 63;
    const uint32_t ra = 4 * t, rb = 4 * NT + 4 * t;
    ef w[8];
    {
        // w_n^idx of the two quads: natural order, one aligned 16-byte twiddle load per quad; bit-reversed,
        // idx(i0 + {0, 1, 2, 3}) = rev(i0) + {0, n/2, n/4, 3n/4}: one twiddle, its negation, one product
        // with w_n^(n/4) and that one's negation
        uint32_t om[8];
        const uint64_t h = n >> 1;
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const uint64_t i0 = j0 + (q ? rb : ra);
            uint32_t *o = om + 4 * q;
            if (pw.bitrev) {
                o[0] = root_pow(pw.tw, n, rev_bits((uint32_t)i0, pw.log_n));
                o[1] = neg(o[0]);
                o[2] = mul(o[0], pw.tw[h + (n >> 2)]);
                o[3] = neg(o[2]);
            } else {
                const bool hi = i0 >= h;
                const uint4 v = *(const uint4 *)(pw.tw + h + (hi ? i0 - h : i0));
                o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
                if (hi)
#pragma unroll
                    for (int k = 0; k < 4; k++) o[k] = neg(o[k]);
            }
        }
        ef d[8];
        ef run = ef_one();
#pragma unroll
        for (int k = 0; k < 8; k++) {
            d[k] = ef_sub(pw.z, ef_base(mul(pw.s, om[k])));
            w[k] = run;
            run = ef_mul(run, d[k]);
        }
        ef iv = ef_inv(run);
#pragma unroll
        for (int k = 7; k >= 0; k--) {
            ef v = ef_mul(iv, w[k]);
            iv = ef_mul(iv, d[k]);
            w[k] = pw.mul_omega ? ef_mul_base(v, om[k]) : v;
        }
    }
    const uint32_t c_begin = by * slab;
    const uint32_t c_end = c_begin + slab < ncols ? c_begin + slab : ncols;
    // the next column block's rows are loaded before this block's products (software pipelining: the
    // loads of block b + 1 are in flight while block b is multiplied and reduced; two register sets used
    // alternately, so no copy forces an early wait).  Global (not flat) loads: flat ones also count on
    // lgkmcnt, and the LDS reduction's waits would drain the prefetched block.  The wave's last lane also
    // loads the row after each of its two quads (the next-row products; the wrap-around) in the same batch.
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(1))) u32x4 *g4;
    typedef const __attribute__((address_space(1))) uint32_t *g1;
    struct Blk {
        uint4 a[CB], b[CB];
        uint32_t xa[CB], xb[CB];
    };
    auto load_block = [&](uint32_t cb, Blk &d) {
        const int nc = (int)(c_end - cb < (uint32_t)CB ? c_end - cb : CB);
#pragma unroll
        for (int k = 0; k < CB; k++) {
            const uint64_t y = cols[cb + (k < nc ? k : 0)];
            const u32x4 qa = *(g4)(y + 4 * (j0 + ra)), qb = *(g4)(y + 4 * (j0 + rb));
            d.a[k] = make_uint4(qa.x, qa.y, qa.z, qa.w);
            d.b[k] = make_uint4(qb.x, qb.y, qb.z, qb.w);
            // every lane, unconditionally: a predicated load would leave the wait counts path-dependent
            // (the compiler then waits for the prefetch too); the neighbours' copies hit the cache
            d.xa[k] = *(g1)(y + 4 * ((j0 + ra + 4) & (n - 1)));
            d.xb[k] = *(g1)(y + 4 * ((j0 + rb + 4) & (n - 1)));
        }
    };
    auto process = [&](uint32_t cb0, const Blk &c) {
        const int nc = (int)(c_end - cb0 < (uint32_t)CB ? c_end - cb0 : CB);
#pragma unroll
        for (int k = 0; k < CB; k++) {
            const uint4 va = c.a[k], vb = c.b[k];
            const uint32_t v[8] = {va.x, va.y, va.z, va.w, vb.x, vb.y, vb.z, vb.w};
            uint64_t a0[4] = {0, 0, 0, 0}, a1[4] = {0, 0, 0, 0};
#pragma unroll
            for (int e = 0; e < 4; e++)
#pragma unroll
                for (int m = 0; m < 4; m++) a0[e] = pair_acc(a0[e], v[m], w[m].c[e], v[m + 4], w[m + 4].c[e]);
            if (with_next) {  // the next row wraps to row 0 at the end of the column
                const uint32_t u[8] = {va.y, va.z, va.w, c.xa[k], vb.y, vb.z, vb.w, c.xb[k]};
#pragma unroll
                for (int e = 0; e < 4; e++)
#pragma unroll
                    for (int m = 0; m < 4; m++) a1[e] = pair_acc(a1[e], u[m], w[m].c[e], u[m + 4], w[m + 4].c[e]);
            }
#pragma unroll
            for (int e = 0; e < 4; e++) {
                // a 32-bit representative, not the canonical value: the sum over the block is reduced once
                red[k * 8 + e][t] = fold_acc(a0[e]);
                red[k * 8 + 4 + e][t] = with_next ? fold_acc(a1[e]) : 0u;
            }
        }
        __syncthreads();
        {
            const uint32_t o = t / TPW, q = t % TPW;  // output word o (column o / 8), partial sums q, q + TPW, ...
            uint64_t acc = 0;
#pragma unroll
            for (int i = 0; i < NT / TPW; i++) acc += red[o][q + TPW * i];  // < 32 * 2^32
            uint32_t r = acc_mod(acc);
#pragma unroll
            for (int sh = 1; sh < TPW; sh <<= 1) r = add(r, __shfl_xor(r, sh, 64));
            if (q == 0 && (int)(o >> 3) < nc) partial[((uint64_t)(cb0 + (o >> 3)) * nseg + bx) * 8 + (o & 7)] = r;
        }
        __syncthreads();  // red is reused by the next column block
    };
    Blk b0, b1;
    if (c_begin < c_end) load_block(c_begin, b0);
    for (uint32_t cb0 = c_begin; cb0 < c_end; cb0 += 2 * CB) {
        const uint32_t cb1 = cb0 + CB;
        if (cb1 < c_end) load_block(cb1, b1);
        process(cb0, b0);
        if (cb1 >= c_end) break;
        if (cb1 + CB < c_end) load_block(cb1 + CB, b0);
        process(cb1, b1);
    }
}
// out[col * 8 + e] = sum over the nseg segments of partial[(col * nseg + seg) * 8 + e]: one wave per
// (column, e) pair group, lanes striding over the segments
__device__ __forceinline__ void open_sum(const uint32_t *__restrict__ partial, int nseg, uint32_t *out, uint32_t col) {
    const int lane = threadIdx.x;
    uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // < nseg P < 2^44
    for (int sg = lane; sg < nseg; sg += 64) {
        const uint4 *x = (const uint4 *)(partial + ((uint64_t)col * nseg + sg) * 8);
        const uint4 lo = x[0], hi = x[1];
        acc[0] += lo.x; acc[1] += lo.y; acc[2] += lo.z; acc[3] += lo.w;
        acc[4] += hi.x; acc[5] += hi.y; acc[6] += hi.z; acc[7] += hi.w;
    }
    uint32_t r[8];
#pragma unroll
    for (int e = 0; e < 8; e++) {
        r[e] = (uint32_t)(acc[e] % P);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) r[e] = add(r[e], __shfl_xor(r[e], o, 64));
    }
    if (lane < 8) out[(uint64_t)col * 8 + lane] = r[lane];
}
// Every group of an opening in one grid per kernel kind (blockIdx.z = group; a group's workgroups beyond its
// own segments / slabs, or of another kind, return at once): one launch instead of one per (height,
// domain, points) group, so the small groups (short chips, quotient chunks) run beside each other
template <int KIND>
__global__ __launch_bounds__(NT) void k_open_dot_groups(const OpenGroup *__restrict__ gs) {
    const OpenGroup g = gs[blockIdx.z];
    if (g.kind != KIND || blockIdx.x >= (uint32_t)g.nseg || blockIdx.y >= g.nslab) return;
    if constexpr (KIND == 0)  // a partial last segment: the LDS weight table
        open_dot_lds(g.cols, g.ncols, g.n, g.w, g.with_next, g.nseg, g.slab, g.partial, blockIdx.x, blockIdx.y);
    else
        open_dot_pf<2>(g.cols, g.ncols, g.n, g.w, g.with_next, g.nseg, g.slab, g.partial, blockIdx.x, blockIdx.y);
}
__global__ __launch_bounds__(64) void k_open_sum_groups(const OpenGroup *__restrict__ gs) {
    const OpenGroup g = gs[blockIdx.z];
    if (blockIdx.x >= g.ncols) return;
    open_sum(g.partial, g.nseg, g.out, blockIdx.x);
}

// grid shape and kernel kind of one group: row segments of OPEN_SEG, and for small matrices the columns split
// into slabs too, so a launch still has ~1024+ workgroups
static void open_group_shape(OpenGroup &g) {
    g.nseg = (int)((g.n + OPEN_SEG - 1) / OPEN_SEG);
    const uint32_t blocks_c = (g.ncols + OPEN_CB - 1) / OPEN_CB;
    uint32_t nslab = (uint32_t)std::min<uint64_t>(blocks_c, std::max<uint64_t>(1, 1024 / (uint64_t)g.nseg));
    g.slab = ((blocks_c + nslab - 1) / nslab) * OPEN_CB;
    g.nslab = (g.ncols + g.slab - 1) / g.slab;
    g.kind = g.n % OPEN_SEG == 0 ? 1 : 0;
}

void launch_open_dot_groups(std::vector<OpenGroup> &gs, hipStream_t s) {
    std::vector<OpenGroup> live;
    for (const OpenGroup &g : gs)
        if (g.ncols) live.push_back(g);
    gs.swap(live);
    if (gs.empty()) return;
    size_t tot = 0;
    uint32_t gx = 1, gy = 1, maxc = 1;
    bool kinds[2] = {false, false};
    for (OpenGroup &g : gs) {
        open_group_shape(g);
        tot += (size_t)g.ncols * g.nseg * 8;
        gx = std::max<uint32_t>(gx, (uint32_t)g.nseg);
        gy = std::max(gy, g.nslab);
        maxc = std::max(maxc, g.ncols);
        kinds[g.kind] = true;
    }
    ARG_CHECK(gs.size() <= 65535, "too many opening groups");
    DBuf part(tot, s), dg((gs.size() * sizeof(OpenGroup) + 3) / 4, s);
    size_t off = 0;
    for (OpenGroup &g : gs) {
        g.partial = part.p + off;
        off += (size_t)g.ncols * g.nseg * 8;
    }
    HIP_CHECK(hipMemcpyAsync(dg.p, gs.data(), gs.size() * sizeof(OpenGroup), hipMemcpyHostToDevice, s));
    const OpenGroup *d = reinterpret_cast<const OpenGroup *>(dg.p);
    const dim3 grid(gx, gy, (unsigned)gs.size());
    if (kinds[0]) hipLaunchKernelGGL(k_open_dot_groups<0>, grid, dim3(NT), 0, s, d);
    if (kinds[1]) hipLaunchKernelGGL(k_open_dot_groups<1>, grid, dim3(NT), 0, s, d);
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_open_sum_groups, dim3(maxc, 1, (unsigned)gs.size()), dim3(64), 0, s, d);
    HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------ FRI reduced openings
// ro[i] = sum_m sum_p (B_{m,p} - A_{m,p} S_m(i)) / (z_p - x_i),  S_m(i) = sum_c alpha^c y_{m,c}[i],
// x_i = 3 w_h^rev(i) (the LDE row's point).  terms: per matrix: [ncols, col table offset, npts,
// (pt, A(4), B(4)) x npts] (words).  One launch per height writes ro outright (no accumulate).  A thread
// takes RED_ROWS rows i + k T (T = the grid's threads: every load instruction stays one coalesced row
// range) and inverts their 2 RED_ROWS denominators together (Montgomery's trick, one EF inversion),
// so no table of inverses crosses HBM.  One row per thread: ~50 VGPRs, 8 waves per SIMD; four rows took
// 177 VGPRs and ran 2.2x slower (the kernel is bound by the loads in flight, not the inversions).
static constexpr int RED_ROWS = 1;
// LB column loads in flight per thread: 4 (per shard 0.93-0.96 ms against
// 1.12 (8), 1.08 (2), 1.41 (1), 1.34 (16): each load instruction of a wave reads 256 B of one column, and fewer
// columns per thread at a time keep more of the concurrent waves on the same columns (profiles/r05_fri_reduce_ab.txt)
template <int LB>
__global__ __launch_bounds__(NT) void k_fri_reduce(ReduceArgs a) {
    const uint64_t T = (uint64_t)gridDim.x * NT, i0 = (uint64_t)blockIdx.x * NT + threadIdx.x;
    ef t0[RED_ROWS], t1[RED_ROWS];
#pragma unroll
    for (int k = 0; k < RED_ROWS; k++) {
        const uint64_t i = i0 + k * T;
        t0[k] = ef_zero();
        t1[k] = ef_zero();
        if (i >= a.h) continue;
        const uint32_t *d = a.desc;
        for (uint32_t m = 0; m < a.nmats; m++) {
            const uint32_t ncols = d[0], coff = d[1], npts = d[2];
            // S = sum_c alpha^c y_c / R: the (uniform) alpha^c split into 16-bit halves, eight
            // v_mad_u64_u32 per element (SGPR multipliers) and no reduction until the matrix ends
            EfAcc acc;
            acc.zero();
            uint32_t c = 0;
            for (; c + LB <= ncols; c += LB) {  // LB loads in flight
                uint32_t v[LB];
#pragma unroll
                for (int q = 0; q < LB; q++) v[q] = ((const uint32_t *)a.cols[coff + c + q])[i];
#pragma unroll
                for (int q = 0; q < LB; q++) acc.base(v[q], a.alpha_pows + 4 * (c + q));
            }
            for (; c < ncols; c++) acc.base(((const uint32_t *)a.cols[coff + c])[i], a.alpha_pows + 4 * c);
            const ef s = acc.value();
            const uint32_t *pp = d + 3;
            for (uint32_t p = 0; p < npts; p++, pp += 9) {
                ef A{{pp[1], pp[2], pp[3], pp[4]}}, B{{pp[5], pp[6], pp[7], pp[8]}};
                ef v = ef_sub(B, ef_mul(A, s));
                if (pp[0]) t1[k] = ef_add(t1[k], v); else t0[k] = ef_add(t0[k], v);
            }
            d = pp;
        }
    }
    // denominators z_p - x_i of the thread's rows (rows past h: 1), one inversion for all of them
    ef den[2 * RED_ROWS], pre[2 * RED_ROWS];
    ef run = ef_one();
#pragma unroll
    for (int k = 0; k < RED_ROWS; k++) {
        const uint64_t i = i0 + k * T;
        const bool in = i < a.h;
        // x = gen w_h^rev(i).  The wave's 64 rows share i >> 6, so rev(i) = rev6(i & 63) 2^(L-6) + rev_{L-6}(i >> 6):
        // w_h^rev(i) = w_64^rev6(lane) (a 64-entry table) times a factor uniform over the wave, instead of 64
        // scattered loads from the 2^L-entry table (one cache line per lane)
        uint32_t x = 0u;
        if (in) {
            if (a.log_h >= 6) {
                const uint32_t lo = (uint32_t)i & 63u, hi = (uint32_t)(i >> 6);
                const uint32_t wl = root_pow(a.tw, 64, rev_bits(lo, 6));
                const uint32_t wh = root_pow(a.tw, a.h, a.log_h > 6 ? rev_bits(hi, a.log_h - 6) : 0u);
                x = mul(a.gen, mul(wh, wl));
            } else {
                x = mul(a.gen, root_pow(a.tw, a.h, rev_bits((uint32_t)i, a.log_h)));
            }
        }
        den[2 * k] = in ? ef_sub(a.z0, ef_base(x)) : ef_one();
        den[2 * k + 1] = in && a.has1 ? ef_sub(a.z1, ef_base(x)) : ef_one();
#pragma unroll
        for (int q = 0; q < 2; q++) {
            pre[2 * k + q] = run;
            run = ef_mul(run, den[2 * k + q]);
        }
    }
    ef iv = ef_inv(run);
#pragma unroll
    for (int k = RED_ROWS - 1; k >= 0; k--) {
        const ef inv1 = ef_mul(iv, pre[2 * k + 1]);
        iv = ef_mul(iv, den[2 * k + 1]);
        const ef inv0 = ef_mul(iv, pre[2 * k]);
        iv = ef_mul(iv, den[2 * k]);
        const uint64_t i = i0 + k * T;
        if (i < a.h) {
            ef r = ef_mul(t0[k], inv0);
            if (a.has1) r = ef_add(r, ef_mul(t1[k], inv1));
            st_ef(a.ro + 4 * i, r);
        }
    }
}

void launch_fri_reduce(const ReduceArgs &a, hipStream_t s) {
    const uint64_t threads = (a.h + RED_ROWS - 1) / RED_ROWS;
    hipLaunchKernelGGL(k_fri_reduce<4>, dim3((unsigned)((threads + NT - 1) / NT)), dim3(NT), 0, s, a);
    HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------ FRI commit phase
// next[i] = (1/2 + b/2 g^-rev(i)) lo + (1/2 - b/2 g^-rev(i)) hi + b^2 ro[i]; g = w_{2h}
// fargs = (b/2, b^2) as two EF values, written on the device by k_fri_chal
__global__ __launch_bounds__(NT) void k_fri_fold(const uint32_t *cur, uint64_t h, int log_h, const uint32_t *fargs,
                                                 const uint32_t *__restrict__ tw_inv, const uint32_t *ro, uint32_t *next) {
    const uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= h) return;
    const ef half_beta = ld_ef(fargs), beta2 = ld_ef(fargs + 4);
    const uint32_t half = halve(ONE);
    const uint32_t g = tw_inv[h + rev_bits((uint32_t)i, log_h)];
    const ef pw = ef_mul_base(half_beta, g);
    const ef lo = ld_ef(cur + 8 * i), hi = ld_ef(cur + 8 * i + 4);
    ef r = ef_add(ef_mul(ef_add_base(pw, half), lo), ef_mul(ef_sub(ef_base(half), pw), hi));
    if (ro) r = ef_add(r, ef_mul(beta2, ld_ef(ro + 4 * i)));
    st_ef(next + 4 * i, r);
}

// one folded element (k_fri_fold's formula) of an h-element output
__device__ __forceinline__ ef fri_fold_one(const uint32_t *cur, uint64_t j, uint64_t h, int log_h, const ef &half_beta,
                                           const ef &beta2, const uint32_t *__restrict__ tw_inv, const uint32_t *ro) {
    const uint32_t half = halve(ONE);
    const uint32_t g = tw_inv[h + rev_bits((uint32_t)j, log_h)];
    const ef pw = ef_mul_base(half_beta, g);
    const ef lo = ld_ef(cur + 8 * j), hi = ld_ef(cur + 8 * j + 4);
    ef r = ef_add(ef_mul(ef_add_base(pw, half), lo), ef_mul(ef_sub(ef_base(half), pw), hi));
    if (ro) r = ef_add(r, ef_mul(beta2, ld_ef(ro + 4 * j)));
    return r;
}

// The fold of round r and the leaves of round r + 1 in one pass: thread i folds next[2i], next[2i + 1]
// (stored: the queries open them) and hashes them into leaf i (one permutation)
__global__ __launch_bounds__(NT) void k_fri_fold_leaves(const uint32_t *cur, uint64_t h, int log_h,
                                                        const uint32_t *fargs, const uint32_t *__restrict__ tw_inv,
                                                        const uint32_t *ro, uint32_t *next, uint32_t *leaves) {
    const uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= h / 2) return;
    const ef hb = ld_ef(fargs), b2 = ld_ef(fargs + 4);
    const ef a = fri_fold_one(cur, 2 * i, h, log_h, hb, b2, tw_inv, ro);
    const ef b = fri_fold_one(cur, 2 * i + 1, h, log_h, hb, b2, tw_inv, ro);
    st_ef(next + 8 * i, a);
    st_ef(next + 8 * i + 4, b);
    uint32_t s[16];
#pragma unroll
    for (int e = 0; e < 4; e++) { s[e] = a.c[e]; s[4 + e] = b.c[e]; s[8 + e] = 0; s[12 + e] = 0; }
    p2::permute(s);
    uint4 *o = (uint4 *)(leaves + 8 * i);
    o[0] = make_uint4(s[0], s[1], s[2], s[3]);
    o[1] = make_uint4(s[4], s[5], s[6], s[7]);
}
// 16-lane form for small rounds: lane l < 8 folds element 2i + l / 4 and keeps component l % 4
__global__ __launch_bounds__(NT) void k_fri_fold_leaves16(const uint32_t *cur, uint64_t h, int log_h,
                                                          const uint32_t *fargs, const uint32_t *__restrict__ tw_inv,
                                                          const uint32_t *ro, uint32_t *next, uint32_t *leaves) {
    const uint64_t t = (uint64_t)blockIdx.x * NT + threadIdx.x;
    const uint64_t i = t >> 4;
    const int l = (int)(t & 15);
    const bool act = i < h / 2 && l < 8;
    uint32_t v = 0;
    if (act) {
        const uint64_t j = 2 * i + (l >> 2);
        const ef r = fri_fold_one(cur, j, h, log_h, ld_ef(fargs), ld_ef(fargs + 4), tw_inv, ro);
        v = r.c[l & 3];
        next[4 * j + (l & 3)] = v;
    }
    const uint32_t x = p2x16::permute(v, p2x16::lane_consts(l));  // all lanes take part
    if (act) leaves[8 * i + l] = x;
}

// leaf i = sponge(cur[2i] || cur[2i+1]) (8 elements: one permutation)
__global__ __launch_bounds__(NT) void k_fri_leaves(const uint32_t *cur, uint64_t h, uint32_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= h) return;
    uint32_t s[16];
    const uint4 a = *(const uint4 *)(cur + 8 * i), b = *(const uint4 *)(cur + 8 * i + 4);
    s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w; s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
#pragma unroll
    for (int k = 8; k < 16; k++) s[k] = 0;
    p2::permute(s);
    uint4 *o = (uint4 *)(out + 8 * i);
    o[0] = make_uint4(s[0], s[1], s[2], s[3]);
    o[1] = make_uint4(s[4], s[5], s[6], s[7]);
}
__global__ __launch_bounds__(NT) void k_fri_leaves16(const uint32_t *cur, uint64_t h, uint32_t *out) {
    const uint64_t t = (uint64_t)blockIdx.x * NT + threadIdx.x;
    const uint64_t i = t >> 4;
    const int l = (int)(t & 15);
    const uint32_t x = p2x16::permute(i < h && l < 8 ? cur[8 * i + l] : 0u, p2x16::lane_consts(l));
    if (i < h && l < 8) out[8 * i + l] = x;
}

// One FRI round of the Fiat-Shamir transcript on the device (fri_chal.cuh), for rounds whose tree
// top did not run it (a one-leaf tree)
__global__ __launch_bounds__(64) void k_fri_chal(DevChallenger *c, const uint32_t *root, uint32_t *root_out,
                                                 uint32_t *fargs) {
    __shared__ ChalShared sh;
    fri_chal_block(sh, c, root, root_out, fargs);
}

void launch_fri_fold(const uint32_t *cur, uint64_t h, const uint32_t *fargs, const uint32_t *tw_inv,
                     const uint32_t *ro, uint32_t *next, hipStream_t s) {
    hipLaunchKernelGGL(k_fri_fold, dim3((unsigned)((h + NT - 1) / NT)), dim3(NT), 0, s, cur, h, ilog2(h), fargs,
                       tw_inv, ro, next);
    HIP_CHECK(hipGetLastError());
}
void launch_fri_fold_leaves(const uint32_t *cur, uint64_t h, const uint32_t *fargs, const uint32_t *tw_inv,
                            const uint32_t *ro, uint32_t *next, uint32_t *leaves, hipStream_t s) {
    ARG_CHECK(h >= 2 && (h & (h - 1)) == 0, "fold+leaves needs a power-of-two output >= 2");
    const uint64_t nl = h / 2;
    if (nl <= 8192)
        hipLaunchKernelGGL(k_fri_fold_leaves16, dim3((unsigned)((nl * 16 + NT - 1) / NT)), dim3(NT), 0, s, cur, h,
                           ilog2(h), fargs, tw_inv, ro, next, leaves);
    else
        hipLaunchKernelGGL(k_fri_fold_leaves, dim3((unsigned)((nl + NT - 1) / NT)), dim3(NT), 0, s, cur, h, ilog2(h),
                           fargs, tw_inv, ro, next, leaves);
    HIP_CHECK(hipGetLastError());
}
void launch_fri_leaves(const uint32_t *cur, uint64_t h, uint32_t *out, hipStream_t s) {
    if (h <= 8192)
        hipLaunchKernelGGL(k_fri_leaves16, dim3((unsigned)((h * 16 + NT - 1) / NT)), dim3(NT), 0, s, cur, h, out);
    else
        hipLaunchKernelGGL(k_fri_leaves, dim3((unsigned)((h + NT - 1) / NT)), dim3(NT), 0, s, cur, h, out);
    HIP_CHECK(hipGetLastError());
}
void launch_fri_chal(DevChallenger *c, const uint32_t *root, uint32_t *root_out, uint32_t *fargs, hipStream_t s) {
    hipLaunchKernelGGL(k_fri_chal, dim3(1), dim3(64), 0, s, c, root, root_out, fargs);
    HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------ proof of work
__global__ __launch_bounds__(NT) void k_pow(PowArgs a, uint32_t base, uint32_t *result) {
    const uint32_t w = base + blockIdx.x * NT + threadIdx.x;
    if (w >= P) return;
    uint32_t s[16];
#pragma unroll
    for (int k = 0; k < 16; k++) s[k] = a.state[k];
#pragma unroll
    for (int k = 0; k < 8; k++)
        if (k < (int)a.nin) s[k] = a.in[k];
    const uint32_t wm = to_mont(w);
#pragma unroll
    for (int k = 0; k < 8; k++)
        if (k == (int)a.nin) s[k] = wm;
    p2::permute(s);
    if ((from_mont(s[7]) & a.mask) == 0) atomicMin(result, w);
}

uint32_t run_pow(const PowArgs &a, hipStream_t s) {
    DBuf res(1, s);
    const uint32_t batch = 1u << 20;
    for (uint64_t base = 0; base < P; base += batch) {
        uint32_t init = 0xffffffffu, got = 0;
        HIP_CHECK(hipMemcpyAsync(res.p, &init, 4, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_pow, dim3(batch / NT), dim3(NT), 0, s, a, (uint32_t)base, res.p);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(&got, res.p, 4, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        if (got != 0xffffffffu) return got;
    }
    throw HipError("no proof-of-work witness found");
}

// ------------------------------------------------------------------ gathers
// item: src (u64 ptr), stride (elements), count, dst offset
__global__ __launch_bounds__(64) void k_gather(const uint64_t *__restrict__ items, uint32_t *dst) {
    const uint64_t *it = items + 3 * blockIdx.x;
    const uint32_t *src = (const uint32_t *)it[0];
    const uint64_t stride = it[1] & 0xffffffffull, count = it[1] >> 32;
    const uint64_t off = it[2];
    for (uint64_t k = threadIdx.x; k < count; k += 64) dst[off + k] = src[k * stride];
}

void launch_gather(const uint64_t *d_items, uint32_t nitems, uint32_t *dst, hipStream_t s) {
    if (!nitems) return;
    hipLaunchKernelGGL(k_gather, dim3(nitems), dim3(64), 0, s, d_items, dst);
    HIP_CHECK(hipGetLastError());
}

}  // namespace zkm
