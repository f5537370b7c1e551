// JIT-specialised quotient and permutation-trace kernels (hiprtc, gfx950).
//
// At setup (MachineProver::setup / pk_to_device) every chip's constraint program and lookup
// descriptors are lowered to straight-line HIP: column reads are hoisted to the top of the kernel
// (so their HBM latency overlaps), constants and VirtualPairCol weights become literals, LogUp
// batches are unrolled, and the folding sum(alpha^(n-1-k) C_k) keeps the reference's constraint
// order (crates/stark/src/folder.rs:79-102, permutation.rs:256-346).  The generic interpreter
// kernel (open_kernels.hip k_quotient) remains as the GPU path when JIT compilation is disabled
// (ZKM_NO_JIT=1) or fails.
//
// Compiled code objects are cached by a hash of (source, arch, options): in memory for the process,
// and on disk in ZKM_JIT_CACHE (default: jit_cache/ next to this library; "off" disables it), so a
// large chip (ShaExtend: ~1 min of hiprtc) compiles once per tree.  __graft_entry__.build() fills
// the cache for the shipped machines on the build host (hiprtc needs no device).
#include "jit.hpp"

#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <future>
#include <map>
#include <mutex>
#include <utime.h>
#include <sstream>
#include <unordered_map>

#include "jit_prelude.inc"

namespace zkm {

int guard_status(const std::exception &e);  // capi.cpp

namespace {

std::string hex(uint32_t v) {
    char b[16];
    snprintf(b, sizeof b, "0x%08xu", v);
    return b;
}

// Column reads are software-pipelined: the i-th distinct read is issued `lookahead` reads ahead
// of its first use and pinned there with a scheduling barrier.  Hoisting every read to the top
// holds ~200 values live (2 waves/SIMD); issuing each at first use leaves the wave waiting on HBM
// at every constraint; a fixed window keeps ~lookahead loads in flight at a modest register cost.
struct Gen {
    std::ostringstream body;
    int tmp = 0;
    std::map<std::string, std::string> loads;  // load expr -> variable
    std::vector<std::string> load_stmts;
    std::ostringstream head;
    std::string var(const std::string &prefix) { return prefix + std::to_string(tmp++); }
    std::string col(const char *arr, uint32_t c, const char *row) {
        std::string key = std::string(arr) + "_" + std::to_string(c) + "_" + row;
        auto it = loads.find(key);
        if (it != loads.end()) return it->second;
        std::string v = "c_" + key;
        body << "//@L " << load_stmts.size() << "\n";
        load_stmts.push_back("    const uint32_t " + v + " = A." + arr + "[(uint64_t)" + std::to_string(c) +
                             " * A.ld + " + row + "];\n");
        loads[key] = v;
        return v;
    }
    // body with the load markers replaced by the pipelined reads (each read issued `look` reads ahead of its
    // first use and pinned there by a scheduling barrier)
    std::string pipelined(int look) const {
        const bool barrier = true;
        std::istringstream in(body.str());
        std::ostringstream out;
        std::string line;
        size_t next = 0;
        while (std::getline(in, line)) {
            if (line.rfind("//@L ", 0) == 0) {
                const size_t i = std::stoul(line.substr(5));
                const size_t upto = std::min(load_stmts.size(), i + 1 + (size_t)look);
                if (next < upto) {
                    for (; next < upto; next++) out << load_stmts[next];
                    if (barrier) out << "    __builtin_amdgcn_sched_barrier(0);\n";
                }
                continue;
            }
            out << line << "\n";
        }
        return out.str();
    }
};

// Chips with more local lookups than this get their LogUp code as a loop over the flattened lookup
// table (chip.cpp flatten_chip) instead of straight-line code: hiprtc time grows much faster than
// linearly with the unrolled lookups (ShaCompress, 116 lookups: minutes; EdAddAssign has 881), while
// the table walk is wave-uniform (scalar loads of the descriptors, one column read per term).
constexpr int kJitLookupUnroll = 64;
constexpr int kPermLdsBatches = 10;  // LogUp batches staged in LDS (4 words x 256 threads each)

// device helpers of the loop form: a VirtualPairCol at a row from the flattened table (advances off)
const char *kLoopHelpers = R"(
__device__ __forceinline__ uint32_t jvpc(const uint32_t *__restrict__ prog, uint32_t &off,
                                         const uint32_t *__restrict__ m, const uint32_t *__restrict__ pp,
                                         uint64_t ld, uint64_t row) {
    const uint32_t nt = prog[off];
    uint32_t acc = prog[off + 1 + 2 * nt];
    for (uint32_t i = 0; i < nt; i++) {
        const uint32_t col = prog[off + 1 + 2 * i], w = prog[off + 2 + 2 * i];
        const uint32_t v = (col & 0x80000000u) ? m[(uint64_t)(col & 0x7fffffffu) * ld + row] : pp[(uint64_t)col * ld + row];
        acc = add(acc, mul(v, w));
    }
    off += 2 + 2 * nt;
    return acc;
}
// rlc = alpha + kind + sum_v beta^(v+1) x_v and the signed multiplicity of lookup i
__device__ __forceinline__ ef jlookup(const uint32_t *__restrict__ prog, uint32_t i, const ef &alpha,
                                      const uint32_t *__restrict__ bp, const uint32_t *__restrict__ m,
                                      const uint32_t *__restrict__ pp, uint64_t ld, uint64_t row, uint32_t &mult) {
    const uint32_t *lk = prog + prog[3] + 4 * i;
    ef d = ef_add_base(alpha, lk[0]);
    uint32_t off = lk[3];
    for (uint32_t v = 0; v < lk[2]; v++) {
        const uint32_t x = jvpc(prog, off, m, pp, ld, row);
        d = ef_add(d, ef_mul_base(ef{{bp[4 * v], bp[4 * v + 1], bp[4 * v + 2], bp[4 * v + 3]}}, x));
    }
    const uint32_t mm = jvpc(prog, off, m, pp, ld, row);
    mult = lk[1] ? mm : neg(mm);
    return d;
}
// num / den of lookups [i0, i1): num = sum_i m_i prod_{j != i} d_j, den = prod_i d_i
__device__ __forceinline__ void jbatch(const uint32_t *__restrict__ prog, uint32_t i0, uint32_t i1, const ef &alpha,
                                       const uint32_t *__restrict__ bp, const uint32_t *__restrict__ m,
                                       const uint32_t *__restrict__ pp, uint64_t ld, uint64_t row, ef &num, ef &den) {
    uint32_t mu;
    den = jlookup(prog, i0, alpha, bp, m, pp, ld, row, mu);
    num = ef{{mu, 0u, 0u, 0u}};
    for (uint32_t i = i0 + 1; i < i1; i++) {
        const ef d = jlookup(prog, i, alpha, bp, m, pp, ld, row, mu);
        num = ef_add(ef_mul(num, d), ef_mul_base(den, mu));
        den = ef_mul(den, d);
    }
}
)";

// value of a VirtualPairCol at the local row
std::string vpc_expr(Gen &g, const VPC &v) {
    std::string acc = kb::to_mont(v.constant) ? hex(kb::to_mont(v.constant)) : "";
    for (size_t i = 0; i < v.cols.size(); i++) {
        const uint32_t col = v.cols[i];
        const std::string x = (col & 0x80000000u) ? g.col("main", col & 0x7fffffffu, "rl") : g.col("prep", col, "rl");
        const uint32_t w = kb::to_mont(v.weights[i]);
        std::string term = (w == kb::ONE) ? x : "mul(" + x + ", " + hex(w) + ")";
        acc = acc.empty() ? term : "add(" + acc + ", " + term + ")";
    }
    if (acc.empty()) acc = "0u";
    std::string t = g.var("v");
    g.body << "    const uint32_t " << t << " = " << acc << ";\n";
    return t;
}

// alpha + kind + sum_v beta^(v+1) x_v (the lookup's random linear combination): values in pairs,
// each pair one v_mad_u64_u32 chain and one lazy reduction per component (kb::ef_dot2)
std::string rlc_expr(Gen &g, const char *alpha, const LookupDesc &lk) {
    std::string rlc = g.var("r");
    g.body << "    ef " << rlc << " = ef_add_base(" << alpha << ", " << hex(kb::to_mont(lk.kind)) << ");\n";
    std::vector<std::string> xs;
    for (size_t v = 0; v < lk.values.size(); v++) xs.push_back(vpc_expr(g, lk.values[v]));
    size_t v = 0;
    for (; v + 2 <= xs.size(); v += 2)
        g.body << "    " << rlc << " = ef_dot2(" << rlc << ", " << xs[v] << ", A.beta_pows + " << 4 * v << ", " << xs[v + 1]
               << ", A.beta_pows + " << 4 * (v + 1) << ");\n";
    if (v < xs.size())
        g.body << "    " << rlc << " = ef_add(" << rlc << ", ef_mul_base(BPOW(" << v << "), " << xs[v] << "));\n";
    return rlc;
}

// One LogUp batch (lookups [i0, i1) of the chip's local lookups): num / den = sum_i m_i / rlc_i with
// den = prod_i rlc_i and num = sum_i m_i prod_{j != i} rlc_j (permutation.rs:29-69 / :256-333), built
// incrementally.  The first lookup sets num = m_0 (a base-field value) and den = rlc_0 directly, and
// while num is still base-field the next step multiplies it as a base element (4 products, not 16):
// a batch of two costs 2 EF x base products and one EF product instead of three EF products.
void lookup_batch(Gen &g, const ChipDesc &c, int i0, int i1, const char *alpha, const std::string &num,
                  const std::string &den) {
    std::string num_base;  // num as a base-field variable while it is one
    for (int i = i0; i < i1; i++) {
        const LookupDesc &lk = c.local[i];
        std::string d = rlc_expr(g, alpha, lk);
        std::string m = vpc_expr(g, lk.mult);
        if (!lk.is_send) {
            std::string t = g.var("t");
            g.body << "    const uint32_t " << t << " = neg(" << m << ");\n";
            m = t;
        }
        if (i == i0) {
            num_base = m;
            g.body << "    " << den << " = " << d << ";\n";
            continue;
        }
        const std::string nd = num_base.empty() ? "ef_mul(" + num + ", " + d + ")" : "ef_mul_base(" + d + ", " + num_base + ")";
        g.body << "    " << num << " = ef_add(" << nd << ", ef_mul_base(" << den << ", " << m << "));\n";
        g.body << "    " << den << " = ef_mul(" << den << ", " << d << ");\n";
        num_base.clear();
    }
    if (!num_base.empty()) g.body << "    " << num << " = ef{{" << num_base << ", 0u, 0u, 0u}};\n";
}

// Chips whose AIR program lowers to more constraints than this get it as a chain of non-inlined
// device functions (each a slice of consecutive constraints with its own column reads and its own
// EfAcc, the kernel adding the slices' folded values), so no single function is huge: hiprtc -O3 time
// grows much faster than linearly with the size of one straight-line function (KeccakSponge, 3788
// constraints in one body: > 40 min; as slices: minutes).  The folded sum is the same field element.
constexpr int kJitSliceConstraints = 2048;
constexpr int kJitSliceLines = 6000;  // generated statements per slice

std::string gen_source(const ChipDesc &c, const std::string &fname) {
    Gen g;
    std::ostringstream o, slices;
    int k = 0;  // constraint index
    // folding sum_k alpha^(n-1-k) C_k: split-constant 64-bit accumulator (kb::EfAcc), reduced once
    auto emit_base = [&](const std::string &x) {
        g.body << "    facc.base(" << x << ", A.pows + " << 4 * k << ");\n";
        k++;
    };
    auto emit_ext = [&](const std::string &x) {
        g.body << "    facc.ext(" << x << ", A.pows + " << 4 * k << ");\n";
        k++;
    };
    // ---- AIR program -> straight-line code ----
    std::vector<std::string> st;
    std::vector<std::string> slot;  // shared subexpressions: slot -> the variable holding its value
    int n_air = 0;
    for (size_t pc = 0; pc < c.code.size();) {  // count the AIR constraints (OP_EMITs)
        const uint32_t op = c.code[pc++];
        if (op == OP_EMIT) n_air++;
        else if (op == OP_MAIN_L || op == OP_MAIN_N || op == OP_PREP_L || op == OP_PREP_N || op == OP_CONST ||
                 op == OP_PV || op == OP_LET || op == OP_GET) pc++;
    }
    const bool sliced = n_air > kJitSliceConstraints;
    // program() puts every shared definition (code, OP_LET) ahead of the first constraint.  Unsliced, each
    // is evaluated there once; sliced, a definition is evaluated in a slice at its first OP_GET there
    // (slices are separate functions), so no value is live across a slice boundary.
    std::vector<std::pair<size_t, size_t>> slot_def;  // code range of each slot's definition
    size_t first_constraint = 0;
    for (size_t pc = 0; pc < c.code.size();) {
        const size_t at = pc;
        const uint32_t op = c.code[pc++];
        if (op == OP_LET) {
            slot_def.emplace_back(first_constraint, at);
            first_constraint = ++pc;
        } else if (op == OP_EMIT) {
            break;
        } else if (op == OP_MAIN_L || op == OP_MAIN_N || op == OP_PREP_L || op == OP_PREP_N || op == OP_CONST ||
                   op == OP_PV || op == OP_GET) {
            pc++;
        }
    }
    std::map<uint32_t, std::string> lazy;  // sliced: slot -> its variable in the current slice
    int n_slices = 0;
    size_t slice_lines = 0;
    auto close_slice = [&]() {
        slices << "__device__ __noinline__ ef zq_slice" << n_slices++ << "(const ZkmQuotJitArgs &A, uint64_t rl, uint64_t rn, "
               << "uint32_t is_first, uint32_t is_last, uint32_t is_trans) {\n"
               << "    (void)rl; (void)rn; (void)is_first; (void)is_last; (void)is_trans;\n"
               << "    EfAcc facc;\n    facc.zero();\n"
               << g.pipelined(8) << "    return facc.value();\n}\n";
        g = Gen{};
        lazy.clear();
        slice_lines = 0;
    };
    // the stack machine over code[from, to)
    std::function<void(size_t, size_t, std::vector<std::string> &)> run;
    run = [&](size_t from, size_t to, std::vector<std::string> &st) {
        for (size_t pc = from; pc < to;) {
            const uint32_t op = c.code[pc++];
            slice_lines++;
            switch (op) {
            case OP_MAIN_L: st.push_back(g.col("main", c.code[pc++], "rl")); break;
            case OP_MAIN_N: st.push_back(g.col("main", c.code[pc++], "rn")); break;
            case OP_PREP_L: st.push_back(g.col("prep", c.code[pc++], "rl")); break;
            case OP_PREP_N: st.push_back(g.col("prep", c.code[pc++], "rn")); break;
            case OP_CONST: st.push_back(hex(kb::to_mont(c.code[pc++]))); break;
            case OP_PV: st.push_back("A.pv[" + std::to_string(c.code[pc++]) + "]"); break;
            case OP_IS_FIRST: st.push_back("is_first"); break;
            case OP_IS_LAST: st.push_back("is_last"); break;
            case OP_IS_TRANS: st.push_back("is_trans"); break;
            case OP_ADD: case OP_SUB: case OP_MUL: {
                std::string b = st.back(); st.pop_back();
                std::string a = st.back(); st.pop_back();
                std::string t = g.var("t");
                const char *f = op == OP_ADD ? "add" : op == OP_SUB ? "sub" : "mul";
                g.body << "    const uint32_t " << t << " = " << f << "(" << a << ", " << b << ");\n";
                st.push_back(t);
                break;
            }
            case OP_NEG: {
                std::string a = st.back(); st.pop_back();
                std::string t = g.var("t");
                g.body << "    const uint32_t " << t << " = neg(" << a << ");\n";
                st.push_back(t);
                break;
            }
            case OP_EMIT: {
                std::string a = st.back(); st.pop_back();
                emit_base(a);
                if (sliced && st.empty() && slice_lines >= (size_t)kJitSliceLines) close_slice();
                break;
            }
            case OP_LET: {  // the value is already a named SSA variable; bind the slot to it
                pc++;
                slot.push_back(st.back());
                st.pop_back();
                break;
            }
            case OP_GET: {
                const uint32_t sl = c.code[pc++];
                if (!sliced) {
                    st.push_back(slot.at(sl));
                } else {
                    auto it = lazy.find(sl);
                    if (it == lazy.end()) {
                        std::vector<std::string> sub;
                        run(slot_def.at(sl).first, slot_def.at(sl).second, sub);
                        it = lazy.emplace(sl, sub.back()).first;
                    }
                    st.push_back(it->second);
                }
                break;
            }
            default: throw ArgError("bad opcode in JIT");
            }
        }
    };
    run(sliced ? first_constraint : 0, c.code.size(), st);
    if (sliced) {
        close_slice();
        g.body << "    ef slices = ef_zero();\n";
        for (int i = 0; i < n_slices; i++)
            g.body << "    slices = ef_add(slices, zq_slice" << i << "(A, rl, rn, is_first, is_last, is_trans));\n";
    }
    // ---- LogUp constraints (permutation.rs:256-333) ----
    const int nloc = (int)c.local.size();
    if (nloc > kJitLookupUnroll) {
        // loop form: batches walked at run time, constraint index k + b
        const int batch = 1 << c.log_qd, nb = c.perm_w - 1;
        g.body << "    {\n"
               << "        ef sl = ef_zero(), sn = ef_zero();\n"
               << "        for (int b = 0; b < " << nb << "; b++) {\n"
               << "            const uint32_t i0 = (uint32_t)b * " << batch << ", i1 = min(i0 + " << batch << "u, "
               << nloc << "u);\n"
               << "            ef num, den;\n"
               << "            jbatch(A.prog, i0, i1, alpha_p, A.beta_pows, A.main, A.prep, A.ld, rl, num, den);\n"
               << "            ef el, en;\n"
               << "            for (int e = 0; e < 4; e++) { el.c[e] = A.perm[(uint64_t)(4 * b + e) * A.ld + rl];"
               << " en.c[e] = A.perm[(uint64_t)(4 * b + e) * A.ld + rn]; }\n"
               << "            facc.ext(ef_sub(ef_mul(den, el), num), A.pows + 4 * (" << k << " + b));\n"
               << "            sl = ef_add(sl, el); sn = ef_add(sn, en);\n"
               << "        }\n"
               << "        ef pl, pn;\n"
               << "        for (int e = 0; e < 4; e++) { pl.c[e] = A.perm[(uint64_t)(" << 4 * nb << " + e) * A.ld + rl];"
               << " pn.c[e] = A.perm[(uint64_t)(" << 4 * nb << " + e) * A.ld + rn]; }\n";
        k += nb;
        g.body << "        facc.ext(ef_mul_base(ef_sub(pl, sl), is_first), A.pows + " << 4 * k << ");\n"
               << "        facc.ext(ef_mul_base(ef_sub(ef_sub(pn, pl), sn), is_trans), A.pows + " << 4 * (k + 1) << ");\n"
               << "        facc.ext(ef_mul_base(ef_sub(pl, lcs), is_last), A.pows + " << 4 * (k + 2) << ");\n"
               << "    }\n";
        k += 3;
    } else if (nloc) {
        const int batch = 1 << c.log_qd, nb = c.perm_w - 1;
        // perm-trace columns (local / next row) are read where they are consumed, so only the
        // running sums sl, sn stay live across the batches
        auto perm_ef = [&](int b, const char *row) {
            std::string v = g.var("pe");
            std::string le = "ef{{";
            for (int e = 0; e < 4; e++) le += (e ? ", " : "") + g.col("perm", 4 * b + e, row);
            g.body << "    const ef " << v << " = " << le << "}};\n";
            return v;
        };
        std::string sl = g.var("sl"), sn = g.var("sn");
        g.body << "    ef " << sl << " = ef_zero(), " << sn << " = ef_zero();\n";
        for (int b = 0; b < nb; b++) {
            std::string prod = g.var("pr"), num = g.var("nu");
            g.body << "    ef " << prod << ", " << num << ";\n";
            lookup_batch(g, c, b * batch, std::min(nloc, (b + 1) * batch), "alpha_p", num, prod);
            const std::string elb = perm_ef(b, "rl");
            std::string cc = g.var("cc");
            g.body << "    const ef " << cc << " = ef_sub(ef_mul(" << prod << ", " << elb << "), " << num << ");\n";
            emit_ext(cc);
            const std::string enb = perm_ef(b, "rn");
            g.body << "    " << sl << " = ef_add(" << sl << ", " << elb << "); " << sn << " = ef_add(" << sn << ", " << enb << ");\n";
        }
        const std::string eln = perm_ef(nb, "rl"), enn = perm_ef(nb, "rn");
        emit_ext("ef_mul_base(ef_sub(" + eln + ", " + sl + "), is_first)");
        emit_ext("ef_mul_base(ef_sub(ef_sub(" + enn + ", " + eln + "), " + sn + "), is_trans)");
        emit_ext("ef_mul_base(ef_sub(" + eln + ", lcs), is_last)");
    }
    if (c.scope == 1) {
        for (int i = 0; i < 7; i++) {
            emit_base("mul(sub(" + g.col("main", c.main_w - 14 + i, "rl") + ", A.gcs[" + std::to_string(i) + "]), is_last)");
            emit_base("mul(sub(" + g.col("main", c.main_w - 7 + i, "rl") + ", A.gcs[" + std::to_string(7 + i) + "]), is_last)");
        }
    }
    ARG_CHECK(k == c.n_constraints, "JIT constraint count mismatch");

    o << slices.str() << "extern \"C\" __global__ void __launch_bounds__(256) " << fname << "(const ZkmQuotJitArgs A) {\n"
      // Each wave takes 64 consecutive LDE rows; the four waves of a workgroup take a chain of
      // row blocks B, next(B), next^2(B), next^3(B) (next = the rows holding the next-row
      // operands; in the bit-reversed block index that is +step), so three of the four waves
      // find their next-row operands in L2, already fetched as another wave's local rows.
      << "    uint64_t t;\n"
      << "    if (A.q >= (uint64_t)(256 * A.step)) {\n"
      << "        const uint64_t g = blockIdx.x, s = (uint64_t)A.step;\n"
      << "        const uint64_t v = 4 * s * (g / s) + (g % s) + s * (threadIdx.x >> 6);\n"
      << "        t = ((uint64_t)rev_bits((uint32_t)v, A.log_q - 6) << 6) + (threadIdx.x & 63);\n"
      << "    } else {\n"
      << "        t = (uint64_t)blockIdx.x * 256 + threadIdx.x;\n"
      << "    }\n"
      << "    if (t >= A.q) return;\n"
      << "    const uint64_t rl = t;\n"
      << "    const uint64_t k = rev_bits((uint32_t)t, A.log_q);\n"
      << "    const uint64_t kn = (k + A.step) & (A.q - 1);\n"
      << "    const uint64_t rn = rev_bits((uint32_t)kn, A.log_q);\n"
      << "    const uint64_t hq = A.q >> 1;\n"
      << "    const uint32_t om = k < hq ? A.tw[hq + k] : neg(A.tw[hq + (k - hq)]);\n"
      << "    const uint32_t x = mul(A.gen, om);\n"
      // Z_H(x) = x^n - 1 = 3^n w_{Q/n}^(k mod Q/n) - 1 (Q/n = 2^log_qd: 1, 2 or 4 values)
      << "    const uint64_t qn = A.q / A.n;\n"
      << "    uint32_t zp = ONE;\n"
      << "    if (qn > 1) { const uint64_t zm = k & (qn - 1), zhh = qn >> 1; zp = zm < zhh ? A.tw[zhh + zm] : neg(A.tw[zhh + (zm - zhh)]); }\n"
      << "    const uint32_t zh = sub(mul(A.gen_pow_n, zp), ONE);\n"
      << "    const uint32_t d_first = sub(x, ONE), d_last = sub(x, A.wn_inv);\n"
      << "    const uint32_t inv_fl = inv(mul(mul(d_first, d_last), zh));\n"
      << "    const uint32_t zh2 = mul(zh, zh);\n"
      << "    const uint32_t is_first = mul(mul(inv_fl, d_last), zh2);\n"
      << "    const uint32_t is_last = mul(mul(inv_fl, d_first), zh2);\n"
      << "    const uint32_t is_trans = d_last;\n"
      << "    const uint32_t inv_z = mul(inv_fl, mul(d_first, d_last));\n"
      << "    const ef alpha_p = ef{{A.alpha_p[0], A.alpha_p[1], A.alpha_p[2], A.alpha_p[3]}};\n"
      << "    const ef lcs = ef{{A.lcs[0], A.lcs[1], A.lcs[2], A.lcs[3]}};\n"
      << "    (void)is_first; (void)is_last; (void)is_trans; (void)alpha_p; (void)lcs;\n"
      << g.head.str()
      << "    EfAcc facc;\n"
      << "    facc.zero();\n"
      << g.pipelined(8)  // measured: 8 -> 2.27 ms, 24 -> 2.44, unpipelined 2.78
      << (sliced ? "    const ef qv = ef_mul_base(ef_add(facc.value(), slices), inv_z);\n"
                 : "    const ef qv = ef_mul_base(facc.value(), inv_z);\n")
      // chunk j = k mod 2^lqd (split_evals); t = rev_Q(k) = rev_lqd(j) * n + rev_n(k >> lqd), so the
      // chunk's position t mod n is its bit-reversed row
      << "    const uint64_t c = k & (uint64_t)(A.step - 1), pos = t & (A.n - 1);\n"
      << "    A.chunks[c * A.cstride + 0 * A.n + pos] = qv.c[0];\n"
      << "    A.chunks[c * A.cstride + 1 * A.n + pos] = qv.c[1];\n"
      << "    A.chunks[c * A.cstride + 2 * A.n + pos] = qv.c[2];\n"
      << "    A.chunks[c * A.cstride + 3 * A.n + pos] = qv.c[3];\n"
      << "}\n";
    return o.str();
}

// Permutation (LogUp) trace rows, generate_permutation_trace (crates/stark/src/permutation.rs:
// 156-203): per batch b, s_b = sum_i m_i / rlc_i as num_b / den_b, built incrementally exactly as
// the interpreter kernel; the nb denominators share ONE extension-field inversion (prefix
// products, Montgomery's trick), then the row total goes to rowsum for the running-sum scan.
// launch bounds of the LogUp kernels: 2 waves per SIMD (a 256-register cap; the unbounded kernel takes
// 267 and runs one wave per SIMD: FibCpu 1.10 -> 0.89 ms; profiles/r03_perm_waves_sweep.txt)
std::string perm_bounds() { return "__launch_bounds__(256, 2)"; }

// Loop form of the LogUp trace (chips with > kJitLookupUnroll lookups): batches in groups of 8 share
// one extension-field inversion (Montgomery's trick in registers).
std::string gen_perm_loop_source(const ChipDesc &c, const std::string &fname) {
    const int nloc = (int)c.local.size(), batch = 1 << c.log_qd, nb = c.perm_w - 1;
    std::ostringstream o;
    o << "extern \"C\" __global__ void __launch_bounds__(256) " << fname << "(const ZkmPermJitArgs A) {\n"
      << "    const uint64_t rl = (uint64_t)blockIdx.x * 256 + threadIdx.x;\n"
      << "    if (rl >= A.ld) return;\n"
      << "    const ef alpha = ef{{A.alpha[0], A.alpha[1], A.alpha[2], A.alpha[3]}};\n"
      << "    ef total = ef_zero();\n"
      << "    for (int g0 = 0; g0 < " << nb << "; g0 += 8) {\n"
      << "        const int gn = min(8, " << nb << " - g0);\n"
      << "        ef num[8], den[8], pre[8];\n"
      << "        ef run = ef_one();\n"
      << "#pragma unroll\n"
      << "        for (int j = 0; j < 8; j++) {\n"
      << "            if (j < gn) {\n"
      << "                const uint32_t i0 = (uint32_t)(g0 + j) * " << batch << ", i1 = min(i0 + " << batch << "u, " << nloc
      << "u);\n"
      << "                jbatch(A.prog, i0, i1, alpha, A.beta_pows, A.main, A.prep, A.ld, rl, num[j], den[j]);\n"
      << "            } else { num[j] = ef_zero(); den[j] = ef_one(); }\n"
      << "            pre[j] = run;\n"
      << "            run = ef_mul(run, den[j]);\n"
      << "        }\n"
      << "        ef iv = ef_inv(run);\n"
      << "#pragma unroll\n"
      << "        for (int j = 7; j >= 0; j--) {\n"
      << "            const ef sj = ef_mul(num[j], ef_mul(iv, pre[j]));\n"
      << "            iv = ef_mul(iv, den[j]);\n"
      << "            if (j < gn) {\n"
      << "                for (int e = 0; e < 4; e++) A.out[(uint64_t)(4 * (g0 + j) + e) * A.ld + rl] = sj.c[e];\n"
      << "                total = ef_add(total, sj);\n"
      << "            }\n"
      << "        }\n"
      << "    }\n"
      << "    A.rowsum[4 * rl + 0] = total.c[0];\n"
      << "    A.rowsum[4 * rl + 1] = total.c[1];\n"
      << "    A.rowsum[4 * rl + 2] = total.c[2];\n"
      << "    A.rowsum[4 * rl + 3] = total.c[3];\n"
      << "}\n";
    return o.str();
}

std::string gen_perm_source(const ChipDesc &c, const std::string &fname) {
    const int nloc = (int)c.local.size();
    if (!nloc) return "";
    if (nloc > kJitLookupUnroll) return gen_perm_loop_source(c, fname);
    Gen g;
    const int batch = 1 << c.log_qd, nb = c.perm_w - 1;
    g.body << "    const ef alpha = ef{{A.alpha[0], A.alpha[1], A.alpha[2], A.alpha[3]}};\n";
    g.body << "    ef total = ef_zero();\n";
    // One inversion per row (Montgomery's trick): s_b = num_b / den_b = (num_b prefix_{b-1}) / prefix_b, so the
    // forward pass parks r_b = num_b prefix_{b-1} in LDS (each thread its own column of a [4 nb][256] word array:
    // no barriers, consecutive threads on consecutive banks) and the backward pass takes s_b = r_b iv, iv <- iv den_b
    // with the denominators in registers: the same EF products as parking num_b and prefix_{b-1} separately, half
    // the LDS (40 KB per workgroup at 10 batches: four workgroups per CU instead of two, and room beside the other
    // slots' kernels).  The register-only form needs 170 VGPRs (two waves); splitting the batches into several
    // inversions measured slower (profiles/r04_logup_open_ab.txt, r03_perm_group_sweep.txt).
    const bool lds = nb >= 2 && nb <= kPermLdsBatches;
    if (lds) {
        for (int b = 0; b < nb; b++) {
            g.body << "    ef num" << b << ", den" << b << ";\n";
            lookup_batch(g, c, b * batch, std::min(nloc, (b + 1) * batch), "alpha", "num" + std::to_string(b),
                         "den" + std::to_string(b));
            if (b == 0) {
                g.body << "    for (int e = 0; e < 4; e++) pl_lds[(0 + e) * 256 + threadIdx.x] = num0.c[e];\n"
                       << "    ef run = den0;\n";
            } else {
                g.body << "    {\n        const ef rb = ef_mul(num" << b << ", run);\n"
                       << "        for (int e = 0; e < 4; e++) pl_lds[(" << 4 * b
                       << " + e) * 256 + threadIdx.x] = rb.c[e];\n    }\n"
                       << "    run = ef_mul(run, den" << b << ");\n";
            }
        }
        g.body << "    ef iv = ef_inv(run);\n";
        for (int b = nb - 1; b >= 0; b--) {
            g.body << "    {\n        ef rr;\n"
                   << "        for (int e = 0; e < 4; e++) rr.c[e] = pl_lds[(" << 4 * b << " + e) * 256 + threadIdx.x];\n"
                   << "        const ef sb = ef_mul(rr, iv);\n";
            if (b > 0) g.body << "        iv = ef_mul(iv, den" << b << ");\n";
            for (int e = 0; e < 4; e++)
                g.body << "        A.out[(uint64_t)" << 4 * b + e << " * A.ld + rl] = sb.c[" << e << "];\n";
            g.body << "        total = ef_add(total, sb);\n    }\n";
        }
    } else {  // one batch, or more than kPermLdsBatches: prefix products in registers
        for (int b = 0; b < nb; b++) {
            g.body << "    ef num" << b << ", den" << b << ";\n";
            lookup_batch(g, c, b * batch, std::min(nloc, (b + 1) * batch), "alpha", "num" + std::to_string(b),
                         "den" + std::to_string(b));
        }
        g.body << "    const ef pre0 = den0;\n";
        for (int b = 1; b < nb; b++)
            g.body << "    const ef pre" << b << " = ef_mul(pre" << b - 1 << ", den" << b << ");\n";
        g.body << "    ef iv0 = ef_inv(pre" << nb - 1 << ");\n";
        for (int b = nb - 1; b > 0; b--) {
            g.body << "    const ef s" << b << " = ef_mul(num" << b << ", ef_mul(iv0, pre" << b - 1 << "));\n";
            g.body << "    iv0 = ef_mul(iv0, den" << b << ");\n";
        }
        g.body << "    const ef s0 = ef_mul(num0, iv0);\n";
        for (int b = 0; b < nb; b++) {
            for (int e = 0; e < 4; e++)
                g.body << "    A.out[(uint64_t)" << 4 * b + e << " * A.ld + rl] = s" << b << ".c[" << e << "];\n";
            g.body << "    total = ef_add(total, s" << b << ");\n";
        }
    }
    std::ostringstream o;
    o << "extern \"C\" __global__ void " << perm_bounds() << " " << fname << "(const ZkmPermJitArgs A) {\n"
      << (lds ? "    __shared__ uint32_t pl_lds[" + std::to_string(4 * nb) + " * 256];\n" : std::string())
      << "    const uint64_t rl = (uint64_t)blockIdx.x * 256 + threadIdx.x;\n"
      << "    if (rl >= A.ld) return;\n"
      << g.head.str() << g.pipelined(48)  // 48 -> 0.99 ms, 8 -> 1.37
      << "    A.rowsum[4 * rl + 0] = total.c[0];\n"
      << "    A.rowsum[4 * rl + 1] = total.c[1];\n"
      << "    A.rowsum[4 * rl + 2] = total.c[2];\n"
      << "    A.rowsum[4 * rl + 3] = total.c[3];\n"
      << "}\n";
    return o.str();
}

std::string chip_source(const ChipDesc &c) {
    std::ostringstream o;
    o << "typedef unsigned int uint32_t;\ntypedef unsigned long long uint64_t;\n"
      << kJitPrelude << "\nusing namespace kb;\n"
      << "#define POW(k) ef{{A.pows[4*(k)], A.pows[4*(k)+1], A.pows[4*(k)+2], A.pows[4*(k)+3]}}\n"
      << "#define BPOW(v) ef{{A.beta_pows[4*(v)], A.beta_pows[4*(v)+1], A.beta_pows[4*(v)+2], A.beta_pows[4*(v)+3]}}\n"
      << ((int)c.local.size() > kJitLookupUnroll ? kLoopHelpers : "")
      << gen_source(c, "zkm_quot_jit") << gen_perm_source(c, "zkm_perm_jit");
    return o.str();
}

}  // namespace

bool jit_enabled() {
    const char *e = getenv("ZKM_NO_JIT");
    return !(e && *e && *e != '0');
}

namespace {

uint64_t fnv1a(const std::string &s, uint64_t h = 1469598103934665603ull) {
    for (unsigned char ch : s) h = (h ^ ch) * 1099511628211ull;
    return h;
}

std::string cache_dir() {
    if (const char *e = getenv("ZKM_JIT_CACHE")) return std::string(e) == "off" ? std::string() : std::string(e);
    Dl_info info;
    if (!dladdr((void *)&fnv1a, &info) || !info.dli_fname) return std::string();
    std::string lib = info.dli_fname;
    const size_t slash = lib.rfind('/');
    return (slash == std::string::npos ? std::string(".") : lib.substr(0, slash)) + "/jit_cache";
}

std::mutex g_cache_mu;
std::unordered_map<uint64_t, std::vector<char>> g_cache;

bool read_file(const std::string &path, std::vector<char> &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return !out.empty();
}

void write_file_atomic(const std::string &dir, const std::string &name, const std::vector<char> &code) {
    mkdir(dir.c_str(), 0755);  // may already exist
    const std::string tmp = dir + "/." + name + "." + std::to_string(getpid()) + ".tmp";
    {
        std::ofstream f(tmp, std::ios::binary);
        if (!f) return;  // read-only tree: the in-memory cache still holds it
        f.write(code.data(), (std::streamsize)code.size());
        if (!f) { unlink(tmp.c_str()); return; }
    }
    if (rename(tmp.c_str(), (dir + "/" + name).c_str()) != 0) unlink(tmp.c_str());
}

std::vector<char> compile_source(const std::string &src, const std::string &name, const std::string &arch_name);

// the hiprtc options compile_source passes (after --offload-arch); the cache key is derived from this
// same list, so an option change can never load a code object built with the old options
const char *const kJitOpts[] = {"-O3", "-std=c++17"};

// everything besides the source that determines the code object: arch, options, hiprtc version
std::string toolchain_id(const std::string &arch_name) {
    int major = 0, minor = 0;
    hiprtcVersion(&major, &minor);
    std::string id = arch_name + "|hiprtc " + std::to_string(major) + "." + std::to_string(minor) + "|";
    for (const char *o : kJitOpts) id += std::string(o) + "|";
    return id;
}

// on-disk format: 8-byte magic, 8-byte FNV-1a of the code object, the code object; a file whose
// magic or checksum does not match is a cache miss (recompiled and rewritten), never loaded
const char kCoMagic[8] = {'Z', 'K', 'M', 'C', 'O', '2', 0, 0};

bool read_cached_code(const std::string &path, std::vector<char> &code) {
    std::vector<char> raw;
    if (!read_file(path, raw) || raw.size() <= 16 || memcmp(raw.data(), kCoMagic, 8) != 0) return false;
    uint64_t want;
    memcpy(&want, raw.data() + 8, 8);
    code.assign(raw.begin() + 16, raw.end());
    return fnv1a(std::string(code.begin(), code.end())) == want;
}

void write_cached_code(const std::string &dir, const std::string &name, const std::vector<char> &code) {
    std::vector<char> raw(kCoMagic, kCoMagic + 8);
    const uint64_t h = fnv1a(std::string(code.begin(), code.end()));
    raw.insert(raw.end(), (const char *)&h, (const char *)&h + 8);
    raw.insert(raw.end(), code.begin(), code.end());
    write_file_atomic(dir, name, raw);
}

}  // namespace

std::vector<char> jit_chip_code(const ChipDesc &c, const std::string &arch_name) {
    const std::string src = chip_source(c);
    const uint64_t key = fnv1a(src, fnv1a(toolchain_id(arch_name)));
    {
        std::lock_guard<std::mutex> g(g_cache_mu);
        auto it = g_cache.find(key);
        if (it != g_cache.end()) return it->second;
    }
    char kname[32];
    snprintf(kname, sizeof kname, "%016llx", (unsigned long long)key);
    const std::string dir = cache_dir(), fname = c.name + "-" + arch_name + "-" + kname + ".co";
    std::vector<char> code;
    if (dir.empty() || !read_cached_code(dir + "/" + fname, code)) {
        code = compile_source(src, c.name, arch_name);
        if (!dir.empty()) write_cached_code(dir, fname, code);
    } else if (getenv("ZKM_JIT_TOUCH")) {
        utime((dir + "/" + fname).c_str(), nullptr);  // the cache prefill prunes files it did not touch
    }
    std::lock_guard<std::mutex> g(g_cache_mu);
    g_cache[key] = code;
    return code;
}

namespace {

std::vector<char> compile_source(const std::string &src, const std::string &name, const std::string &arch_name) {
    if (const char *d = getenv("ZKM_JIT_DUMP")) {
        if (FILE *f = fopen((std::string(d) + "/" + name + ".hip").c_str(), "w")) {
            fputs(src.c_str(), f);
            fclose(f);
        }
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "quotient_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        throw HipError("hiprtcCreateProgram failed");
    std::string arch = "--offload-arch=" + arch_name;
    std::vector<const char *> opts = {arch.c_str()};
    for (const char *o : kJitOpts) opts.push_back(o);
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    if (rc != HIPRTC_SUCCESS) {
        size_t ls = 0;
        hiprtcGetProgramLogSize(prog, &ls);
        std::string log(ls + 1, '\0');
        hiprtcGetProgramLog(prog, &log[0]);
        hiprtcDestroyProgram(&prog);
        throw HipError("hiprtc compile failed for chip " + name + ": " + log.substr(0, 2000));
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    std::vector<char> code(cs);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    return code;
}

}  // namespace

namespace {

// cheap identity of everything chip_source reads, so a repeated setup (the compress stage sets up a
// program per proof, prover/src/lib.rs:807) neither regenerates the kernel source nor reloads the module
uint64_t chip_key(const ChipDesc &c, int device) {
    std::vector<uint32_t> w = {(uint32_t)device, (uint32_t)c.prep_w, (uint32_t)c.main_w, (uint32_t)c.scope,
                               (uint32_t)c.local_only, (uint32_t)c.log_qd, (uint32_t)c.n_main, (uint32_t)c.perm_w,
                               (uint32_t)c.n_constraints, (uint32_t)c.max_stack, (uint32_t)c.code.size()};
    w.insert(w.end(), c.code.begin(), c.code.end());
    auto vpc = [&](const VPC &v) {
        w.push_back((uint32_t)v.cols.size());
        w.insert(w.end(), v.cols.begin(), v.cols.end());
        w.insert(w.end(), v.weights.begin(), v.weights.end());
        w.push_back(v.constant);
    };
    w.push_back((uint32_t)c.local.size());
    for (const LookupDesc &l : c.local) {
        w.push_back(l.kind);
        w.push_back(l.scope);
        w.push_back(l.is_send);
        w.push_back((uint32_t)l.values.size());
        for (const VPC &v : l.values) vpc(v);
        vpc(l.mult);
    }
    const std::string bytes((const char *)w.data(), w.size() * 4);
    return fnv1a(bytes, fnv1a(c.name));
}

std::mutex g_loaded_mu;
std::unordered_map<uint64_t, JitKernel> g_loaded;  // loaded for the process lifetime

}  // namespace

// The returned kernel's module belongs to the process-wide cache (mod is left null, so a proving key's
// destructor does not unload it).
JitKernel jit_chip(const ChipDesc &c, int device) {
    const uint64_t key = chip_key(c, device);
    {
        std::lock_guard<std::mutex> g(g_loaded_mu);
        auto it = g_loaded.find(key);
        if (it != g_loaded.end()) return it->second;
    }
    JitKernel k;
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device));
    std::string arch = prop.gcnArchName;
    arch = arch.substr(0, arch.find(':'));  // "gfx950:sramecc+:xnack-" -> "gfx950"
    const std::vector<char> code = jit_chip_code(c, arch);
    hipModule_t mod = nullptr;
    HIP_CHECK(hipModuleLoadData(&mod, code.data()));
    HIP_CHECK(hipModuleGetFunction(&k.fn, mod, "zkm_quot_jit"));
    if (!c.local.empty()) HIP_CHECK(hipModuleGetFunction(&k.fn_perm, mod, "zkm_perm_jit"));
    k.ok = true;
    std::lock_guard<std::mutex> g(g_loaded_mu);
    auto ins = g_loaded.emplace(key, k);
    if (!ins.second) (void)hipModuleUnload(mod);  // another thread loaded the same chip meanwhile
    return ins.first->second;
}

void launch_quotient_jit(const JitKernel &k, const ZkmQuotJitArgs &a, hipStream_t s) {
    ZkmQuotJitArgs args = a;
    void *params[] = {&args};
    const unsigned grid = (unsigned)((a.q + 255) / 256);
    HIP_CHECK(hipModuleLaunchKernel(k.fn, grid, 1, 1, 256, 1, 1, 0, s, params, nullptr));
}

void launch_perm_jit(const JitKernel &k, const ZkmPermJitArgs &a, hipStream_t s) {
    ZkmPermJitArgs args = a;
    void *params[] = {&args};
    const unsigned grid = (unsigned)((a.ld + 255) / 256);
    HIP_CHECK(hipModuleLaunchKernel(k.fn_perm, grid, 1, 1, 256, 1, 1, 0, s, params, nullptr));
}

}  // namespace zkm

extern "C" int zkm_quotient_jit_compile(const uint32_t *blob, size_t nwords, uint64_t *code_bytes) {
    try {
        ARG_CHECK(blob && code_bytes, "null argument");
        const zkm::Machine m = zkm::parse_machine(blob, nwords);
        std::vector<std::future<size_t>> fut;  // chips compile concurrently (and fill the cache)
        for (const auto &c : m.chips)
            fut.push_back(std::async(std::launch::async, [&c] { return zkm::jit_chip_code(c, "gfx950").size(); }));
        uint64_t total = 0;
        for (auto &f : fut) total += f.get();
        *code_bytes = total;
        return 0;
    } catch (const std::exception &e) {
        return zkm::guard_status(e);
    }
}
