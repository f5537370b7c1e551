// MI355X shard prover: MachineProver::{setup, commit, open} behind the C ABI.
//
// Host-side orchestration follows the reference step by step:
//   StarkMachine::setup            crates/stark/src/machine.rs:332-439
//   CpuProver::commit              crates/stark/src/prover.rs:258-292
//   CpuProver::open                crates/stark/src/prover.rs:298-653
//   TwoAdicFriPcs::open + FRI      Plonky3 fork @faa24ca (not vendored); semantics pinned by the
//                                  verifier restatement crates/recursion/circuit/src/fri.rs:34-405
// Every O(N) step runs on the GPU (open_kernels.hip, ntt.hip, merkle.hip); the host keeps the
// Fiat-Shamir transcript (a few hundred Poseidon2 permutations) and assembles the proof.
#include <algorithm>
#include <tuple>
#include <array>
#include <cstring>
#include <future>
#include <numeric>
#include <optional>

#include "../../include/zkm_hip.h"
#include "chip.hpp"
#include "jit.hpp"
#include "internal.hpp"
#include "open_kernels.hpp"
#include "p2.cuh"
#include "prof.hpp"

namespace zkm {

using namespace kb;
using Digest = std::array<uint32_t, 8>;

int guard_status(const std::exception &e);
extern thread_local std::string g_last_error;

static const uint32_t CURVE_START[14] = {637514027u, 1595065213u, 1998064738u, 72333738u,  1211544370u,
                                         822986770u, 1518535784u, 1604177449u, 90440090u, 259343427u,
                                         140470264u, 1162099742u, 941559812u,  1064053343u};

// ------------------------------------------------------------------ host challenger (Montgomery)
struct Challenger {
    uint32_t st[16] = {0};
    uint32_t in[8] = {0};
    int nin = 0;
    uint32_t out[8] = {0};
    int nout = 0;
    void duplex() {
        for (int i = 0; i < nin; i++) st[i] = in[i];
        nin = 0;
        p2::permute(st);
        memcpy(out, st, 32);
        nout = 8;
    }
    void observe(uint32_t v) {
        nout = 0;
        in[nin++] = v;
        if (nin == 8) duplex();
    }
    void observe(const uint32_t *v, size_t n) { for (size_t i = 0; i < n; i++) observe(v[i]); }
    void observe_ef(const ef &e) { observe(e.c, 4); }
    uint32_t sample() {
        if (nin || !nout) duplex();
        return out[--nout];
    }
    ef sample_ef() {
        ef e;
        for (int i = 0; i < 4; i++) e.c[i] = sample();
        return e;
    }
    uint32_t sample_bits(int bits) { return from_mont(sample()) & ((1u << bits) - 1u); }
    void load(const zkm_challenger_t &c) {
        for (int i = 0; i < 16; i++) st[i] = to_mont(c.sponge_state[i]);
        nin = (int)c.num_inputs;
        nout = (int)c.num_outputs;
        ARG_CHECK(nin <= 8 && nout <= 8, "challenger buffers");
        for (int i = 0; i < 8; i++) { in[i] = to_mont(c.input_buffer[i]); out[i] = to_mont(c.output_buffer[i]); }
    }
    void store(zkm_challenger_t &c) const {
        for (int i = 0; i < 16; i++) c.sponge_state[i] = from_mont(st[i]);
        c.num_inputs = (uint32_t)nin;
        c.num_outputs = (uint32_t)nout;
        for (int i = 0; i < 8; i++) {
            c.input_buffer[i] = i < nin ? from_mont(in[i]) : 0u;
            c.output_buffer[i] = i < nout ? from_mont(out[i]) : 0u;
        }
    }
};

// ------------------------------------------------------------------ keys and shard data
// identity of a machine layout for commit/open: the blob words and the blowup (what commit reads)
static uint64_t machine_digest(const uint32_t *blob, size_t n, uint32_t log_blowup) {
    uint64_t h = 1469598103934665603ull ^ log_blowup;
    for (size_t i = 0; i < n; i++) h = (h ^ blob[i]) * 1099511628211ull;
    return h;
}

// zkm_machine: what MachineProver::commit needs and nothing else (no preprocessed data), so a
// caller whose commit receives no key (the trait's commit, prover.rs:111-115) does not have to
// guess one; zkm_open checks that the committed data and the key describe the same machine.
struct MachineHandle {
    Machine m;
    zkm_config_t cfg{};
    uint64_t digest = 0;
};

struct Pk {
    int device = 0;
    Machine m;
    zkm_config_t cfg{};
    uint64_t digest = 0;       // machine_digest of the blob it was set up from
    uint32_t commit[8];        // Montgomery
    uint32_t pc_start;         // Montgomery
    uint32_t gcs[14];          // Montgomery
    std::vector<int> trace_chip;
    std::vector<uint64_t> heights;
    std::vector<DBuf> traces;  // column-major natural (Montgomery)
    DTree tree;                // LDEs owned by tree.owned
    std::vector<DBuf> progs;   // flattened chip programs (device)
    std::vector<JitKernel> jit;  // per-chip specialised quotient kernels (jit.cpp); !ok -> interpreter
    ~Pk() {
        for (auto &k : jit)
            if (k.mod) (void)hipModuleUnload(k.mod);
    }
    int pk_index(int chip) const {
        for (size_t i = 0; i < trace_chip.size(); i++)
            if (trace_chip[i] == chip) return (int)i;
        return -1;
    }
};

struct MainData {
    uint64_t machine = 0;          // machine_digest of the machine it was committed under
    std::vector<int> chip;         // machine chip index, in commit order (height desc, name)
    std::vector<uint64_t> heights;
    std::vector<DBuf> store;       // one column-major natural buffer per height group
    std::vector<const uint32_t *> trace;  // chip i's columns inside its group's buffer
    DTree tree;
    std::vector<uint32_t> pv;      // canonical
};

static std::vector<int> sort_order(const std::vector<uint64_t> &h, const std::vector<std::string> &names) {
    std::vector<int> o(h.size());
    std::iota(o.begin(), o.end(), 0);
    std::stable_sort(o.begin(), o.end(), [&](int a, int b) {
        if (h[a] != h[b]) return h[a] > h[b];
        return names[a] < names[b];
    });
    return o;
}

// Bit-reversed coset LDE with blowup 2^lb of src (N x W) into dst (column stride N << lb): row i holds
// p(shift * w_{2^lb N}^{rev(i)}).  The blowup-2 kernels give rows [0, 2N) directly; for blowup 4, rows
// [2N, 4N) are the blowup-2 LDE with shift * w_{4N} (rev_{4N}(2N + j) = 2 rev_{2N}(j) + 1), so two
// passes fill the two halves of every column directly.
static void lde_into(Ctx &c, const DMat &src, uint32_t shift, bool bitrev_in, int lb, uint32_t *dst, hipStream_t s) {
    const uint64_t N = src.height, W = src.width;
    if (!W) return;
    ARG_CHECK(lb == 1 || lb == 2, "log_blowup must be 1 or 2");
    if (lb == 1) {
        DMat d{dst, 2 * N, W};
        if (bitrev_in) lde_batch_bitrev_in(c, src, shift, d, s);
        else lde_batch(c, src, shift, d, s);
        return;
    }
    // each blowup-2 pass writes its half of every 4N-row column in place (column stride 4N); natural
    // input shares the inverse transform between the halves (ZKM_LDE4_SHARED=0: two full passes)
    static const bool shared = [] {
        const char *e = getenv("ZKM_LDE4_SHARED");
        return !(e && e[0] == '0');
    }();
    if (!bitrev_in && shared) {
        lde_batch_blowup4(c, src, shift, mul(shift, two_adic_gen(ilog2(N) + 2)), dst, s);
        return;
    }
    for (int half = 0; half < 2; half++) {
        const uint32_t sh = half ? mul(shift, two_adic_gen(ilog2(N) + 2)) : shift;
        if (bitrev_in) lde_batch_bitrev_in_strided(c, src, sh, dst + half * 2 * N, 4 * N, s);
        else lde_batch_strided(c, src, sh, dst + half * 2 * N, 4 * N, s);
    }
}

static void add_lde(Ctx &c, DTree &t, const DMat &src, uint32_t shift, bool bitrev_in, int lb, hipStream_t s) {
    const uint64_t H = src.height << lb;
    t.owned.emplace_back(H * (src.width ? src.width : 1), s);
    lde_into(c, src, shift, bitrev_in, lb, t.owned.back().p, s);
    t.mats.push_back(DMat{t.owned.back().p, H, src.width});
}

// One LDE launch sequence for several same-height matrices whose columns sit side by side in `src`
// (column stride N): the evaluations go to one buffer owned by the tree, and each matrix gets its
// sub-view (returned in order; the caller places them in the tree's commit order).  Same-height
// chips of a shard thus share launches instead of taking a handful each.
static std::vector<DMat> lde_group(Ctx &c, DTree &t, const uint32_t *src, uint64_t N, const std::vector<uint64_t> &widths,
                                   uint32_t shift, bool bitrev_in, int lb, hipStream_t s) {
    const uint64_t W = std::accumulate(widths.begin(), widths.end(), (uint64_t)0), H = N << lb;
    t.owned.emplace_back(H * (W ? W : 1), s);
    uint32_t *dst = t.owned.back().p;
    lde_into(c, DMat{const_cast<uint32_t *>(src), N, W}, shift, bitrev_in, lb, dst, s);
    std::vector<DMat> v;
    uint64_t off = 0;
    for (uint64_t w : widths) {
        v.push_back(DMat{dst + off * H, H, w});
        off += w;
    }
    return v;
}

// ------------------------------------------------------------------ proof object + bincode
struct ChipOpen {
    std::vector<ef> prep_l, prep_n, main_l, main_n, perm_l, perm_n;
    std::vector<ef> quot;  // nq * 4
    uint32_t gcs[14];
    ef lcs;
    uint64_t log_degree;
};
struct BatchOpen {
    std::vector<std::vector<uint32_t>> vals;
    std::vector<Digest> path;
};
struct Step {
    ef sib;
    std::vector<Digest> path;
};
struct Query {
    std::vector<BatchOpen> input;
    std::vector<Step> steps;
};
struct Proof {
    Digest main_c, perm_c, quot_c;
    std::vector<ChipOpen> chips;
    std::vector<Digest> fri_commits;
    std::vector<Query> queries;
    ef final_poly;
    uint32_t pow;
    std::vector<std::string> names;
    std::vector<uint32_t> pv;  // canonical
};

struct Writer {
    std::vector<uint8_t> b;
    bool mont;
    void put(const void *p, size_t n) { b.insert(b.end(), (const uint8_t *)p, (const uint8_t *)p + n); }
    void u64(uint64_t v) { put(&v, 8); }
    void f(uint32_t mont_val) { uint32_t v = mont ? mont_val : from_mont(mont_val); put(&v, 4); }
    void fc(uint32_t canon) { uint32_t v = mont ? to_mont(canon) : canon; put(&v, 4); }
    void e(const ef &x) { for (int i = 0; i < 4; i++) f(x.c[i]); }
    void d(const Digest &x) { for (int i = 0; i < 8; i++) f(x[i]); }
    void ev(const std::vector<ef> &v) { u64(v.size()); for (auto &x : v) e(x); }
    void dv(const std::vector<Digest> &v) { u64(v.size()); for (auto &x : v) d(x); }
};

// bincode-1 (fixint, LE) layout of ShardProof (crates/stark/src/types.rs:77-83); chip_ordering
// sorted by index; field elements canonical unless cfg.proof_montgomery.
static std::vector<uint8_t> serialize(const Proof &p, bool mont) {
    Writer w{{}, mont};
    w.b.reserve(4u << 20);  // shard proofs are 0.05-3 MB: one allocation instead of ~20 regrowths
    w.d(p.main_c); w.d(p.perm_c); w.d(p.quot_c);
    w.u64(p.chips.size());
    for (auto &c : p.chips) {
        w.ev(c.prep_l); w.ev(c.prep_n); w.ev(c.main_l); w.ev(c.main_n); w.ev(c.perm_l); w.ev(c.perm_n);
        w.u64(c.quot.size() / 4);
        for (size_t j = 0; j < c.quot.size() / 4; j++) {
            w.u64(4);
            for (int e = 0; e < 4; e++) w.e(c.quot[4 * j + e]);
        }
        for (int j = 0; j < 14; j++) w.f(c.gcs[j]);
        w.e(c.lcs);
        w.u64(c.log_degree);
    }
    w.dv(p.fri_commits);
    w.u64(p.queries.size());
    for (auto &q : p.queries) {
        w.u64(q.input.size());
        for (auto &bo : q.input) {
            w.u64(bo.vals.size());
            for (auto &row : bo.vals) { w.u64(row.size()); for (uint32_t x : row) w.f(x); }
            w.dv(bo.path);
        }
        w.u64(q.steps.size());
        for (auto &st : q.steps) { w.e(st.sib); w.dv(st.path); }
    }
    w.e(p.final_poly);
    w.f(p.pow);
    w.u64(p.names.size());
    for (size_t i = 0; i < p.names.size(); i++) {
        w.u64(p.names[i].size());
        w.put(p.names[i].data(), p.names[i].size());
        w.u64(i);
    }
    w.u64(p.pv.size());
    for (uint32_t x : p.pv) w.fc(x);
    return std::move(w.b);
}

static Digest dig(const uint32_t *r) { Digest d; memcpy(d.data(), r, 32); return d; }

// ------------------------------------------------------------------ open
struct OpenReq {
    int round, mat;
    int npts;
    ef pts[2];
    std::vector<ef> vals[2];
};

static std::vector<uint8_t> open_shard(Ctx &c, const Pk &pk, MainData &md, Challenger &ch, hipStream_t s) {
    const Machine &m = pk.m;
    const int lb = (int)pk.cfg.log_blowup;
    const int n = (int)md.chip.size();
    Proof proof;
    proof.main_c = dig(md.tree.root);
    for (int i = 0; i < n; i++) proof.names.push_back(m.chips[md.chip[i]].name);
    proof.pv = md.pv;

    // observe public values then the main commitment (prover.rs:322-323)
    ARG_CHECK((int)md.pv.size() >= m.num_pv, "fewer public values than num_pv_elts");
    for (int i = 0; i < m.num_pv; i++) ch.observe(to_mont(md.pv[i]));
    ch.observe(md.tree.root, 8);
    const ef perm_alpha = ch.sample_ef(), perm_beta = ch.sample_ef();
    // beta^(j+1) for every lookup arity (rlc = alpha + kind + sum_j beta^(j+1) v_j, permutation.rs:48-57)
    size_t max_arity = 1;
    for (auto &cd : m.chips)
        for (auto &l : cd.local) max_arity = std::max(max_arity, l.values.size());
    std::vector<uint32_t> bpow(4 * max_arity);
    {
        ef b = perm_beta;
        for (size_t j = 0; j < max_arity; j++) { memcpy(&bpow[4 * j], b.c, 16); b = ef_mul(b, perm_beta); }
    }
    DBuf d_bpow(bpow.size(), s);
    HIP_CHECK(hipMemcpyAsync(d_bpow.p, bpow.data(), bpow.size() * 4, hipMemcpyHostToDevice, s));

    PROF("open_total", s, 0);
    // ---- permutation traces (prover.rs:337-365) ----
    proof.chips.resize(n);
    // chips come in commit order (height desc), so same-height chips are adjacent: one perm-trace
    // buffer per height group, LDE'd together once every chip of the group has its trace
    std::vector<const uint32_t *> perm_traces(n);
    std::vector<DBuf> perm_store;
    std::vector<int> grp_end(n);
    for (int a = 0, b; a < n; a = b) {
        uint64_t W = 0;
        for (b = a; b < n && md.heights[b] == md.heights[a]; b++) W += 4 * (uint64_t)m.chips[md.chip[b]].perm_w;
        perm_store.emplace_back(md.heights[a] * (W ? W : 1), s);
        uint64_t off = 0;
        for (int k = a; k < b; k++) {
            perm_traces[k] = perm_store.back().p + off * md.heights[a];
            off += 4 * (uint64_t)m.chips[md.chip[k]].perm_w;
            grp_end[k] = b;
        }
    }
    DTree perm_tree;
    // each chip's local sum (last row of the last perm column) and global sum (last 14 main columns of
    // a Global-scope chip) are read back asynchronously; tree_build below synchronises the stream
    std::vector<uint32_t> sums_host(18 * (size_t)n + 1, 0);
    for (int i = 0; i < n; i++) {
        const ChipDesc &cd = m.chips[md.chip[i]];
        const uint64_t N = md.heights[i];
        const int pki = pk.pk_index(md.chip[i]);
        ARG_CHECK(pki < 0 || pk.heights[pki] == N, "preprocessed and main heights differ");
        ChipOpen &co = proof.chips[i];
        co.log_degree = (uint64_t)ilog2(N);
        co.lcs = ef_zero();
        const int pw = cd.perm_w;
        if (pw) {
            DBuf rowsum(4 * N, s);
            PermArgs a{pk.progs[md.chip[i]].p, md.trace[i], pki >= 0 ? pk.traces[pki].p : nullptr, N, perm_alpha,
                       d_bpow.p, 1 << cd.log_qd, pw - 1, const_cast<uint32_t *>(perm_traces[i]), rowsum.p};
            {
                PROF("perm_trace", s, 4.0 * N * (cd.main_w + cd.prep_w) + 16.0 * N * (pw + 2));
                const JitKernel &jk = pk.jit[md.chip[i]];
                if (jk.fn_perm) {
                    ZkmPermJitArgs ja{};
                    ja.main = a.main; ja.prep = a.prep; ja.beta_pows = a.beta_pows; ja.out = a.out;
                    ja.rowsum = a.rowsum; ja.ld = N; ja.prog = a.prog;
                    memcpy(ja.alpha, a.alpha.c, 16);
                    launch_perm_jit(jk, ja, s);
                }
                launch_perm_trace(a, s, jk.fn_perm != nullptr);
            }
            // the 4 words are rows N-1 of 4 columns N apart: one strided 2D copy
            HIP_CHECK(hipMemcpy2DAsync(&sums_host[18 * i], 4, perm_traces[i] + (uint64_t)(4 * (pw - 1)) * N + N - 1,
                                       N * 4, 4, 4, hipMemcpyDeviceToHost, s));
        }
        if (cd.scope == 1) {
            HIP_CHECK(hipMemcpy2DAsync(&sums_host[18 * i + 4], 4, md.trace[i] + (uint64_t)(cd.main_w - 14) * N + N - 1,
                                       N * 4, 4, 14, hipMemcpyDeviceToHost, s));
        } else {
            for (int k = 0; k < 14; k++) co.gcs[k] = to_mont(CURVE_START[k]);
        }
        if (grp_end[i] == i + 1) {  // last chip of its height group: LDE the group
            int a = i;
            while (a > 0 && md.heights[a - 1] == N) a--;
            std::vector<uint64_t> ws;
            for (int k = a; k <= i; k++) ws.push_back(4 * (uint64_t)m.chips[md.chip[k]].perm_w);
            for (const DMat &v : lde_group(c, perm_tree, perm_traces[a], N, ws, to_mont(GENERATOR), false, lb, s))
                perm_tree.mats.push_back(v);
        }
    }
    tree_build(perm_tree, s);  // synchronises the stream: sums_host is filled
    for (int i = 0; i < n; i++) {
        const ChipDesc &cd = m.chips[md.chip[i]];
        if (cd.perm_w) proof.chips[i].lcs = ef{{sums_host[18 * i], sums_host[18 * i + 1], sums_host[18 * i + 2],
                                                sums_host[18 * i + 3]}};
        if (cd.scope == 1) memcpy(proof.chips[i].gcs, &sums_host[18 * i + 4], 14 * 4);
    }
    proof.perm_c = dig(perm_tree.root);
    ch.observe(perm_tree.root, 8);
    for (int i = 0; i < n; i++) {
        ch.observe_ef(proof.chips[i].lcs);
        ch.observe(proof.chips[i].gcs, 14);
    }
    const ef alpha = ch.sample_ef();

    // ---- quotient values, split, commit (prover.rs:415-498) ----
    std::vector<uint32_t> pv_mont(md.pv.size() + 1, 0);
    for (size_t k = 0; k < md.pv.size(); k++) pv_mont[k] = to_mont(md.pv[k]);
    DBuf d_pv(pv_mont.size(), s);
    HIP_CHECK(hipMemcpyAsync(d_pv.p, pv_mont.data(), pv_mont.size() * 4, hipMemcpyHostToDevice, s));
    DTree q_tree;
    // Quotient chunks grouped like the perm traces, by (height, log_qd): in a group of g chips, chunk
    // j of the group's k-th chip is columns 4k..4k+3 of block j (block stride 4gN), so every chunk j
    // of the group is one bit-reversed-input LDE with the shared shift (3 w^j)^-1.
    std::vector<DBuf> q_store;
    std::vector<std::vector<const uint32_t *>> q_ptr(n);
    std::vector<std::vector<DMat>> q_view(n);
    std::vector<uint64_t> q_cstride(n);
    std::vector<int> q_first(n);
    for (int a = 0, b; a < n; a = b) {
        const int lqd = m.chips[md.chip[a]].log_qd;
        for (b = a; b < n && md.heights[b] == md.heights[a] && m.chips[md.chip[b]].log_qd == lqd; b++) {}
        const uint64_t N = md.heights[a], T = 4 * (uint64_t)(b - a);
        q_store.emplace_back(((uint64_t)1 << lqd) * T * N, s);
        for (int k = a; k < b; k++) {
            q_first[k] = a;
            q_cstride[k] = T * N;
            for (int j = 0; j < (1 << lqd); j++) q_ptr[k].push_back(q_store.back().p + j * T * N + 4 * (uint64_t)(k - a) * N);
        }
    }
    std::vector<int> chunk_chip;  // chip of each quotient chunk
    // alpha^(n-1-k) per constraint k of every chip (folder.rs:79-102, powers reversed prover.rs:453-456),
    // one upload for the whole shard
    std::vector<uint64_t> pows_off(n + 1, 0);
    for (int i = 0; i < n; i++) pows_off[i + 1] = pows_off[i] + 4 * ((uint64_t)m.chips[md.chip[i]].n_constraints + 1);
    std::vector<uint32_t> pows_all(pows_off[n] + 1, 0);
    for (int i = 0; i < n; i++) {
        const int nc = m.chips[md.chip[i]].n_constraints;
        ef a = ef_one();
        for (int k = nc - 1; k >= 0; k--) {
            memcpy(&pows_all[pows_off[i] + 4 * k], a.c, 16);
            a = ef_mul(a, alpha);
        }
    }
    DBuf d_pows_all(pows_all.size(), s);
    HIP_CHECK(hipMemcpyAsync(d_pows_all.p, pows_all.data(), pows_all.size() * 4, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));  // pows_all (pageable) has been read
    for (int i = 0; i < n; i++) {
        const ChipDesc &cd = m.chips[md.chip[i]];
        const uint64_t N = md.heights[i];
        const int logN = ilog2(N), lqd = cd.log_qd;
        ARG_CHECK(lqd <= lb, "log_quotient_degree > log_blowup is not supported (Plonky3 asserts too)");
        const uint64_t Q = N << lqd;
        const uint32_t *d_pows = d_pows_all.p + pows_off[i];
        const int pki = pk.pk_index(md.chip[i]);
        QuotArgs qa{};
        qa.prog = pk.progs[md.chip[i]].p;
        qa.main = md.tree.mats[i].d;
        qa.prep = pki >= 0 ? pk.tree.mats[pki].d : nullptr;
        qa.perm = perm_tree.mats[i].d;
        qa.ld = N << lb;  // the quotient domain's Q = N 2^lqd points are the first Q bit-reversed LDE rows
        qa.n = N; qa.q = Q; qa.log_n = logN; qa.log_q = logN + lqd; qa.step = 1 << lqd;
        qa.tw = c.tw_fwd;
        qa.gen = to_mont(GENERATOR);
        qa.gen_pow_n = pow(qa.gen, N);
        qa.wn_inv = inv(two_adic_gen(logN));
        qa.pv = d_pv.p;
        qa.pows = d_pows;
        qa.alpha_p = perm_alpha; qa.beta_pows = d_bpow.p; qa.lcs = proof.chips[i].lcs;
        memcpy(qa.gcs, proof.chips[i].gcs, sizeof qa.gcs);
        qa.batch = 1 << lqd; qa.perm_w = cd.perm_w; qa.global = cd.scope == 1; qa.main_w = cd.main_w;
        qa.chunks = const_cast<uint32_t *>(q_ptr[i][0]);
        qa.cstride = q_cstride[i];
        qa.n_slots = cd.n_slots;
        {
            PROF("quotient", s, 8.0 * Q * (cd.main_w + cd.prep_w + 4 * cd.perm_w) + 16.0 * Q);
            const JitKernel &jk = pk.jit[md.chip[i]];
            if (jk.ok) {
                ZkmQuotJitArgs ja{};
                ja.main = qa.main; ja.prep = qa.prep; ja.perm = qa.perm; ja.pv = qa.pv; ja.pows = qa.pows;
                ja.beta_pows = qa.beta_pows; ja.tw = qa.tw; ja.chunks = qa.chunks; ja.cstride = qa.cstride;
                ja.ld = qa.ld; ja.n = qa.n; ja.q = qa.q; ja.log_n = qa.log_n; ja.log_q = qa.log_q; ja.step = qa.step;
                ja.gen = qa.gen; ja.gen_pow_n = qa.gen_pow_n; ja.wn_inv = qa.wn_inv; ja.prog = qa.prog;
                memcpy(ja.alpha_p, qa.alpha_p.c, 16); memcpy(ja.lcs, qa.lcs.c, 16); memcpy(ja.gcs, qa.gcs, sizeof ja.gcs);
                launch_quotient_jit(jk, ja, s);
            } else {
                launch_quotient(qa, s);
            }
        }
        if (i + 1 == n || q_first[i + 1] != q_first[i]) {  // last chip of its group: LDE the group's chunks
            const int a = q_first[i];
            const uint32_t wq = two_adic_gen(logN + lqd);
            const std::vector<uint64_t> ws(i - a + 1, 4);
            for (int j = 0; j < (1 << lqd); j++) {
                std::vector<DMat> v = lde_group(c, q_tree, q_ptr[a][j], N, ws, inv(pow(wq, (uint64_t)j)), true, lb, s);
                for (int k = a; k <= i; k++) q_view[k].push_back(v[k - a]);
            }
        }
    }
    for (int i = 0; i < n; i++)
        for (const DMat &v : q_view[i]) {
            q_tree.mats.push_back(v);
            chunk_chip.push_back(i);
        }
    tree_build(q_tree, s);
    proof.quot_c = dig(q_tree.root);
    ch.observe(q_tree.root, 8);
    const ef zeta = ch.sample_ef();

    // ---- opening points (prover.rs:503-544) ----
    const DTree *trees[4] = {&pk.tree, &md.tree, &perm_tree, &q_tree};
    std::vector<OpenReq> req;
    for (size_t t = 0; t < pk.trace_chip.size(); t++) {
        OpenReq r{0, (int)t, 1, {zeta, zeta}, {}};
        if (!m.chips[pk.trace_chip[t]].local_only) { r.pts[1] = ef_mul_base(zeta, two_adic_gen(ilog2(pk.heights[t]))); r.npts = 2; }
        req.push_back(r);
    }
    for (int i = 0; i < n; i++) {
        OpenReq r{1, i, 1, {zeta, zeta}, {}};
        if (!m.chips[md.chip[i]].local_only) { r.pts[1] = ef_mul_base(zeta, two_adic_gen(ilog2(md.heights[i]))); r.npts = 2; }
        req.push_back(r);
    }
    for (int i = 0; i < n; i++) req.push_back(OpenReq{2, i, 2, {zeta, ef_mul_base(zeta, two_adic_gen(ilog2(md.heights[i])))}, {}});
    for (size_t j = 0; j < chunk_chip.size(); j++) req.push_back(OpenReq{3, (int)j, 1, {zeta, zeta}, {}});

    // ---- opened values by barycentric evaluation over the trace domain ----
    //   p(z) = ((z/s)^N - 1)/N * sum_j y_j w^j / (z/s - w^j); next point g z uses y_{j+1}.
    // All dot products are launched back to back and read back with one copy.
    {
        // row segments per column chunk (k_open_dot grid: nseg x ceil(W / OPEN_CB)), sized per request
        struct Pend { OpenReq *r; const uint32_t *ybase; uint64_t N, W; bool bitrev; uint32_t shift; uint64_t coff, poff; ef pre; int nseg; };
        std::vector<Pend> pend;
        uint64_t ncols_all = 0, nparts = 0;
        for (auto &r : req) {
            Pend q{&r, nullptr, 0, 0, false, ONE, 0, 0, ef_zero(), 1};
            if (r.round == 0) { q.ybase = pk.traces[r.mat].p; q.N = pk.heights[r.mat]; q.W = m.chips[pk.trace_chip[r.mat]].prep_w; }
            else if (r.round == 1) { q.ybase = md.trace[r.mat]; q.N = md.heights[r.mat]; q.W = m.chips[md.chip[r.mat]].main_w; }
            else if (r.round == 2) { q.ybase = perm_traces[r.mat]; q.N = md.heights[r.mat]; q.W = 4 * m.chips[md.chip[r.mat]].perm_w; }
            else {
                const int ci = chunk_chip[r.mat];
                int j = 0;
                for (int k = 0; k < r.mat; k++) if (chunk_chip[k] == ci) j++;
                q.N = md.heights[ci];
                const int lqd = m.chips[md.chip[ci]].log_qd;
                q.ybase = q_ptr[ci][j];
                q.W = 4;
                q.bitrev = true;
                q.shift = mul(to_mont(GENERATOR), pow(two_adic_gen(ilog2(q.N) + lqd), (uint64_t)j));
            }
            r.vals[0].assign(q.W, ef_zero());
            r.vals[1].assign(q.W, ef_zero());
            const ef zs = ef_mul_base(zeta, inv(q.shift));
            q.pre = ef_mul_base(ef_sub(ef_pow(zs, q.N), ef_one()), inv(to_mont((uint32_t)(q.N % P))));
            if (q.W) pend.push_back(q);
        }
        // Matrices that share the height, the evaluation domain (shift) and the number of points share one
        // weight table and one k_open_dot launch over all their columns (every chip of a height group:
        // preprocessed, main and LogUp traces; quotient chunk j of every chip of a (height, log_qd));
        // each group's columns are contiguous in the column table and its partial sums in `part`.
        auto key = [](const Pend &q) { return std::make_tuple(q.N, q.bitrev, q.shift, q.r->npts); };
        std::stable_sort(pend.begin(), pend.end(), [&](const Pend &a, const Pend &b) { return key(a) < key(b); });
        struct Group { size_t first, last; uint64_t coff, poff, W; int nseg; };
        std::vector<Group> groups;
        for (size_t i = 0; i < pend.size(); i++) {
            if (groups.empty() || key(pend[groups.back().first]) != key(pend[i])) groups.push_back({i, i, 0, 0, 0, 1});
            groups.back().last = i;
            groups.back().W += pend[i].W;
        }
        for (auto &g : groups) {
            g.coff = ncols_all;
            g.poff = nparts;
            g.nseg = 1;  // launch_open_dot reduces its row segments on the device
            for (size_t i = g.first; i <= g.last; i++) {
                Pend &q = pend[i];
                q.coff = ncols_all;
                q.nseg = g.nseg;
                q.poff = g.poff + (q.coff - g.coff) * (uint64_t)g.nseg * 8;
                ncols_all += q.W;
            }
            nparts += g.W * (uint64_t)g.nseg * 8;
        }
        std::vector<uint64_t> cols(ncols_all + 1);
        for (auto &q : pend)
            for (uint64_t k = 0; k < q.W; k++) cols[q.coff + k] = (uint64_t)(uintptr_t)(q.ybase + k * q.N);
        DBuf dcols(2 * cols.size(), s), part(nparts + 1, s);
        HIP_CHECK(hipMemcpyAsync(dcols.p, cols.data(), cols.size() * 8, hipMemcpyHostToDevice, s));
        // every group in one launch per kernel kind (blockIdx.z = group): the short chips' and the quotient
        // chunks' groups run beside each other instead of as a chain of latency-bound launches
        std::vector<OpenGroup> ogs;
        double open_bytes = 0;
        for (auto &g : groups) {
            const Pend &q = pend[g.first];
            // barycentric weights w^j / (zeta' - w^j): traces in natural row order (shift 1 after the
            // zeta / shift substitution), quotient chunks bit-reversed; generated by the kernel itself
            const OpenWeights w{q.bitrev ? ef_mul_base(zeta, inv(q.shift)) : zeta, ONE, c.tw_fwd, ilog2(q.N),
                                q.bitrev ? 1 : 0, 1};
            ogs.push_back(OpenGroup{(const uint64_t *)dcols.p + g.coff, q.N, w, (uint32_t)g.W, 0, 0, 0,
                                    q.r->npts == 2 ? 1 : 0, 0, nullptr, part.p + g.poff});
            open_bytes += 4.0 * q.N * g.W;
        }
        {
            PROF("open_eval", s, open_bytes);
            launch_open_dot_groups(ogs, s);  // ogs lives to the synchronisation below
        }
        std::vector<uint32_t> hp(nparts + 1);
        HIP_CHECK(hipMemcpyAsync(hp.data(), part.p, nparts * 4, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        for (auto &q : pend)
            for (uint64_t k = 0; k < q.W; k++) {
                ef a0 = ef_zero(), a1 = ef_zero();
                for (int sg = 0; sg < q.nseg; sg++) {
                    const uint32_t *x = &hp[q.poff + (k * q.nseg + sg) * 8];
                    a0 = ef_add(a0, ef{{x[0], x[1], x[2], x[3]}});
                    a1 = ef_add(a1, ef{{x[4], x[5], x[6], x[7]}});
                }
                q.r->vals[0][k] = ef_mul(q.pre, a0);
                q.r->vals[1][k] = ef_mul(q.pre, a1);  // (g z)^N = z^N for the trace-domain generator g
            }
    }

    // ---- PCS open: FRI alpha, reduced openings (fri.rs:71-215 semantics) ----
    const ef fri_alpha = ch.sample_ef();
    int log_max = 0;
    for (auto *t : trees) log_max = std::max(log_max, t->log_max);
    std::vector<DBuf> ro(32);
    std::vector<int> pow_cnt(32, 0);
    {
        // group (round, mat) by LDE height, in global order
        struct Item { const DMat *mat; const OpenReq *r; };
        std::vector<std::vector<Item>> by_h(32);
        for (auto &r : req) {
            const DMat *mm = &trees[r.round]->mats[r.mat];
            by_h[ilog2(mm->height)].push_back(Item{mm, &r});
        }
        uint64_t max_w = 1;
        for (auto &r : req) max_w = std::max<uint64_t>(max_w, trees[r.round]->mats[r.mat].width);
        std::vector<uint32_t> apow(4 * max_w);
        {
            ef a = ef_one();
            for (uint64_t k = 0; k < max_w; k++) { memcpy(&apow[4 * k], a.c, 16); a = ef_mul(a, fri_alpha); }
        }
        DBuf d_apow(apow.size(), s);
        HIP_CHECK(hipMemcpyAsync(d_apow.p, apow.data(), apow.size() * 4, hipMemcpyHostToDevice, s));
        auto alpha_pow = [&](uint64_t e) { return ef_pow(fri_alpha, e); };
        // the per-height column tables and descriptors are pageable host memory read by async copies:
        // they live until the one synchronisation after the loop
        std::vector<std::vector<uint64_t>> keep_cols;
        std::vector<std::vector<uint32_t>> keep_desc;
        for (int lh = 0; lh < 32; lh++) {
            if (by_h[lh].empty()) continue;
            const uint64_t H = 1ull << lh;
            const uint64_t N = H >> lb;
            ro[lh] = DBuf(4 * H, s);  // written whole by this height's one k_fri_reduce
            // the denominators 1/(z - 3 w_H^rev(i)) for z = zeta and zeta * w_N are inverted in the kernel
            const ef znext = ef_mul_base(zeta, two_adic_gen(ilog2(N)));
            bool need1 = false;
            keep_cols.emplace_back();
            keep_desc.emplace_back();
            std::vector<uint64_t> &cols = keep_cols.back();
            std::vector<uint32_t> &desc = keep_desc.back();
            for (auto &it : by_h[lh]) {
                const uint64_t W = it.mat->width;
                desc.push_back((uint32_t)W);
                desc.push_back((uint32_t)cols.size());
                desc.push_back((uint32_t)it.r->npts);
                for (uint64_t k = 0; k < W; k++) cols.push_back((uint64_t)(uintptr_t)(it.mat->d + k * it.mat->height));
                for (int p = 0; p < it.r->npts; p++) {
                    // offset alpha^pow; A = alpha^pow, B = alpha^pow * sum_c alpha^c p_c(z)
                    const ef ao = alpha_pow((uint64_t)pow_cnt[lh]);
                    ef sz = ef_zero();
                    ef ac = ef_one();
                    for (uint64_t k = 0; k < W; k++) { sz = ef_add(sz, ef_mul(ac, it.r->vals[p][k])); ac = ef_mul(ac, fri_alpha); }
                    const ef B = ef_mul(ao, sz);
                    const bool is_next = p == 1;
                    ARG_CHECK(!is_next || ef_eq(it.r->pts[1], znext), "unexpected opening point");
                    if (is_next) need1 = true;
                    desc.push_back(is_next ? 1u : 0u);
                    for (int e = 0; e < 4; e++) desc.push_back(ao.c[e]);
                    for (int e = 0; e < 4; e++) desc.push_back(B.c[e]);
                    pow_cnt[lh] += (int)W;
                }
            }
            DBuf dcols(2 * cols.size() + 2, s), ddesc(desc.size() + 1, s);
            if (!cols.empty()) HIP_CHECK(hipMemcpyAsync(dcols.p, cols.data(), cols.size() * 8, hipMemcpyHostToDevice, s));
            HIP_CHECK(hipMemcpyAsync(ddesc.p, desc.data(), desc.size() * 4, hipMemcpyHostToDevice, s));
            ReduceArgs ra{(const uint64_t *)dcols.p, ddesc.p, (uint32_t)by_h[lh].size(), d_apow.p, zeta, znext,
                          need1 ? 1 : 0, to_mont(GENERATOR), c.tw_fwd, ilog2(H), ro[lh].p, H};
            { PROF("fri_reduce", s, 4.0 * H * cols.size() + 16.0 * H); launch_fri_reduce(ra, s); }
        }
        HIP_CHECK(hipStreamSynchronize(s));  // keep_cols / keep_desc / apow have been read
    }

    // ---- FRI commit phase ----
    const int nrounds = log_max - lb;
    std::vector<DTree> ftrees(std::max(nrounds, 0));
    DBuf cur;
    uint64_t cur_n = 1ull << log_max;
    // round 0 folds the tallest height's reduced openings themselves (nothing else reads them): no 2^(L+1) x 16 B
    // device copy (a 134 MB blit per 2^22 shard)
    ARG_CHECK(ro[log_max].p, "no reduced openings at the tallest height");
    cur = std::move(ro[log_max]);
    // the commit phase only (the scope ends after the readback below, before the PoW)
    std::optional<ProfScope> fri_prof;
    fri_prof.emplace("fri_commit_phase", s, 0);
    // transcript on the device for the whole phase: no host round trip per round
    DBuf dchal_buf((sizeof(DevChallenger) + 3) / 4, s), droots(8 * std::max(nrounds, 1), s),
        dfargs(8 * std::max(nrounds, 1), s);
    DevChallenger hc{};
    memcpy(hc.st, ch.st, 64);
    memcpy(hc.in, ch.in, 32);
    memcpy(hc.out, ch.out, 32);
    hc.nin = (uint32_t)ch.nin;
    hc.nout = (uint32_t)ch.nout;
    DevChallenger *dchal = reinterpret_cast<DevChallenger *>(dchal_buf.p);
    HIP_CHECK(hipMemcpyAsync(dchal, &hc, sizeof hc, hipMemcpyHostToDevice, s));
    // per round: the tree over the round's leaves, whose top launch also runs the transcript step (root
    // observed, beta sampled), then one pass that folds and already hashes the next round's leaves
    DBuf leaves;
    for (int rd = 0; rd < nrounds; rd++) {
        const int lf = log_max - 1 - rd;
        const uint64_t h = cur_n >> 1;
        if (rd == 0) {
            leaves = DBuf(8 * h, s);
            launch_fri_leaves(cur.p, h, leaves.p, s);
        }
        // keep the folded-from vector: queries open (lo, hi) pairs of it
        ftrees[rd].owned.push_back(std::move(cur));
        const FriChal fc{dchal, droots.p + 8 * rd, dfargs.p + 8 * rd};
        if (!tree_from_leaves(ftrees[rd], std::move(leaves), h, s, false, &fc))
            launch_fri_chal(dchal, ftrees[rd].layers[ftrees[rd].log_max], droots.p + 8 * rd, dfargs.p + 8 * rd, s);
        DBuf next(4 * h, s);
        const uint32_t *rof = ro[lf].p ? ro[lf].p : nullptr;
        if (rd + 1 < nrounds) {
            leaves = DBuf(8 * (h / 2), s);
            launch_fri_fold_leaves(ftrees[rd].owned.back().p, h, dfargs.p + 8 * rd, c.tw_inv, rof, next.p, leaves.p,
                                   s);
        } else {
            launch_fri_fold(ftrees[rd].owned.back().p, h, dfargs.p + 8 * rd, c.tw_inv, rof, next.p, s);
        }
        cur = std::move(next);
        cur_n = h;
    }
    std::vector<uint32_t> fin(4 * cur_n), hroots(8 * std::max(nrounds, 1));
    HIP_CHECK(hipMemcpyAsync(fin.data(), cur.p, fin.size() * 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(hroots.data(), droots.p, hroots.size() * 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(&hc, dchal, sizeof hc, hipMemcpyDeviceToHost, s));
    fri_prof.reset();
    HIP_CHECK(hipStreamSynchronize(s));
    for (int rd = 0; rd < nrounds; rd++) {
        memcpy(ftrees[rd].root, &hroots[8 * rd], 32);
        proof.fri_commits.push_back(dig(ftrees[rd].root));
    }
    memcpy(ch.st, hc.st, 64);
    memcpy(ch.in, hc.in, 32);
    memcpy(ch.out, hc.out, 32);
    ch.nin = (int)hc.nin;
    ch.nout = (int)hc.nout;
    proof.final_poly = ef{{fin[0], fin[1], fin[2], fin[3]}};
    bool final_ok = true;
    for (uint64_t i = 1; i < cur_n; i++)
        final_ok &= memcmp(&fin[4 * i], &fin[0], 16) == 0;
    ch.observe_ef(proof.final_poly);

    // ---- proof of work (canonical: smallest witness) ----
    {
        PowArgs pa{};
        memcpy(pa.state, ch.st, 64);
        memcpy(pa.in, ch.in, 32);
        pa.nin = (uint32_t)ch.nin;
        pa.mask = (1u << pk.cfg.pow_bits) - 1u;
        PROF("pow", s, 0);
        const uint32_t w = pk.cfg.pow_bits ? run_pow(pa, s) : 0u;
        proof.pow = to_mont(w);
        ch.observe(to_mont(w));
        const uint32_t bits = ch.sample_bits((int)pk.cfg.pow_bits);
        ARG_CHECK(bits == 0, "proof-of-work witness check failed");
    }

    // ---- queries: gather rows and Merkle paths ----
    const uint32_t nq = pk.cfg.num_queries;
    std::vector<uint64_t> idx(nq);
    for (uint32_t q = 0; q < nq; q++) idx[q] = ch.sample_bits(log_max);
    std::vector<uint64_t> items;  // (src, stride | count << 32, dst)
    uint64_t total = 0;
    auto item = [&](const uint32_t *src, uint64_t stride, uint64_t count) {
        items.push_back((uint64_t)(uintptr_t)src);
        items.push_back(stride | (count << 32));
        items.push_back(total);
        total += count;
    };
    for (uint32_t q = 0; q < nq; q++) {
        for (int t = 0; t < 4; t++) {
            const DTree *tt = trees[t];
            const uint64_t ri = idx[q] >> (log_max - tt->log_max);
            for (auto &mm : tt->mats) {
                const uint64_t row = ri >> (tt->log_max - ilog2(mm.height));
                if (mm.width) item(mm.d + row, mm.height, mm.width);
            }
            for (int l = 0; l < tt->log_max; l++) item(tt->layers[l] + ((ri >> l) ^ 1) * 8, 1, 8);
        }
        for (int rd = 0; rd < nrounds; rd++) {
            const uint64_t ii = idx[q] >> rd, pair = ii >> 1;
            item(ftrees[rd].owned.back().p + 8 * pair + 4 * ((ii ^ 1) & 1), 1, 4);
            for (int l = 0; l < ftrees[rd].log_max; l++) item(ftrees[rd].layers[l] + ((pair >> l) ^ 1) * 8, 1, 8);
        }
    }
    HPROF("gather_wait");
    DBuf ditems(items.size() * 2 + 2, s), dout(total + 1, s);
    HIP_CHECK(hipMemcpyAsync(ditems.p, items.data(), items.size() * 8, hipMemcpyHostToDevice, s));
    launch_gather((const uint64_t *)ditems.p, (uint32_t)(items.size() / 3), dout.p, s);
    std::vector<uint32_t> g(total + 1);
    HIP_CHECK(hipMemcpyAsync(g.data(), dout.p, total * 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    uint64_t off = 0;
    proof.queries.resize(nq);
    for (uint32_t q = 0; q < nq; q++) {
        Query &Q = proof.queries[q];
        for (int t = 0; t < 4; t++) {
            const DTree *tt = trees[t];
            BatchOpen bo;
            for (auto &mm : tt->mats) {
                bo.vals.emplace_back(g.begin() + off, g.begin() + off + mm.width);
                off += mm.width;
            }
            for (int l = 0; l < tt->log_max; l++) { bo.path.push_back(dig(&g[off])); off += 8; }
            Q.input.push_back(std::move(bo));
        }
        for (int rd = 0; rd < nrounds; rd++) {
            Step st;
            st.sib = ef{{g[off], g[off + 1], g[off + 2], g[off + 3]}};
            off += 4;
            for (int l = 0; l < ftrees[rd].log_max; l++) { st.path.push_back(dig(&g[off])); off += 8; }
            Q.steps.push_back(std::move(st));
        }
    }

    // ---- opened values into the proof (prover.rs:558-640) ----
    for (int i = 0; i < n; i++) {
        ChipOpen &co = proof.chips[i];
        const int pki = pk.pk_index(md.chip[i]);
        const int pw_ = m.chips[md.chip[i]].prep_w;
        if (pki >= 0) {
            const OpenReq &r = req[pki];
            co.prep_l = r.vals[0];
            co.prep_n = r.npts == 2 ? r.vals[1] : std::vector<ef>(pw_, ef_zero());
        }
        const OpenReq &mr = req[pk.trace_chip.size() + i];
        co.main_l = mr.vals[0];
        co.main_n = mr.npts == 2 ? mr.vals[1] : std::vector<ef>(mr.vals[0].size(), ef_zero());
        const OpenReq &pr = req[pk.trace_chip.size() + n + i];
        co.perm_l = pr.vals[0];
        co.perm_n = pr.vals[1];
    }
    {
        size_t qi = pk.trace_chip.size() + 2 * n;
        for (int i = 0; i < n; i++) {
            const int nq_ = 1 << m.chips[md.chip[i]].log_qd;
            for (int j = 0; j < nq_; j++, qi++)
                for (int e = 0; e < 4; e++) proof.chips[i].quot.push_back(req[qi].vals[0][e]);
        }
    }
    HIP_CHECK(hipStreamSynchronize(s));
    if (!final_ok) throw std::runtime_error("UNSATISFIED: FRI final polynomial is not constant");
    HPROF("serialize");
    return serialize(proof, pk.cfg.proof_montgomery != 0);
}

}  // namespace zkm

using namespace zkm;

static int status_of(const std::exception &e) {
    // the failing call's stream was drained by its StreamLease; other streams are not touched
    std::string w = e.what();
    if (w.rfind("UNSATISFIED", 0) == 0) { g_last_error = w; return ZKM_ERR_UNSATISFIED; }
    if (w.find("not supported") != std::string::npos) { g_last_error = w; return ZKM_ERR_UNSUPPORTED; }
    return guard_status(e);
}
#define GUARD_BEGIN try {
#define GUARD_END                         \
    }                                     \
    catch (const std::exception &e) {     \
        return status_of(e);              \
    }

extern "C" {

int zkm_setup(zkm_ctx *ctx, const uint32_t *blob, size_t nwords, const zkm_config_t *cfg, const zkm_matrix_t *prep,
              uint32_t nprep, uint32_t pc_start, const uint32_t gcs[14], zkm_pk **pk_out, uint32_t commit_out[8]) {
    GUARD_BEGIN
    ARG_CHECK(ctx && blob && cfg && pk_out && commit_out && gcs, "null argument");
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    HIP_CHECK(hipSetDevice(c->device));
    ARG_CHECK(cfg->log_blowup == 1 || cfg->log_blowup == 2, "log_blowup must be 1 or 2");
    ARG_CHECK(cfg->pow_bits < 31, "pow_bits");
    auto pk = std::make_unique<Pk>();
    pk->device = c->device;
    pk->m = parse_machine(blob, nwords);
    pk->cfg = *cfg;
    pk->digest = machine_digest(blob, nwords, cfg->log_blowup);
    pk->pc_start = to_mont(pc_start);
    for (int k = 0; k < 14; k++) pk->gcs[k] = to_mont(gcs[k]);
    ARG_CHECK(nprep == pk->m.chips.size(), "one preprocessed matrix slot per machine chip");
    StreamLease L(c);
    for (auto &cd : pk->m.chips) {
        std::vector<uint32_t> f = flatten_chip(cd);
        pk->progs.emplace_back(f.size(), L.s);
        HIP_CHECK(hipMemcpyAsync(pk->progs.back().p, f.data(), f.size() * 4, hipMemcpyHostToDevice, L.s));
        HIP_CHECK(hipStreamSynchronize(L.s));
    }
    pk->jit.resize(pk->m.chips.size());
    if (jit_enabled()) {
        // hiprtc compiles are independent per chip: run them concurrently
        std::vector<std::future<JitKernel>> fut;
        for (auto &cd : pk->m.chips)
            fut.push_back(std::async(std::launch::async, [&cd, dev = c->device] {
                (void)hipSetDevice(dev);
                try {
                    return jit_chip(cd, dev);
                } catch (const std::exception &e) {
                    fprintf(stderr, "zkm: quotient JIT failed for chip %s, using the interpreter kernel: %s\n",
                            cd.name.c_str(), e.what());
                    return JitKernel{};
                }
            }));
        for (size_t i = 0; i < fut.size(); i++) pk->jit[i] = fut[i].get();
    }
    // preprocessed traces sorted by (height desc, name) (machine.rs:383-384)
    std::vector<int> chips;
    std::vector<uint64_t> hs;
    std::vector<std::string> names;
    for (size_t i = 0; i < pk->m.chips.size(); i++) {
        if (pk->m.chips[i].prep_w == 0) continue;
        ARG_CHECK(prep[i].data && prep[i].width == (uint64_t)pk->m.chips[i].prep_w, "preprocessed trace shape");
        chips.push_back((int)i);
        hs.push_back(prep[i].height);
        names.push_back(pk->m.chips[i].name);
    }
    ARG_CHECK(!chips.empty(), "machine has no preprocessed trace (MerkleTree of an empty batch)");
    for (int o : sort_order(hs, names)) {
        const int ci = chips[o];
        ARG_CHECK((prep[ci].height & (prep[ci].height - 1)) == 0, "heights must be powers of two");
        pk->trace_chip.push_back(ci);
        pk->heights.push_back(prep[ci].height);
        pk->traces.push_back(upload_matrix(*c, prep[ci], L.s));
        DMat src{pk->traces.back().p, prep[ci].height, prep[ci].width};
        add_lde(*c, pk->tree, src, to_mont(GENERATOR), false, (int)cfg->log_blowup, L.s);
    }
    tree_build(pk->tree, L.s);
    memcpy(pk->commit, pk->tree.root, 32);
    for (int k = 0; k < 8; k++) commit_out[k] = from_mont(pk->commit[k]);
    *pk_out = reinterpret_cast<zkm_pk *>(pk.release());
    return ZKM_OK;
    GUARD_END
}

void zkm_pk_free(zkm_pk *p) {
    if (!p) return;
    Pk *pk = reinterpret_cast<Pk *>(p);
    (void)hipSetDevice(pk->device);
    (void)hipDeviceSynchronize();
    delete pk;
}

int zkm_pk_observe(const zkm_pk *p, zkm_challenger_t *c) {
    GUARD_BEGIN
    ARG_CHECK(p && c, "null argument");
    const Pk *pk = reinterpret_cast<const Pk *>(p);
    Challenger ch;
    ch.load(*c);
    ch.observe(pk->commit, 8);
    ch.observe(pk->pc_start);
    ch.observe(pk->gcs, 14);
    ch.observe(0u);
    ch.store(*c);
    return ZKM_OK;
    GUARD_END
}

}  // extern "C"

// MachineProver::commit against a machine layout (from a key or a zkm_machine handle)
static int commit_impl(zkm_ctx *ctx, const Machine &mach, uint32_t log_blowup, uint64_t digest,
                       const zkm_matrix_t *traces, uint32_t ntraces, const uint32_t *pv, uint32_t npv,
                       zkm_main **out, uint32_t commit_out[8]) {
    GUARD_BEGIN
    ARG_CHECK(ctx && traces && ntraces && out && commit_out && (pv || !npv), "null argument");
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    HIP_CHECK(hipSetDevice(c->device));
    StreamLease L(c);
    auto md = std::make_unique<MainData>();
    md->machine = digest;
    std::vector<uint64_t> hs;
    std::vector<std::string> names;
    std::vector<int> chip;
    for (uint32_t i = 0; i < ntraces; i++) {
        ARG_CHECK(traces[i].name, "trace without a chip name");
        const int ci = mach.index_of(traces[i].name);
        ARG_CHECK(ci >= 0, std::string("unknown chip ") + traces[i].name);
        ARG_CHECK(traces[i].width == (uint64_t)mach.chips[ci].main_w, "main trace width mismatch");
        ARG_CHECK(traces[i].height >= 16 && (traces[i].height & (traces[i].height - 1)) == 0,
                  "trace heights must be powers of two >= 16");
        hs.push_back(traces[i].height);
        names.push_back(traces[i].name);
        chip.push_back(ci);
    }
    PROF("commit_total", L.s, 0);
    HPROF("commit");
    // sorted by (height desc, name) (prover.rs:264); each run of equal heights is uploaded side by
    // side into one column-major buffer and LDE'd in one batch
    const std::vector<int> ord = sort_order(hs, names);
    for (size_t a = 0, b; a < ord.size(); a = b) {
        const uint64_t N = hs[ord[a]];
        uint64_t W = 0;
        for (b = a; b < ord.size() && hs[ord[b]] == N; b++) W += traces[ord[b]].width;
        md->store.emplace_back(N * (W ? W : 1), L.s);
        uint32_t *base = md->store.back().p;
        std::vector<uint64_t> ws;
        uint64_t off = 0;
        for (size_t k = a; k < b; k++) {
            const int o = ord[k];
            md->chip.push_back(chip[o]);
            md->heights.push_back(N);
            md->trace.push_back(base + off * N);
            upload_matrix_into(*c, traces[o], base + off * N, L.s);
            ws.push_back(traces[o].width);
            off += traces[o].width;
        }
        for (const DMat &v : lde_group(*c, md->tree, base, N, ws, to_mont(GENERATOR), false, (int)log_blowup, L.s))
            md->tree.mats.push_back(v);
    }
    tree_build(md->tree, L.s);
    md->pv.assign(pv, pv + npv);
    for (int k = 0; k < 8; k++) commit_out[k] = from_mont(md->tree.root[k]);
    *out = reinterpret_cast<zkm_main *>(md.release());
    return ZKM_OK;
    GUARD_END
}

extern "C" {

int zkm_commit(zkm_ctx *ctx, const zkm_pk *p, const zkm_matrix_t *traces, uint32_t ntraces, const uint32_t *pv,
               uint32_t npv, zkm_main **out, uint32_t commit_out[8]) {
    if (!p) { g_last_error = "null argument"; return ZKM_ERR_ARG; }
    const Pk *pk = reinterpret_cast<const Pk *>(p);
    return commit_impl(ctx, pk->m, pk->cfg.log_blowup, pk->digest, traces, ntraces, pv, npv, out, commit_out);
}

int zkm_machine_new(const uint32_t *blob, size_t nwords, const zkm_config_t *cfg, zkm_machine **out) {
    GUARD_BEGIN
    ARG_CHECK(blob && cfg && out, "null argument");
    ARG_CHECK(cfg->log_blowup == 1 || cfg->log_blowup == 2, "log_blowup must be 1 or 2");
    auto mh = std::make_unique<MachineHandle>();
    mh->m = parse_machine(blob, nwords);
    mh->cfg = *cfg;
    mh->digest = machine_digest(blob, nwords, cfg->log_blowup);
    *out = reinterpret_cast<zkm_machine *>(mh.release());
    return ZKM_OK;
    GUARD_END
}

void zkm_machine_free(zkm_machine *m) { delete reinterpret_cast<MachineHandle *>(m); }

int zkm_commit_machine(zkm_ctx *ctx, const zkm_machine *m, const zkm_matrix_t *traces, uint32_t ntraces,
                       const uint32_t *pv, uint32_t npv, zkm_main **out, uint32_t commit_out[8]) {
    if (!m) { g_last_error = "null argument"; return ZKM_ERR_ARG; }
    const MachineHandle *mh = reinterpret_cast<const MachineHandle *>(m);
    return commit_impl(ctx, mh->m, mh->cfg.log_blowup, mh->digest, traces, ntraces, pv, npv, out, commit_out);
}

void zkm_main_free(zkm_main *m) {
    if (!m) return;
    delete reinterpret_cast<MainData *>(m);
}

int zkm_open(zkm_ctx *ctx, const zkm_pk *p, zkm_main *mainp, zkm_challenger_t *chs, uint8_t **proof_out,
             uint64_t *proof_len) {
    std::unique_ptr<MainData> md(reinterpret_cast<MainData *>(mainp));
    GUARD_BEGIN
    ARG_CHECK(ctx && p && mainp && chs && proof_out && proof_len, "null argument");
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    const Pk *pk = reinterpret_cast<const Pk *>(p);
    ARG_CHECK(md->machine == pk->digest, "zkm_open: the shard was committed under a different machine than the key's");
    HIP_CHECK(hipSetDevice(c->device));
    StreamLease L(c);
    Challenger ch;
    ch.load(*chs);
    HPROF("open");
    std::vector<uint8_t> bytes = open_shard(*c, *pk, *md, ch, L.s);
    HIP_CHECK(hipStreamSynchronize(L.s));
    ch.store(*chs);
    uint8_t *buf = (uint8_t *)malloc(bytes.size());
    ARG_CHECK(buf, "out of host memory");
    memcpy(buf, bytes.data(), bytes.size());
    *proof_out = buf;
    *proof_len = bytes.size();
    HPROF("free_main");
    md.reset();
    return ZKM_OK;
    GUARD_END
}

int zkm_prove_shard(zkm_ctx *ctx, const zkm_pk *pk, const zkm_matrix_t *traces, uint32_t ntraces, const uint32_t *pv,
                    uint32_t npv, const zkm_challenger_t *base, uint8_t **proof_out, uint64_t *proof_len) {
    if (!base) { g_last_error = "null challenger"; return ZKM_ERR_ARG; }
    zkm_main *md = nullptr;
    uint32_t root[8];
    int rc = zkm_commit(ctx, pk, traces, ntraces, pv, npv, &md, root);
    if (rc) return rc;
    zkm_challenger_t ch = *base;
    return zkm_open(ctx, pk, md, &ch, proof_out, proof_len);
}

}  // extern "C"
