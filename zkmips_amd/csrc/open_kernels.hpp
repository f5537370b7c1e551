// Kernel argument blocks and launchers of open_kernels.hip.
#pragma once
#include <vector>
#include "internal.hpp"

namespace zkm {

struct PermArgs {
    const uint32_t *prog;     // flattened chip program (device)
    const uint32_t *main;     // trace, column-major natural, n rows
    const uint32_t *prep;     // preprocessed trace or nullptr
    uint64_t n;
    kb::ef alpha;             // local permutation challenge alpha
    const uint32_t *beta_pows;// beta^(j+1), EF, j < max lookup arity (device)
    int batch, nb;            // lookups per batch, number of batch columns
    uint32_t *out;            // flattened perm trace, column-major (4 * (nb + 1) columns)
    uint32_t *rowsum;         // scratch: n EF
};
// rows_done: the per-row batch columns and rowsum were already written (JIT kernel); only scan
void launch_perm_trace(const PermArgs &a, hipStream_t s, bool rows_done = false);

struct QuotArgs {
    const uint32_t *prog;
    const uint32_t *main, *prep, *perm;  // LDEs (column stride ld, bit-reversed rows)
    uint64_t ld;                         // LDE height (2n)
    uint64_t n, q;                       // trace height, quotient domain size
    int log_n, log_q, step;
    const uint32_t *tw;                  // forward twiddles
    uint32_t gen, gen_pow_n, wn_inv;     // 3, 3^n, w_n^-1 (Montgomery)
    const uint32_t *pv;                  // public values (Montgomery)
    const uint32_t *pows;                // alpha^(nc-1-k), EF
    kb::ef alpha_p, lcs;
    const uint32_t *beta_pows;           // beta^(j+1), EF (device)
    uint32_t gcs[14];
    int batch, perm_w, global, main_w;
    uint32_t *chunks;                    // 2^lqd chunks x 4 columns x n rows (bit-reversed rows)
    uint64_t cstride;                    // words from chunk j to chunk j+1
    // shared subexpressions (OP_LET / OP_GET): value slots in global scratch, slot s of row t at
    // slots[s * slot_rows + (t - t0)]; the rows run in windows of slot_rows starting at t0
    int n_slots;
    uint32_t *slots;
    uint64_t slot_rows, t0;
};
void launch_quotient(const QuotArgs &a, hipStream_t s);

void launch_inv_points(const kb::ef &z, uint32_t s, const uint32_t *tw, uint64_t M, bool bitrev, bool mul_omega,
                       uint32_t *out, hipStream_t st);
// the weights of an opening, w_j = (mul_omega ? w_n^idx : 1) / (z - s w_n^idx), idx = bitrev ? rev(j) : j
// (launch_inv_points' table, generated inside the opening kernel instead)
struct OpenWeights {
    kb::ef z;
    uint32_t s;
    const uint32_t *tw;  // forward twiddles
    int log_n, bitrev, mul_omega;
};
// One opening group: the columns of one (height, evaluation domain, point set), whose weights are shared.
// The caller fills cols (device column pointer table), n, w, ncols, with_next and out; the launcher sets
// the grid shape, kernel kind and partial-sum buffer.
struct OpenGroup {
    const uint64_t *cols;
    uint64_t n;
    OpenWeights w;
    uint32_t ncols, slab, nslab;
    int nseg, with_next, kind;
    uint32_t *partial, *out;
};
// Every group's dot products in one launch per kernel kind (+ one segment-sum launch); `gs` is uploaded
// asynchronously from host memory, so it must outlive the stream's execution of these launches.
void launch_open_dot_groups(std::vector<OpenGroup> &gs, hipStream_t s);

struct ReduceArgs {
    const uint64_t *cols;      // column pointer table
    const uint32_t *desc;      // per-matrix descriptors
    uint32_t nmats;
    const uint32_t *alpha_pows;// alpha^c, EF
    kb::ef z0, z1;             // the opening points (z1 = zeta w_N, used when has1)
    int has1;
    uint32_t gen;              // coset shift of the LDE rows (Montgomery)
    const uint32_t *tw;        // forward twiddles: x_i = gen w_h^rev(i)
    int log_h;
    uint32_t *ro;              // EF reduced openings, h entries (written, not accumulated)
    uint64_t h;
};
void launch_fri_reduce(const ReduceArgs &a, hipStream_t s);
// duplex-challenger state in device memory (Montgomery), same fields as the host Challenger
struct DevChallenger {
    uint32_t st[16];
    uint32_t in[8];
    uint32_t nin;
    uint32_t out[8];
    uint32_t nout;
};
void launch_fri_chal(DevChallenger *c, const uint32_t *root, uint32_t *root_out, uint32_t *fargs, hipStream_t s);
void launch_fri_fold(const uint32_t *cur, uint64_t h, const uint32_t *fargs, const uint32_t *tw_inv,
                     const uint32_t *ro, uint32_t *next, hipStream_t s);
void launch_fri_leaves(const uint32_t *cur, uint64_t h, uint32_t *out, hipStream_t s);
// fold into next (h elements) and hash next's pairs into the next round's h / 2 leaves
void launch_fri_fold_leaves(const uint32_t *cur, uint64_t h, const uint32_t *fargs, const uint32_t *tw_inv,
                            const uint32_t *ro, uint32_t *next, uint32_t *leaves, hipStream_t s);
// the transcript step a FRI tree's top launch runs after the root (fri_chal.cuh)
struct FriChal {
    DevChallenger *c;
    uint32_t *root_out, *fargs;
};

struct PowArgs {
    uint32_t state[16];
    uint32_t in[8];
    uint32_t nin;
    uint32_t mask;
};
uint32_t run_pow(const PowArgs &a, hipStream_t s);

void launch_gather(const uint64_t *d_items, uint32_t nitems, uint32_t *dst, hipStream_t s);

// LDE variant for bit-reversed input evaluations (quotient chunks)
void lde_batch_bitrev_in(Ctx &c, const DMat &src, uint32_t shift_mont, DMat &dst, hipStream_t s);
// tree from a precomputed leaf digest layer (FRI commit-phase trees)
// read_root = false: the root stays on the device (t.layers[t.log_max]); t.root is not set
// with fc, the launch that computes the root also runs the FRI transcript step; returns whether it did
bool tree_from_leaves(DTree &t, DBuf &&leaves, uint64_t nleaves, hipStream_t s, bool read_root = true,
                      const FriChal *fc = nullptr);

}  // namespace zkm
