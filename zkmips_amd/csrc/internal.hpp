// Internal declarations of the MI355X shard prover (not part of the C ABI).
#pragma once
#include "prof.hpp"
#include <hip/hip_runtime.h>

#include <cstdint>
#include <exception>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "kb31.cuh"

namespace zkm {

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct ArgError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define HIP_CHECK(expr)                                                                       \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess)                                                                 \
            throw ::zkm::HipError(std::string(#expr) + ": " + hipGetErrorString(_e) + " @" + \
                                  __FILE__ + ":" + std::to_string(__LINE__));                 \
    } while (0)
#define ARG_CHECK(cond, msg)                        \
    do {                                            \
        if (!(cond)) throw ::zkm::ArgError(msg);    \
    } while (0)

inline int ilog2(uint64_t n) {
    int l = 0;
    while ((1ull << l) < n) l++;
    return l;
}

// Caching device allocator (pool.cpp): stream-tagged reuse of hipMalloc'd blocks.
void *pool_alloc(size_t bytes, hipStream_t s);
void pool_free(void *p, hipStream_t s);
void pool_trim();  // synchronises the device, returns cached blocks to the driver
void pool_stats(size_t *in_use, size_t *cached);

// Stream-ordered device buffer.
struct DBuf {
    uint32_t *p = nullptr;
    size_t words = 0;
    hipStream_t s = nullptr;
    DBuf() = default;
    DBuf(size_t n, hipStream_t st) : words(n), s(st) {
        if (n) p = (uint32_t *)pool_alloc(n * sizeof(uint32_t), st);
    }
    DBuf(const DBuf &) = delete;
    DBuf &operator=(const DBuf &) = delete;
    DBuf(DBuf &&o) noexcept { *this = std::move(o); }
    DBuf &operator=(DBuf &&o) noexcept {
        reset();
        p = o.p; words = o.words; s = o.s;
        o.p = nullptr; o.words = 0;
        return *this;
    }
    void reset() {
        if (p) pool_free(p, s);
        p = nullptr;
        words = 0;
    }
    ~DBuf() { reset(); }
};

// Column-major device matrix (Montgomery values), column stride = height.
struct DMat {
    uint32_t *d = nullptr;
    uint64_t height = 0, width = 0;
};

// Device Merkle tree over several column-major matrices (MerkleTreeMmcs semantics,
// pinned by crates/recursion/circuit/src/fri.rs:363-405).
struct DTree {
    std::vector<DMat> mats;        // commit order
    std::vector<DBuf> owned;       // storage of mats (if owned)
    int log_max = 0;
    std::vector<uint32_t *> layers;  // layers[i]: (max_h >> i) digests x 8 words, digest-major
    std::vector<DBuf> layer_store;   // storage behind `layers`
    uint32_t root[8];              // Montgomery
};

struct Ctx {
    int device = 0;
    // cached per (log n, shift): LDE twist tables (lo[4096] | hi[n/4096]) x 2 cosets
    std::vector<std::pair<std::pair<int, uint32_t>, DBuf>> twists;
    int tw_log = 0;                 // twiddle tables cover transforms up to 2^tw_log
    uint32_t *tw_fwd = nullptr;     // tw[h + j] = w_{2h}^j  (Montgomery), size 2^tw_log
    uint32_t *tw_inv = nullptr;
    uint32_t *tt_fwd = nullptr;     // per-thread twiddle rows of the 8192-point tiles (ntt.hip)
    uint32_t *tt_inv = nullptr;
    std::mutex mu;
    std::vector<hipStream_t> free_streams;
    hipStream_t acquire_stream();
    void release_stream(hipStream_t s);
};

// One HIP stream per entry-point call.  When the call unwinds with an exception, only this
// stream is drained (device buffers are stream-ordered in the pool; host temporaries that async
// copies may still touch are gone once the stream is idle) — other shards' streams keep running.
struct StreamLease {
    Ctx *c;
    hipStream_t s;
    int exc0;
    explicit StreamLease(Ctx *ctx) : c(ctx), s(ctx->acquire_stream()), exc0(std::uncaught_exceptions()) {}
    ~StreamLease() {
        if (std::uncaught_exceptions() > exc0) (void)hipStreamSynchronize(s);
        c->release_stream(s);
    }
};

// host/device row-major zkm_matrix_t -> device column-major Montgomery (capi.cpp)
}  // namespace zkm
#include "../../include/zkm_hip.h"
namespace zkm {
void upload_matrix_into(Ctx &c, const zkm_matrix_t &m, uint32_t *col, hipStream_t s);
DBuf upload_matrix(Ctx &c, const zkm_matrix_t &m, hipStream_t s);

// ---------------------------------------------------------------- kernels (launchers)
// host row-major (canonical or Montgomery) -> device column-major Montgomery
// max_grid > 0 caps the workgroup count (grid-stride loop): used when d_rowmajor is page-locked host
// memory read over PCIe by the kernel itself, so a few workgroups keep the link busy
void launch_to_col_major(const uint32_t *d_rowmajor, uint64_t h, uint64_t w, bool montgomery_in,
                         uint32_t *d_col, hipStream_t s, unsigned max_grid = 0);
void launch_from_col_major(const uint32_t *d_col, uint64_t h, uint64_t w, uint32_t *d_rowmajor_canon,
                           hipStream_t s);
void build_twiddles(Ctx &c, int log_max);
// Bit-reversed coset LDE of `src` (h x w col-major) into `dst` (2h x w col-major):
// dst column c row i = p_c(shift * w_{2h}^{rev(i)}), p_c interpolating src column c on H_h.
void lde_batch(Ctx &c, const DMat &src, uint32_t shift_mont, DMat &dst, hipStream_t s);
// same, for evaluations given in bit-reversed row order
void lde_batch_bitrev_in(Ctx &c, const DMat &src, uint32_t shift_mont, DMat &dst, hipStream_t s);
// the same, column c of the 2N-row result at dst + c * dst_stride (dst_stride >= 2N)
void lde_batch_strided(Ctx &c, const DMat &src, uint32_t shift_mont, uint32_t *dst, uint64_t dst_stride, hipStream_t s);
void lde_batch_bitrev_in_strided(Ctx &c, const DMat &src, uint32_t shift_mont, uint32_t *dst, uint64_t dst_stride,
                                 hipStream_t s);
// blowup 4 (dst: 4h x w col-major) from natural-order src, one shared inverse transform
void lde_batch_blowup4(Ctx &c, const DMat &src, uint32_t shift0_mont, uint32_t shift1_mont, uint32_t *dst,
                       hipStream_t s);

// Merkle
void tree_build(DTree &t, hipStream_t s);
void launch_poseidon2_batch(uint32_t *d_states, uint64_t n, hipStream_t s);

}  // namespace zkm
