// C ABI entry points (include/zkm_hip.h): context, PCS commit, kernel-level helpers.
// Shard prover entry points (setup/commit/open) live in prover.cpp.
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/zkm_hip.h"
#include "internal.hpp"

namespace zkm {

thread_local std::string g_last_error;

hipStream_t Ctx::acquire_stream() {
    {
        std::lock_guard<std::mutex> g(mu);
        if (!free_streams.empty()) {
            hipStream_t s = free_streams.back();
            free_streams.pop_back();
            return s;
        }
    }
    HIP_CHECK(hipSetDevice(device));
    hipStream_t s;
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
}
void Ctx::release_stream(hipStream_t s) {
    std::lock_guard<std::mutex> g(mu);
    free_streams.push_back(s);
}

int guard_status(const std::exception &e) {
    g_last_error = e.what();
    if (dynamic_cast<const ArgError *>(&e)) return ZKM_ERR_ARG;
    return ZKM_ERR_HIP;
}

static bool zero_copy_enabled() {  // read per call (a getenv per matrix is noise next to a shard proof)
    const char *e = getenv("ZKM_ZERO_COPY");
    return e && *e && *e != '0';
}

// true when p lies in page-locked host memory (zkm_host_alloc / hipHostMalloc / hipHostRegister)
static bool host_pinned(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// host (or device) row-major matrix -> device column-major Montgomery, written to `col`
// (height * width words).  A page-locked host source is read by the DMA engine asynchronously,
// after this host thread has gone on to queue the shard's kernels (other shards' streams keep the
// GPU busy meanwhile); every entry point synchronises its stream before returning, so the
// caller's buffer outlives the copy.  (A FIFO of all calls' copies on one context stream was
// measured slower: 49.9 vs 45.1 ms per shard at 3 in flight.)  A pageable source is staged by the
// runtime and waited for.
void upload_matrix_into(Ctx &c, const zkm_matrix_t &m, uint32_t *col, hipStream_t s) {
    (void)c;
    ARG_CHECK(m.data || m.height * m.width == 0, "matrix data is NULL");
    const uint64_t n = m.height * m.width;
    if (!n) return;
    const bool mont = (m.repr & 0xffu) == ZKM_REPR_MONTGOMERY;
    if (m.repr & ZKM_MEM_DEVICE) {
        launch_to_col_major(m.data, m.height, m.width, mont, col, s);
        return;
    }
    const bool pinned = host_pinned(m.data);
    if (pinned && zero_copy_enabled() && m.width <= 128) {
        // ZKM_ZERO_COPY=1: the transpose kernel reads the page-locked host rows over PCIe itself (a
        // capped grid keeps the link busy without occupying the GPU); no DMA-engine copy
        void *dp = nullptr;
        HIP_CHECK(hipHostGetDevicePointer(&dp, const_cast<void *>(static_cast<const void *>(m.data)), 0));
        launch_to_col_major((const uint32_t *)dp, m.height, m.width, mont, col, s, 128);
        return;
    }
    DBuf raw(n, s);
    HIP_CHECK(hipMemcpyAsync(raw.p, m.data, n * 4, hipMemcpyHostToDevice, s));
    launch_to_col_major(raw.p, m.height, m.width, mont, col, s);
    if (!pinned) HIP_CHECK(hipStreamSynchronize(s));
}

DBuf upload_matrix(Ctx &c, const zkm_matrix_t &m, hipStream_t s) {
    DBuf col(m.height * m.width ? m.height * m.width : 1, s);
    upload_matrix_into(c, m, col.p, s);
    return col;
}

}  // namespace zkm

using namespace zkm;

#define GUARD_BEGIN try {
#define GUARD_END                                  \
    }                                              \
    catch (const std::exception &e) {              \
        return guard_status(e);                    \
    }

extern "C" {

const char *zkm_last_error(void) { return g_last_error.c_str(); }

int zkm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int zkm_init(int device, zkm_ctx **out) {
    GUARD_BEGIN
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        g_last_error = "no HIP device " + std::to_string(device);
        return ZKM_ERR_NO_DEVICE;
    }
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0) {
        g_last_error = std::string("device is ") + prop.gcnArchName + ", this library is built for gfx950";
        return ZKM_ERR_NO_DEVICE;
    }
    HIP_CHECK(hipSetDevice(device));
    auto *c = new Ctx();
    c->device = device;
    build_twiddles(*c, 24);  // transforms up to 2^24 (two-adicity)
    *out = reinterpret_cast<zkm_ctx *>(c);
    return ZKM_OK;
    GUARD_END
}

void zkm_destroy(zkm_ctx *ctx) {
    if (!ctx) return;
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    // Streams are intentionally not destroyed: proving keys and shard data may outlive the
    // context handle, and their stream-ordered buffers are released on the stream that made them.
    (void)hipFree(c->tw_fwd);
    (void)hipFree(c->tw_inv);
    (void)hipFree(c->tt_fwd);  // tt_inv shares the allocation
    delete c;       // cached twist tables go back to the pool
    pool_trim();    // blocks still owned by live keys / shard data stay allocated
}

void zkm_free_bytes(uint8_t *p) { free(p); }

int zkm_host_alloc(size_t bytes, void **out) {
    GUARD_BEGIN
    ARG_CHECK(out, "null argument");
    *out = nullptr;
    HIP_CHECK(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return ZKM_OK;
    GUARD_END
}

void zkm_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

int zkm_coset_lde_ex(zkm_ctx *ctx, const zkm_matrix_t *m, uint32_t shift, int bitrev_in, uint32_t *out);
int zkm_coset_lde(zkm_ctx *ctx, const zkm_matrix_t *m, uint32_t shift, uint32_t *out) {
    return zkm_coset_lde_ex(ctx, m, shift, 0, out);
}
int zkm_coset_lde_ex(zkm_ctx *ctx, const zkm_matrix_t *m, uint32_t shift, int bitrev_in, uint32_t *out) {
    GUARD_BEGIN
    ARG_CHECK(ctx && m && out, "null argument");
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    HIP_CHECK(hipSetDevice(c->device));
    StreamLease L(c);
    DBuf col = upload_matrix(*c, *m, L.s);
    DMat src{col.p, m->height, m->width};
    DBuf ld(2 * m->height * m->width, L.s);
    DMat dst{ld.p, 2 * m->height, m->width};
    if (bitrev_in) lde_batch_bitrev_in(*c, src, kb::to_mont(shift), dst, L.s);
    else lde_batch(*c, src, kb::to_mont(shift), dst, L.s);
    DBuf rm(2 * m->height * m->width, L.s);
    launch_from_col_major(ld.p, 2 * m->height, m->width, rm.p, L.s);
    HIP_CHECK(hipMemcpyAsync(out, rm.p, 2 * m->height * m->width * 4, hipMemcpyDeviceToHost, L.s));
    HIP_CHECK(hipStreamSynchronize(L.s));
    return ZKM_OK;
    GUARD_END
}

int zkm_poseidon2_permute(zkm_ctx *ctx, uint32_t *states, uint64_t n) {
    GUARD_BEGIN
    ARG_CHECK(ctx && (states || !n), "null argument");
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    HIP_CHECK(hipSetDevice(c->device));
    StreamLease L(c);
    std::vector<uint32_t> h(states, states + n * 16);
    for (auto &x : h) x = kb::to_mont(x);
    DBuf d(n * 16, L.s);
    HIP_CHECK(hipMemcpyAsync(d.p, h.data(), n * 64, hipMemcpyHostToDevice, L.s));
    launch_poseidon2_batch(d.p, n, L.s);
    HIP_CHECK(hipMemcpyAsync(h.data(), d.p, n * 64, hipMemcpyDeviceToHost, L.s));
    HIP_CHECK(hipStreamSynchronize(L.s));
    for (uint64_t i = 0; i < n * 16; i++) states[i] = kb::from_mont(h[i]);
    return ZKM_OK;
    GUARD_END
}

int zkm_pcs_commit_root(zkm_ctx *ctx, const zkm_matrix_t *mats, uint32_t n, uint32_t root_out[8]) {
    GUARD_BEGIN
    ARG_CHECK(ctx && mats && n && root_out, "null argument");
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    HIP_CHECK(hipSetDevice(c->device));
    StreamLease L(c);
    DTree t;
    for (uint32_t i = 0; i < n; i++) {
        DBuf col = upload_matrix(*c, mats[i], L.s);
        DMat src{col.p, mats[i].height, mats[i].width};
        t.owned.emplace_back(2 * mats[i].height * (mats[i].width ? mats[i].width : 1), L.s);
        DMat dst{t.owned.back().p, 2 * mats[i].height, mats[i].width};
        lde_batch(*c, src, kb::to_mont(kb::GENERATOR), dst, L.s);
        t.mats.push_back(dst);
    }
    tree_build(t, L.s);
    for (int k = 0; k < 8; k++) root_out[k] = kb::from_mont(t.root[k]);
    return ZKM_OK;
    GUARD_END
}

int zkm_bench_lde(zkm_ctx *ctx, uint64_t h, uint64_t w, int iters, double *ms_out) {
    GUARD_BEGIN
    ARG_CHECK(ctx && ms_out && iters > 0, "null argument");
    Ctx *c = reinterpret_cast<Ctx *>(ctx);
    HIP_CHECK(hipSetDevice(c->device));
    StreamLease L(c);
    DBuf src(h * w, L.s), dst(2 * h * w, L.s);
    // deterministic fill: Montgomery of index hash (values in [0,p))
    std::vector<uint32_t> host(h * w);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto &v : host) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint32_t)(x % kb::P); }
    HIP_CHECK(hipMemcpyAsync(src.p, host.data(), h * w * 4, hipMemcpyHostToDevice, L.s));
    DMat s{src.p, h, w}, d{dst.p, 2 * h, w};
    lde_batch(*c, s, kb::to_mont(3), d, L.s);  // warm-up
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    HIP_CHECK(hipEventRecord(e0, L.s));
    for (int i = 0; i < iters; i++) lde_batch(*c, s, kb::to_mont(3), d, L.s);
    HIP_CHECK(hipEventRecord(e1, L.s));
    HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    *ms_out = ms / iters;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return ZKM_OK;
    GUARD_END
}

}  // extern "C"
