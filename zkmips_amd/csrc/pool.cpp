// Caching device allocator behind DBuf.
//
// hipMallocAsync/hipFreeAsync cost tens of microseconds of host time per call on this stack (a
// proof frees ~850 buffers: ~17 ms of a 78 ms step went to hipFreeAsync alone), so device memory
// is allocated once with hipMalloc and recycled.  A freed block remembers the stream it was freed
// on; reuse on the same stream is ordered by the stream itself, reuse on another stream first
// makes that stream wait for everything already submitted to the old one.  Blocks are never
// returned to the driver until zkm_destroy, or when hipMalloc fails (then the cache is trimmed
// after a device synchronisation and the allocation retried).
#include <map>
#include <mutex>
#include <unordered_map>

#include "internal.hpp"

namespace zkm {

namespace {

struct Block {
    void *p;
    size_t size;
    hipStream_t s;
};

struct Pool {
    std::mutex mu;
    std::multimap<size_t, Block> free_;        // by size
    std::unordered_map<void *, size_t> live_;  // ptr -> block size
    size_t cached = 0, in_use = 0;
};

std::mutex g_pools_mu;
std::map<int, Pool *> g_pools;

Pool &pool_for(int dev) {
    std::lock_guard<std::mutex> g(g_pools_mu);
    Pool *&p = g_pools[dev];
    if (!p) p = new Pool();
    return *p;
}

int current_device() {
    int d = 0;
    (void)hipGetDevice(&d);
    return d;
}

size_t round_size(size_t b) {
    if (b <= (1u << 20)) return (b + 511) & ~(size_t)511;
    return (b + (1u << 16) - 1) & ~(((size_t)1 << 16) - 1);
}

// waste bound for reusing a larger cached block
bool fits(size_t block, size_t want) { return block - want <= want / 4 + 4096; }

}  // namespace

void *pool_alloc(size_t bytes, hipStream_t s) {
    const size_t want = round_size(bytes ? bytes : 1);
    Pool &P = pool_for(current_device());
    {
        std::lock_guard<std::mutex> g(P.mu);
        // prefer a block freed on this stream, otherwise the tightest one
        auto lo = P.free_.lower_bound(want);
        auto pick = P.free_.end();
        for (auto it = lo; it != P.free_.end() && fits(it->first, want); ++it) {
            if (pick == P.free_.end()) pick = it;
            if (it->second.s == s) { pick = it; break; }
        }
        if (pick != P.free_.end()) {
            Block b = pick->second;
            P.free_.erase(pick);
            P.live_[b.p] = b.size;
            P.cached -= b.size;
            P.in_use += b.size;
            if (b.s != s) {
                hipEvent_t ev;
                HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                HIP_CHECK(hipEventRecord(ev, b.s));
                HIP_CHECK(hipStreamWaitEvent(s, ev, 0));
                HIP_CHECK(hipEventDestroy(ev));
            }
            return b.p;
        }
    }
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        pool_trim();
        HIP_CHECK(hipMalloc(&p, want));
    }
    std::lock_guard<std::mutex> g(P.mu);
    P.live_[p] = want;
    P.in_use += want;
    return p;
}

void pool_free(void *p, hipStream_t s) {
    if (!p) return;
    Pool &P = pool_for(current_device());
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.live_.find(p);
    if (it == P.live_.end()) return;  // not ours (cannot happen through DBuf)
    const size_t sz = it->second;
    P.live_.erase(it);
    P.in_use -= sz;
    P.cached += sz;
    P.free_.emplace(sz, Block{p, sz, s});
}

void pool_trim() {
    Pool &P = pool_for(current_device());
    (void)hipDeviceSynchronize();
    std::lock_guard<std::mutex> g(P.mu);
    for (auto &kv : P.free_) (void)hipFree(kv.second.p);
    P.free_.clear();
    P.cached = 0;
}

void pool_stats(size_t *in_use, size_t *cached) {
    Pool &P = pool_for(current_device());
    std::lock_guard<std::mutex> g(P.mu);
    *in_use = P.in_use;
    *cached = P.cached;
}

}  // namespace zkm
