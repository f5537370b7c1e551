// Poseidon2 Merkle commitment (MerkleTreeMmcs over PaddingFreeSponge<P,16,8,8> leaves and
// TruncatedPermutation<P,2,8,16> nodes, crates/stark/src/kb31_poseidon2.rs:173-177) on gfx950.
//
// Tree semantics pinned by crates/recursion/circuit/src/fri.rs:363-405:
//   leaf i   = sponge(row i of every tallest matrix, concatenated in commit order)
//   node     = compress(left, right), then, if matrices of that height exist,
//              compress(node, sponge(their rows)).
// One thread hashes one row: matrices are column-major, so a wavefront reads 64 consecutive
// rows of a column (256 B) per absorbed element.  Digests are stored digest-major (32 B each).
#include <algorithm>
#include <numeric>

#include "internal.hpp"
#include "open_kernels.hpp"
#include "p2.cuh"
#include "fri_chal.cuh"
#include "prof.hpp"

namespace zkm {

static constexpr int NT = 256;

// Sponge digest of row i of `ncols` columns (device pointer table); the state stays in the
// permutation's internal representation between chunks (p2::Sponge).
__device__ __forceinline__ void sponge_row(const uint64_t *__restrict__ cols, int ncols, uint64_t i, uint32_t d[8]) {
    // global (not flat) loads: flat loads also count on lgkmcnt, so every scalar-load wait inside
    // the permutation would drain the prefetched chunk
    typedef const __attribute__((address_space(1))) uint32_t *gptr;
    p2::sponge_hash(ncols, [&](int k) { return ((gptr)cols[k])[i]; }, d);
}

__global__ __launch_bounds__(NT) void k_hash_leaves(const uint64_t *__restrict__ cols, int ncols, uint64_t nrows,
                                                    uint32_t *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= nrows) return;
    uint32_t s[8];
    sponge_row(cols, ncols, i, s);
    uint4 *o = (uint4 *)(out + i * 8);
    o[0] = make_uint4(s[0], s[1], s[2], s[3]);
    o[1] = make_uint4(s[4], s[5], s[6], s[7]);
}

// One node per thread: compress(left, right).  (Levels with injected matrices: k_compress_inject; keeping a
// sponge path in this kernel held it to 82 VGPRs, five waves per SIMD, instead of eight.)
__global__ __launch_bounds__(NT) void k_compress_level(const uint32_t *__restrict__ prev, uint32_t *__restrict__ out,
                                                       uint64_t h) {
    uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= h) return;
    uint32_t s[16];
    const uint4 *p = (const uint4 *)(prev + i * 16);
    uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w; s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
    s[8] = c.x; s[9] = c.y; s[10] = c.z; s[11] = c.w; s[12] = d.x; s[13] = d.y; s[14] = d.z; s[15] = d.w;
    p2::permute(s);
    uint4 *o = (uint4 *)(out + i * 8);
    o[0] = make_uint4(s[0], s[1], s[2], s[3]);
    o[1] = make_uint4(s[4], s[5], s[6], s[7]);
}

// Level with injected matrices whose rows were hashed beforehand (by k_hash_leaves, the prefetching
// one-thread-per-row sponge): node = compress(compress(left, right), digest of the injected row).
__global__ __launch_bounds__(NT) void k_compress_inject(const uint32_t *__restrict__ prev, uint32_t *__restrict__ out,
                                                        uint64_t h, const uint32_t *__restrict__ inj_digest) {
    uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= h) return;
    uint32_t s[16];
    const uint4 *p = (const uint4 *)(prev + i * 16);
    uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w; s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
    s[8] = c.x; s[9] = c.y; s[10] = c.z; s[11] = c.w; s[12] = d.x; s[13] = d.y; s[14] = d.z; s[15] = d.w;
    p2::permute(s);
    const uint4 *q = (const uint4 *)(inj_digest + i * 8);
    uint4 e = q[0], f = q[1];
    s[8] = e.x; s[9] = e.y; s[10] = e.z; s[11] = e.w; s[12] = f.x; s[13] = f.y; s[14] = f.z; s[15] = f.w;
    p2::permute(s);
    uint4 *o = (uint4 *)(out + i * 8);
    o[0] = make_uint4(s[0], s[1], s[2], s[3]);
    o[1] = make_uint4(s[4], s[5], s[6], s[7]);
}

__global__ void k_p2_batch(uint32_t *st, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    uint32_t s[16];
#pragma unroll
    for (int k = 0; k < 16; k++) s[k] = st[i * 16 + k];
    p2::permute(s);
#pragma unroll
    for (int k = 0; k < 16; k++) st[i * 16 + k] = s[k];
}

__global__ __launch_bounds__(NT) void k_p2_batch16(uint32_t *st, uint64_t n);

// small batches are latency-bound: they take the 16-lane form
void launch_poseidon2_batch(uint32_t *d, uint64_t n, hipStream_t s) {
    if (!n) return;
    if (n <= 1024)
        hipLaunchKernelGGL(k_p2_batch16, dim3((unsigned)((n * 16 + NT - 1) / NT)), dim3(NT), 0, s, d, n);
    else
        hipLaunchKernelGGL(k_p2_batch, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, s, d, n);
    HIP_CHECK(hipGetLastError());
}

// ---- latency-bound levels: one node per 16-lane row (p2x16) ----
static constexpr uint64_t SMALL16 = 8192;  // levels with <= SMALL16 nodes use the 16-lane form
static constexpr int NT_TOP = 1024;
static constexpr uint64_t TOP_MAX = NT_TOP / 16;  // levels with <= TOP_MAX nodes: one workgroup
// levels with <= this many nodes: k_subtree16 (the threshold sweep, profiles/r03_sub16.txt)
static uint64_t sub16_max() { return 16384; }

__global__ __launch_bounds__(NT) void k_compress16(const uint32_t *__restrict__ prev, uint32_t *__restrict__ out,
                                                   uint64_t h) {
    const uint64_t t = (uint64_t)blockIdx.x * NT + threadIdx.x;
    const uint64_t i = t >> 4;
    const int l = (int)(t & 15);
    const p2x16::Lane c = p2x16::lane_consts(l);
    const uint32_t x = p2x16::permute(i < h ? prev[i * 16 + l] : 0u, c);  // all lanes take part
    if (i < h && l < 8) out[i * 8 + l] = x;
}

__global__ __launch_bounds__(NT) void k_p2_batch16(uint32_t *st, uint64_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * NT + threadIdx.x;
    const uint64_t i = t >> 4;
    const int l = (int)(t & 15);
    const uint32_t x = p2x16::permute(i < n ? st[i * 16 + l] : 0u, p2x16::lane_consts(l));
    if (i < n) st[i * 16 + l] = x;
}

// Builds `nlev` levels above `prev` (2*h1 digests, h1 <= TOP_MAX) in one workgroup: level k has
// h1 >> k nodes and is written contiguously to out (level 0 first); levels also live in LDS.
__global__ __launch_bounds__(NT_TOP) void k_tree_top(const uint32_t *__restrict__ prev, uint64_t h1, int nlev,
                                                     uint32_t *__restrict__ out) {
    __shared__ uint32_t buf[2][TOP_MAX * 8];
    const int i = threadIdx.x >> 4, l = threadIdx.x & 15;
    const p2x16::Lane c = p2x16::lane_consts(l);
    uint64_t h = h1, off = 0;
    for (int lev = 0; lev < nlev; lev++, h >>= 1) {
        const uint32_t *src = lev == 0 ? prev : buf[(lev - 1) & 1];
        const uint32_t x = p2x16::permute((uint64_t)i < h ? src[i * 16 + l] : 0u, c);
        if ((uint64_t)i < h && l < 8) {
            buf[lev & 1][i * 8 + l] = x;
            out[(off + i) * 8 + l] = x;
        }
        __syncthreads();
        off += h;
    }
}

// Up to 7 levels above `prev` (2h child digests) in one launch: workgroup b owns the subtree whose
// bottom is nodes [m b, m b + m) of the first level (m = min(h, 64)), one node per 16-lane row; level k
// of the launch has h >> k nodes, stored contiguously from out + 8 (h (2 - 2^(1-k))) and kept in LDS for
// the next level.  A wave whose four rows have no node at a level skips the permutation (uniform
// branch), so the upper levels of a subtree run with the SIMDs free for the waves that work.
// With chal (the launch that ends at a FRI tree's root, one workgroup), the round's transcript step
// follows in the same workgroup (fri_chal.cuh).
__global__ __launch_bounds__(NT_TOP) void k_subtree16(const uint32_t *__restrict__ prev, uint64_t h, int nlev,
                                                      uint32_t *__restrict__ out, DevChallenger *chal,
                                                      uint32_t *root_out, uint32_t *fargs) {
    __shared__ uint32_t buf[2][TOP_MAX * 8];
    __shared__ ChalShared sh;
    const int g = threadIdx.x >> 4, l = threadIdx.x & 15, wave_g0 = (threadIdx.x >> 6) * 4;
    const p2x16::Lane c = p2x16::lane_consts(l);
    const uint64_t m = h < TOP_MAX ? h : TOP_MAX;
    uint64_t hl = h, off = 0, mk = m;
    for (int lev = 0; lev < nlev && mk; lev++, off += hl, hl >>= 1, mk >>= 1) {
        if ((uint64_t)wave_g0 < mk) {
            const uint64_t node = (uint64_t)blockIdx.x * mk + g;
            const bool act = (uint64_t)g < mk;
            const uint32_t in = !act ? 0u : lev == 0 ? prev[node * 16 + l] : buf[(lev - 1) & 1][g * 16 + l];
            const uint32_t x = p2x16::permute(in, c);
            if (act && l < 8) {
                buf[lev & 1][g * 8 + l] = x;
                out[(off + node) * 8 + l] = x;
            }
        }
        __syncthreads();
    }
    if (chal) fri_chal_block(sh, chal, buf[(nlev - 1) & 1], root_out, fargs);
}

static DBuf upload_cols(const std::vector<const DMat *> &group, std::vector<uint64_t> &host, hipStream_t s) {
    host.clear();
    for (const DMat *m : group)
        for (uint64_t c = 0; c < m->width; c++) host.push_back((uint64_t)(uintptr_t)(m->d + c * m->height));
    DBuf d(host.size() * 2 + 2, s);
    if (!host.empty()) HIP_CHECK(hipMemcpyAsync(d.p, host.data(), host.size() * 8, hipMemcpyHostToDevice, s));
    return d;
}

// Levels 1..log_max above layers[0]; inj[L] = column table of matrices injected at level L.
static bool build_levels(DTree &t, uint64_t maxh, const std::vector<std::pair<const DBuf *, int>> &inj, hipStream_t s,
                         const FriChal *fc = nullptr) {
    bool chal_done = false;
    uint64_t h = maxh;
    for (int L = 1; L <= t.log_max; L++) {
        h >>= 1;
        bool later_inj = false;
        for (int k = L; k <= t.log_max; k++) later_inj |= inj[k].second != 0;
        const int ninj = inj[L].second;
        if (h <= sub16_max() && ninj == 0) {
            // subtree launches: one node per workgroup at the top of each (up to 7 levels), never across
            // a level with injected matrices
            const uint64_t m = h < TOP_MAX ? h : TOP_MAX;
            int nlev = 1;
            while (nlev < ilog2(m) + 1 && L + nlev <= t.log_max && inj[L + nlev].second == 0) nlev++;
            uint64_t tot = 0;
            for (int k = 0; k < nlev; k++) tot += h >> k;
            t.layer_store.emplace_back(tot * 8, s);
            uint32_t *base = t.layer_store.back().p;
            uint64_t off = 0;
            for (int k = 0; k < nlev; k++) { t.layers[L + k] = base + off * 8; off += h >> k; }
            const bool top = fc && L + nlev - 1 == t.log_max && h / m == 1;
            hipLaunchKernelGGL(k_subtree16, dim3((unsigned)(h / m)), dim3(NT_TOP), 0, s,
                               (const uint32_t *)t.layers[L - 1], h, nlev, base, top ? fc->c : nullptr,
                               top ? fc->root_out : nullptr, top ? fc->fargs : nullptr);
            HIP_CHECK(hipGetLastError());
            chal_done |= top;
            L += nlev - 1;
            h >>= nlev - 1;
            continue;
        }
        if (h <= TOP_MAX && !later_inj) {
            // remaining levels L..log_max in one workgroup, one contiguous allocation
            const int nlev = t.log_max - L + 1;
            t.layer_store.emplace_back(2 * h * 8, s);
            uint32_t *base = t.layer_store.back().p;
            uint64_t off = 0, hh = h;
            for (int k = L; k <= t.log_max; k++, hh >>= 1) { t.layers[k] = base + off * 8; off += hh; }
            hipLaunchKernelGGL(k_tree_top, dim3(1), dim3(NT_TOP), 0, s, (const uint32_t *)t.layers[L - 1], h, nlev, base);
            HIP_CHECK(hipGetLastError());
            break;
        }
        t.layer_store.emplace_back(h * 8, s);
        t.layers[L] = t.layer_store.back().p;
        if (h <= SMALL16 && ninj == 0) {
            hipLaunchKernelGGL(k_compress16, dim3((unsigned)((h * 16 + NT - 1) / NT)), dim3(NT), 0, s,
                               (const uint32_t *)t.layers[L - 1], t.layers[L], h);
            HIP_CHECK(hipGetLastError());
            continue;
        }
        if (ninj > 0) {
            // the injected rows go through the leaf kernel first (its prefetching sponge runs at the
            // VALU-issue bound; one thread doing compress + sponge + compress ran at ~0.75 of it)
            DBuf dig(8 * h, s);
            hipLaunchKernelGGL(k_hash_leaves, dim3((unsigned)((h + NT - 1) / NT)), dim3(NT), 0, s,
                               (const uint64_t *)inj[L].first->p, ninj, h, dig.p);
            HIP_CHECK(hipGetLastError());
            hipLaunchKernelGGL(k_compress_inject, dim3((unsigned)((h + NT - 1) / NT)), dim3(NT), 0, s,
                               (const uint32_t *)t.layers[L - 1], t.layers[L], h, (const uint32_t *)dig.p);
            HIP_CHECK(hipGetLastError());
            continue;
        }
        hipLaunchKernelGGL(k_compress_level, dim3((unsigned)((h + NT - 1) / NT)), dim3(NT), 0, s,
                           (const uint32_t *)t.layers[L - 1], t.layers[L], h);
        HIP_CHECK(hipGetLastError());
    }
    return chal_done;
}

void tree_build(DTree &t, hipStream_t s) {
    const int n = (int)t.mats.size();
    ARG_CHECK(n > 0, "empty MMCS batch");
    std::vector<int> order(n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return t.mats[a].height > t.mats[b].height; });
    const uint64_t maxh = t.mats[order[0]].height;
    ARG_CHECK((maxh & (maxh - 1)) == 0, "matrix heights must be powers of two");
    t.log_max = ilog2(maxh);
    t.layers.assign(t.log_max + 1, nullptr);
    t.layer_store.clear();
    std::vector<std::vector<uint64_t>> keep(t.log_max + 2);
    std::vector<DBuf> colbufs;
    colbufs.reserve(t.log_max + 2);
    std::vector<std::pair<const DBuf *, int>> inj(t.log_max + 1, {nullptr, 0});
    size_t pos = 0;
    std::vector<const DMat *> grp;
    while (pos < order.size() && t.mats[order[pos]].height == maxh) grp.push_back(&t.mats[order[pos++]]);
    colbufs.push_back(upload_cols(grp, keep[0], s));
    const int ncols = (int)keep[0].size();
    uint64_t h = maxh;
    for (int L = 1; L <= t.log_max; L++) {
        h >>= 1;
        grp.clear();
        while (pos < order.size() && t.mats[order[pos]].height == h) grp.push_back(&t.mats[order[pos++]]);
        if (grp.empty()) continue;
        colbufs.push_back(upload_cols(grp, keep[L], s));
        // a group of zero-width matrices still injects hash(empty) = the zero digest
        inj[L] = {&colbufs.back(), keep[L].empty() ? -1 : (int)keep[L].size()};
    }
    ARG_CHECK(pos == order.size(), "matrix heights must be powers of two <= max");
    t.layer_store.emplace_back(maxh * 8, s);
    t.layers[0] = t.layer_store.back().p;
    {
        PROF("merkle_leaves", s, 4.0 * maxh * ncols + 32.0 * maxh);  // algorithmic bytes
        prof_add("merkle_leaves_perms", (double)maxh * ((ncols + 7) / 8));
        hipLaunchKernelGGL(k_hash_leaves, dim3((unsigned)((maxh + NT - 1) / NT)), dim3(NT), 0, s,
                           (const uint64_t *)colbufs[0].p, ncols, maxh, t.layers[0]);
        HIP_CHECK(hipGetLastError());
    }
    {
        PROF("merkle_nodes", s, 96.0 * maxh);
        build_levels(t, maxh, inj, s);
    }
    HIP_CHECK(hipMemcpyAsync(t.root, t.layers[t.log_max], 32, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
}

bool tree_from_leaves(DTree &t, DBuf &&leaves, uint64_t nleaves, hipStream_t s, bool read_root, const FriChal *fc) {
    ARG_CHECK(nleaves && (nleaves & (nleaves - 1)) == 0, "leaf count must be a power of two");
    t.log_max = ilog2(nleaves);
    t.layers.assign(t.log_max + 1, nullptr);
    t.layer_store.clear();
    t.layer_store.push_back(std::move(leaves));
    t.layers[0] = t.layer_store.back().p;
    std::vector<std::pair<const DBuf *, int>> inj(t.log_max + 1, {nullptr, 0});
    const bool chal = build_levels(t, nleaves, inj, s, fc);
    if (read_root) {
        HIP_CHECK(hipMemcpyAsync(t.root, t.layers[t.log_max], 32, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
    }
    return chal;
}

}  // namespace zkm
