// sparse_ids.hpp — device code of the sparse-id mode (GS_CC_SPARSE_IDS): DisjointSet<Long> over
// arbitrary 64-bit vertex ids (any Java long, negative ones included), as the reference's
// DisjointSet<R> keys its HashMaps by the id itself (summaries/DisjointSet.java:28-34).
//
// Layout: an open-addressing table keys[H] (H = power of two >= 2 x vertex capacity, linear
// probing, splitmix64 hash, empty = INT64_MIN) gives every id a SLOT; slot H is reserved for
// the id INT64_MIN itself. The union-find state is the ordinary parent[] over H + 1 slots, so
// the fold, the giant filter, the close and the incremental close run unchanged on slot
// numbers. Slots are not ordered like ids, so a root is the smallest SLOT of its component, not
// its smallest id: the canonical label (minimum id of the component, what the reference's
// emissions canonicalise to) is a separate min-reduction into minkey[root] (k_minkey_*), done
// when an emission asks for it.
//
// Insertion claims a slot by CAS of its key word (no value word to publish, so no thread ever
// waits for another: a lane spinning on a same-wave lane's write would deadlock).
#pragma once

#include "cc_kernels.hpp"

namespace gsgpu {

constexpr int64_t kEmptyKey = INT64_MIN;

struct SparseArgs {
    int64_t* keys;            // H words
    uint32_t hbits;           // H = 2^hbits
    unsigned long long* nkeys;    // distinct ids inserted (capacity check)
    uint64_t vcap;            // vertex capacity (GS_ERR_CAPACITY beyond it)
    uint32_t* err;            // err[0] bit 1: table full / capacity exceeded
};

__device__ __forceinline__ uint32_t sparse_home(int64_t id, uint32_t hbits) {
    return (uint32_t)(splitmix64((uint64_t)id) >> (64 - hbits));
}

// slot of id; inserts it when absent (INSERT) or returns kInvalid (lookup only / table full)
template <bool INSERT>
__device__ __forceinline__ uint32_t sparse_slot(const SparseArgs& s, int64_t id) {
    const uint32_t H = 1u << s.hbits;
    if (id == kEmptyKey) return H;                     // the reserved slot
    uint32_t h = sparse_home(id, s.hbits);
    for (uint32_t step = 0; step < H; ++step) {
        int64_t k = __hip_atomic_load(&s.keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == id) return h;
        if (k == kEmptyKey) {
            if (!INSERT) return kInvalid;
            const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long*>(&s.keys[h]),
                                                     (unsigned long long)kEmptyKey, (unsigned long long)id);
            if ((int64_t)old == kEmptyKey) {
                const unsigned long long c = atomicAdd(s.nkeys, 1ull);
                if (c >= s.vcap) atomicOr(s.err, 2u);
                return h;
            }
            if ((int64_t)old == id) return h;
        }
        h = (h + 1) & (H - 1);
    }
    if (INSERT) atomicOr(s.err, 2u);
    return kInvalid;
}

__device__ __forceinline__ int64_t slot_key(const SparseArgs& s, uint32_t slot) {
    return slot == (1u << s.hbits) ? kEmptyKey : s.keys[slot];
}

// UpdateCC over arbitrary int64 ids (SoA a/b, or AoS pairs in a): slots, then the usual filter +
// union on slot numbers.
template <bool AOS, bool MARK>
__global__ __launch_bounds__(256) void k_fold_sparse(const int64_t* __restrict__ a, const int64_t* __restrict__ b,
                                                     FoldArgs f, SparseArgs s) {
    const bool filt = *f.giant != kInvalid;
    if (!filt) f.sbits = nullptr;                    // the next close is a full pass (k_fold)
    FoldStats st;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g * 2 < f.n; g += stride) {
        uint32_t u[2], v[2];
        bool ok[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint64_t e = g * 2 + k;
            ok[k] = e < f.n;
            u[k] = v[k] = 0;
            if (ok[k]) {
                const int64_t x = AOS ? a[2 * e] : a[e];
                const int64_t y = AOS ? a[2 * e + 1] : b[e];
                u[k] = sparse_slot<true>(s, x);
                v[k] = sparse_slot<true>(s, y);
                ok[k] = u[k] != kInvalid && v[k] != kInvalid;
                if (!ok[k]) { u[k] = 0; v[k] = 0; }
            }
        }
        uint32_t gflag[2];
        if (filt) filter_group<false, 2, false>(f, u, v, ok, nullptr, HotArgs{nullptr, 0, nullptr}, false, false, false, gflag);
        union_group<MARK, false, 2>(f, u, v, ok, st);
    }
}

// DisjointSet.merge(other) between sparse summaries: union(key, parent key) for every slot of
// `other` in the summary (DisjointSet.java:127-131 iterates other.getMatches()).
template <bool MARK>
__global__ __launch_bounds__(256) void k_merge_sparse(const uint32_t* __restrict__ oparent, SparseArgs os,
                                                      FoldArgs f, SparseArgs s) {
    const uint32_t n = (1u << os.hbits) + 1;
    FoldStats st;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t p = oparent[i];
        if (p == kInvalid) continue;
        const uint32_t u[1] = {sparse_slot<true>(s, slot_key(os, i))};
        const uint32_t v[1] = {sparse_slot<true>(s, slot_key(os, p))};
        const bool ok[1] = {u[0] != kInvalid && v[0] != kInvalid};
        const uint32_t uu[1] = {ok[0] ? u[0] : 0u}, vv[1] = {ok[0] ? v[0] : 0u};
        union_group<MARK, false, 1>(f, uu, vv, ok, st);
    }
}

// Partial-summary export of a sparse-id summary (multi-GPU CombineCC, comm.hip): as k_export_log,
// every pending hook-log entry (a slot hooked since the last export, or a self-loop first touch)
// becomes the pair (id, id of its root slot) as two int64 words: the receiver hashes both ids into
// its own slots and unions them (DisjointSet.merge over the pairs, DisjointSet.java:127-131). The
// root's id is any member's of the component (slot roots are not id minima); a union only needs
// one. ctr = [length, read cursor, finished workgroups]; at most cap pairs written, the rest stay.
__global__ __launch_bounds__(256) void k_export_log_sparse(const uint32_t* __restrict__ log, unsigned long long* __restrict__ ctr,
                                                           const uint32_t* __restrict__ parent, SparseArgs s,
                                                           int64_t* __restrict__ pairs, uint64_t cap,
                                                           unsigned long long* __restrict__ count) {
    const unsigned long long len = ctr[0], rd = ctr[1];
    const unsigned long long n = len - rd;
    const unsigned long long take = n < cap ? n : cap;
    if (blockIdx.x == 0 && threadIdx.x == 0) *count = n;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < take;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const uint32_t v = log[rd + i];
        pairs[2 * i] = slot_key(s, v);
        pairs[2 * i + 1] = slot_key(s, find_root_ro(parent, v));
    }
    __syncthreads();
    if (threadIdx.x == 0 && len >= rd) {             // the last workgroup consumes what was written
        const unsigned long long done = atomicAdd(&ctr[2], 1ull);
        if (done == gridDim.x - 1) {
            if (rd + take == len) { ctr[0] = 0; ctr[1] = 0; }
            else ctr[1] = rd + take;
            ctr[2] = 0;
        }
    }
}

// Folds received sparse partial summaries laid out in slots (comm.hip's speculative all-gather):
// slot q = [uint64 count][cap pairs (id, id) as int64], slot_words 32-bit words apart; pairs
// [lo, min(count, hi)) of every slot but `skip` are hashed to slots (inserted if new) and unioned.
// blockIdx.y = slot. No marks (the others' deltas are theirs to export).
__global__ __launch_bounds__(256) void k_fold_slots_sparse(const uint32_t* __restrict__ slots, uint64_t slot_words, int skip,
                                                           uint64_t lo, uint64_t hi, FoldArgs f, SparseArgs s, SlotCaps caps) {
    const int q = blockIdx.y;
    if (q == skip) return;                           // uniform
    if (caps.n && caps.v[q] < hi) hi = caps.v[q];
    if (*f.giant == kInvalid) f.sbits = nullptr;     // the next close is a full pass (k_fold)
    const uint32_t* sq = slots + (uint64_t)q * slot_words;
    const unsigned long long cnt = *reinterpret_cast<const unsigned long long*>(sq);
    const uint64_t n = cnt < hi ? cnt : hi;
    const int64_t* pairs = reinterpret_cast<const int64_t*>(sq + 2);
    FoldStats st;
    for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t a = sparse_slot<true>(s, pairs[2 * i]), b = sparse_slot<true>(s, pairs[2 * i + 1]);
        const bool ok[1] = {a != kInvalid && b != kInvalid};
        const uint32_t u[1] = {ok[0] ? a : 0u}, v[1] = {ok[0] ? b : 0u};
        union_group<false, false, 1>(f, u, v, ok, st);
    }
}

// minkey[r] = key of every root r (parent compressed: parent[s] is s's root)
__global__ __launch_bounds__(256) void k_minkey_init(const uint32_t* __restrict__ parent, uint32_t n, SparseArgs s,
                                                     int64_t* __restrict__ minkey) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (parent[i] == i) minkey[i] = slot_key(s, i);
}

// minkey[root(s)] = min over the component's ids. Members of the giant (root g) are reduced in
// the workgroup first (one atomic per workgroup instead of one per member on one word).
__global__ __launch_bounds__(256) void k_minkey_reduce(const uint32_t* __restrict__ parent, uint32_t n, SparseArgs s,
                                                       const uint32_t* __restrict__ giant, int64_t* __restrict__ minkey) {
    __shared__ long long wmin[4];
    const uint32_t g = giant[0];
    long long gmin = INT64_MAX;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t p = parent[i];
        if (p == kInvalid || p == i) continue;
        const long long k = slot_key(s, i);
        if (p == g) gmin = k < gmin ? k : gmin;
        else atomicMin(reinterpret_cast<long long*>(&minkey[p]), k);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const long long o = __shfl_down(gmin, off, 64);
        gmin = o < gmin ? o : gmin;
    }
    if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = gmin;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long m = wmin[0];
        for (int w = 1; w < 4; ++w) m = wmin[w] < m ? wmin[w] : m;
        if (m != INT64_MAX && g != kInvalid) atomicMin(reinterpret_cast<long long*>(&minkey[g]), m);
    }
}

// n_vertices, n_components and the emission checksum over (id, min id) of every slot in the summary
__global__ __launch_bounds__(256) void k_stats_sparse(const uint32_t* __restrict__ parent, uint32_t n, SparseArgs s,
                                                      const int64_t* __restrict__ minkey, unsigned long long* __restrict__ out) {
    unsigned long long seen = 0, roots = 0, h = 0;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t p = parent[i];
        if (p == kInvalid) continue;
        ++seen;
        roots += (p == i);
        h += pair_mix((uint64_t)slot_key(s, i), (uint64_t)minkey[p]);
    }
    __shared__ unsigned long long red[3][4];
    seen = wave_sum(seen); roots = wave_sum(roots); h = wave_sum(h);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) { red[0][wid] = seen; red[1][wid] = roots; red[2][wid] = h; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long a = 0, r = 0, c = 0;
        for (int w = 0; w < 4; ++w) { a += red[0][w]; r += red[1][w]; c += red[2][w]; }
        atomicAdd(&out[0], a);
        atomicAdd(&out[1], r);
        atomicAdd(&out[2], c);
    }
}

// (id, label) of every slot in the summary, unordered (compacted per wave; sorted on the host side
// of the call by a device radix sort)
__global__ __launch_bounds__(256) void k_emit_sparse(const uint32_t* __restrict__ parent, uint32_t n, SparseArgs s,
                                                     const int64_t* __restrict__ minkey, int64_t* __restrict__ ko,
                                                     int64_t* __restrict__ lo, unsigned long long* __restrict__ counter) {
    const int lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < n; i0 += stride) {
        const uint32_t i = i0 + threadIdx.x;
        const uint32_t p = i < n ? parent[i] : kInvalid;
        const bool in = p != kInvalid;
        const uint64_t m = __ballot(in);
        unsigned long long base = 0;
        if (lane == 0 && m) base = atomicAdd(counter, (unsigned long long)__popcll(m));
        base = __shfl(base, 0, 64);
        if (in) {
            const uint64_t pos = base + __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
            ko[pos] = slot_key(s, i);
            lo[pos] = minkey[p];
        }
    }
}

// DisjointSet.find for ids: canonical label, found[i] = 0 when the id is not in the summary
// (null; its label word is then -1, which is also a valid Long id: the flag disambiguates)
__global__ __launch_bounds__(256) void k_find_sparse(const int64_t* __restrict__ ids, int64_t* __restrict__ out,
                                                     uint8_t* __restrict__ found, uint64_t n,
                                                     const uint32_t* __restrict__ parent, SparseArgs s,
                                                     const int64_t* __restrict__ minkey) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t slot = sparse_slot<false>(s, ids[i]);
        const bool in = slot != kInvalid && parent[slot] != kInvalid;
        out[i] = in ? minkey[find_root_ro(parent, slot)] : -1;
        if (found) found[i] = in ? 1 : 0;
    }
}

__global__ __launch_bounds__(256) void k_fill64(int64_t* __restrict__ p, uint64_t n, int64_t v) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

}  // namespace gsgpu
