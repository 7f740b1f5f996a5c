// bip.hip — BipartitenessCheck on the device: the reference's Candidates summary
// (summaries/Candidates.java:25-197, library/BipartitenessCheck.java:50-133) restated as a
// union-find with parity, extern "C" in include/gsgpu.h (gs_bip_*).
//
// State: one uint32 word per vertex id (ids < 2^31 - 1):
//   w[v] == kInvalid           v not in the summary
//   w[v] == (p << 1) | a       v hangs below p (p <= v), a = parity of v relative to p
//   w[v] == (v << 1)           v is a root
// A vertex's sign in the emission is true iff its parity relative to its root is 0. As in the
// CC kernels the larger root is hooked under the smaller one, so every root is its component's
// minimum id = the reference's component key (edgeToCandidate keys a component by its smaller
// endpoint, merges keep the smaller key: Candidates.java:54-61, :167), and the key vertex is
// signed true (BipartitenessCheckTest.java:45-48).
// An edge (u, v) requires parity(u) != parity(v); a merged partial summary contributes
// (v, parent(v)) with the parity it records. A constraint between two vertices already in one
// component that does not hold is an odd cycle: the summary fails for good, like
// Candidates.fail() (:194-196), and emits "(false,{})".
// Self-loops only add their vertex: edgeToCandidate(v, v) adds (v, true), its (v, false) is
// refused by add() and the refusal ignored (BipartitenessCheck.java:54-61, Candidates.java:55-67).
//
// Concurrency follows cc_kernels.hpp: hooks are atomicCAS on the larger root's word (a failed
// hook re-finds both roots), path halving is a no-return atomicMin of a packed word (the packed
// order is the parent order, and the parity to a given ancestor is unique, so any two writers
// agree on it), a walk treats a word that is not below its index (a stale kInvalid) as a root.
#include <algorithm>
#include <cstring>
#include <unordered_map>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "common.hpp"
#include "bip_literal.hpp"

namespace gsgpu {

constexpr uint32_t kBipMaxCap = 0x7FFFFFFFu;      // ids < 2^31 - 1: packed words never equal kInvalid

struct BipArgs {
    uint32_t* w;
    uint32_t cap;
    uint32_t* flags;      // flags[0]: bit 0 range error; flags[1]: 1 = odd cycle seen (not bipartite)
};

// (root, parity of x relative to root) given wx = a read of w[x]
__device__ __forceinline__ uint32_t bip_find(uint32_t* __restrict__ w, uint32_t x, uint32_t wx, uint32_t& par) {
    uint32_t cur = x, wc = wx;
    par = 0;
    for (;;) {
        const uint32_t p = wc >> 1;
        if (p >= cur) return cur;                     // root, or a stale kInvalid read
        const uint32_t wp = w[p];
        par ^= wc & 1u;
        const uint32_t pp = wp >> 1;
        if (pp < p)                                   // halve: cur now points at its grandparent
            __hip_atomic_fetch_min(&w[cur], (pp << 1) | ((wc ^ wp) & 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cur = p;
        wc = wp;
    }
}

__device__ __forceinline__ uint32_t bip_make(uint32_t* __restrict__ w, uint32_t v) {
    const uint32_t wv = w[v];
    if (wv != kInvalid) return wv;
    const uint32_t old = atomicCAS(&w[v], kInvalid, v << 1);
    return old == kInvalid ? (v << 1) : old;
}

// require parity(u) ^ parity(v) == rel (1 for an edge)
__device__ __forceinline__ void bip_union(const BipArgs& a, uint32_t u, uint32_t v, uint32_t rel) {
    uint32_t wu = bip_make(a.w, u);
    if (u == v) return;                               // self-loop: makeSet only
    uint32_t wv = bip_make(a.w, v);
    for (;;) {
        uint32_t pu, pv;
        const uint32_t ru = bip_find(a.w, u, wu, pu);
        const uint32_t rv = bip_find(a.w, v, wv, pv);
        if (ru == rv) {
            if ((pu ^ pv) != rel) atomicOr(&a.flags[1], 1u);
            return;
        }
        const uint32_t hi = ru > rv ? ru : rv, lo = ru > rv ? rv : ru;
        const uint32_t want = (lo << 1) | (pu ^ pv ^ rel);
        if (atomicCAS(&a.w[hi], hi << 1, want) == (hi << 1)) return;
        wu = a.w[u];                                  // hi was hooked meanwhile: walk again
        wv = a.w[v];
    }
}

typedef uint32_t u32x4b __attribute__((ext_vector_type(4)));

// BipartitenessCheck.updateFunction.foldEdges (BipartitenessCheck.java:93-95) over a batch
template <typename IdT, bool AOS, bool VEC>
__global__ __launch_bounds__(256) void k_bip_fold(const IdT* __restrict__ a, const IdT* __restrict__ b, uint64_t n,
                                                  BipArgs ba) {
    if (ba.flags[1]) return;                          // failed for good: nothing to add
    const uint64_t groups = (n + 3) / 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += stride) {
        uint32_t u[4], v[4];
        bool ok[4];
        bool bad = false;
        if (VEC && g * 4 + 4 <= n) {
            const u32x4b x = __builtin_nontemporal_load(reinterpret_cast<const u32x4b*>(a) + g);
            const u32x4b y = __builtin_nontemporal_load(reinterpret_cast<const u32x4b*>(b) + g);
            u[0] = x.x; u[1] = x.y; u[2] = x.z; u[3] = x.w;
            v[0] = y.x; v[1] = y.y; v[2] = y.z; v[3] = y.w;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                ok[k] = u[k] < ba.cap && v[k] < ba.cap;
                bad |= !ok[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t e = g * 4 + k;
                IdT x = 0, y = 0;
                if (e < n) {
                    x = AOS ? a[2 * e] : a[e];
                    y = AOS ? a[2 * e + 1] : b[e];
                }
                const bool in = e < n;
                ok[k] = in && (uint64_t)x < ba.cap && (uint64_t)y < ba.cap && !(sizeof(IdT) == 8 && ((int64_t)x < 0 || (int64_t)y < 0));
                bad |= in && !ok[k];
                u[k] = (uint32_t)x;
                v[k] = (uint32_t)y;
            }
        }
        if (bad) atomicOr(&ba.flags[0], 1u);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (ok[k]) bip_union(ba, u[k], v[k], 1u);
    }
}

// Candidates.merge of another summary (Candidates.java:70-128, combineFunction :121-124):
// every (v, parent) of `from` with its recorded parity
__global__ __launch_bounds__(256) void k_bip_merge(const uint32_t* __restrict__ from, uint32_t n,
                                                   const uint32_t* __restrict__ from_flags, BipArgs ba) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && from_flags[1]) atomicOr(&ba.flags[1], 1u);   // fail propagates (:72-74)
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += stride) {
        const uint32_t wv = from[v];
        if (wv == kInvalid) continue;
        bip_union(ba, v, wv >> 1, wv & 1u);
    }
}

// Merger emission: full compression (only v's thread writes w[v]; read-only walks)
__global__ __launch_bounds__(256) void k_bip_compress(uint32_t* __restrict__ w, uint32_t n) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += stride) {
        const uint32_t wv = w[v];
        if (wv == kInvalid || (wv >> 1) == v) continue;
        uint32_t cur = wv >> 1, par = wv & 1u, wc = w[cur];
        while ((wc >> 1) < cur) {
            par ^= wc & 1u;
            cur = wc >> 1;
            wc = w[cur];
        }
        const uint32_t nw = (cur << 1) | par;
        if (nw != wv) w[v] = nw;
    }
}

// n_vertices, n_components, checksum over (v, key << 1 | sign) of every vertex in the summary
__global__ __launch_bounds__(256) void k_bip_stats(const uint32_t* __restrict__ w, uint32_t n, unsigned long long* out) {
    unsigned long long seen = 0, roots = 0, h = 0;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += stride) {
        const uint32_t wv = w[v];
        if (wv == kInvalid) continue;
        ++seen;
        roots += (wv >> 1) == v;
        h += pair_mix(v, ((uint64_t)(wv >> 1) << 1) | ((wv & 1u) ? 0u : 1u));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        seen += __shfl_down(seen, off, 64);
        roots += __shfl_down(roots, off, 64);
        h += __shfl_down(h, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&out[0], seen);
        atomicAdd(&out[1], roots);
        atomicAdd(&out[2], h);
    }
}

// (vertex, key, sign) of every vertex in the summary, ordered by vertex: per-tile counts, a
// one-block scan, then an ordered scatter (as gs_cc_emit_pairs)
constexpr uint32_t kBipTile = 4096;
__global__ __launch_bounds__(256) void k_bip_count(const uint32_t* __restrict__ w, uint32_t n, uint32_t* cnt) {
    __shared__ uint32_t s;
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    uint32_t c = 0;
    const uint64_t base = (uint64_t)blockIdx.x * kBipTile;
    for (uint32_t i = threadIdx.x; i < kBipTile; i += 256)
        c += (base + i < n && w[base + i] != kInvalid);
    atomicAdd(&s, c);
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = s;
}

__global__ __launch_bounds__(1024) void k_bip_scan(const uint32_t* __restrict__ cnt, uint64_t* __restrict__ off, uint32_t nt) {
    __shared__ unsigned long long part[1024];
    const uint32_t per = (nt + blockDim.x - 1) / blockDim.x;
    const uint32_t lo = threadIdx.x * per, hi = min(lo + per, nt);
    unsigned long long s = 0;
    for (uint32_t i = lo; i < hi; ++i) s += cnt[i];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long run = 0;
        for (uint32_t t = 0; t < blockDim.x; ++t) { const unsigned long long x = part[t]; part[t] = run; run += x; }
        off[nt] = run;
    }
    __syncthreads();
    unsigned long long run = part[threadIdx.x];
    for (uint32_t i = lo; i < hi; ++i) { off[i] = run; run += cnt[i]; }
}

template <typename IdT>
__global__ __launch_bounds__(256) void k_bip_scatter(const uint32_t* __restrict__ w, uint32_t n, const uint64_t* __restrict__ off,
                                                     IdT* __restrict__ vo, IdT* __restrict__ ko, uint8_t* __restrict__ so,
                                                     uint64_t cap) {
    // one wave walks the tile in order, 64 vertices per step, ballot-compacted
    __shared__ unsigned long long wbase[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * kBipTile;
    constexpr uint32_t kSub = kBipTile / 4;          // each wave owns a quarter of the tile, in order
    // count of each quarter, so the waves know where their quarter starts
    uint32_t c = 0;
    for (uint32_t i = lane; i < kSub; i += 64) {
        const uint64_t v = base + wid * kSub + i;
        c += (v < n && w[v] != kInvalid);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
    if (lane == 0) wbase[wid] = c;
    __syncthreads();
    unsigned long long pos = off[blockIdx.x];
    for (int q = 0; q < wid; ++q) pos += wbase[q];
    for (uint32_t i0 = 0; i0 < kSub; i0 += 64) {
        const uint64_t v = base + wid * kSub + i0 + lane;
        const uint32_t wv = v < n ? w[v] : kInvalid;
        const bool in = wv != kInvalid;
        const uint64_t m = __ballot(in);
        const uint64_t at = pos + __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
        if (in && at < cap) {
            vo[at] = (IdT)v;
            ko[at] = (IdT)(wv >> 1);
            so[at] = (wv & 1u) ? 0 : 1;
        }
        pos += __popcll(m);
    }
}

// ---- GS_BIP_REFERENCE_LITERAL: the literal Candidates engine (bip_literal.hpp) as one workgroup ----
constexpr uint32_t kLitThreads = 256;

// the engine's execution context on the device: the workgroup, LDS for the block scan
struct LitX {
    uint32_t* scan;                                   // LDS [kLitThreads]
    __device__ uint32_t tid() const { return threadIdx.x; }
    __device__ uint32_t nt() const { return blockDim.x; }
    __device__ void sync() const { __syncthreads(); }
    __device__ uint32_t atomic_add(uint32_t* p, uint32_t v) const { return atomicAdd(p, v); }
    __device__ void atomic_min(uint32_t* p, uint32_t v) const { atomicMin(p, v); }
    __device__ void atomic_or(uint32_t* p, uint32_t v) const { atomicOr(p, v); }
    // exclusive prefix sum of v over the workgroup (Hillis-Steele in LDS), *total = the sum
    __device__ uint32_t scan_excl(uint32_t v, uint32_t* total) const {
        const uint32_t t = threadIdx.x, n = blockDim.x;
        scan[t] = v;
        __syncthreads();
        for (uint32_t off = 1; off < n; off <<= 1) {
            const uint32_t y = t >= off ? scan[t - off] : 0u;
            __syncthreads();
            scan[t] += y;
            __syncthreads();
        }
        *total = scan[n - 1];
        const uint32_t incl = scan[t];
        __syncthreads();
        return incl - v;
    }
};

// updateFunction.foldEdges over a batch, edge after edge (the rule is sequential; each edge's work
// is spread over the workgroup)
template <typename IdT>
__global__ __launch_bounds__(kLitThreads) void k_bipl_fold(lit::State S, const IdT* a, const IdT* b, uint64_t n, int aos) {
    __shared__ lit::Shared sh;
    __shared__ uint32_t scan[kLitThreads];
    LitX x{scan};
    lit::fold_edges(x, S, sh, a, b, n, aos != 0);
}

// into.merge(from) (Candidates.java:77-139)
__global__ __launch_bounds__(kLitThreads) void k_bipl_merge(lit::State S, lit::State F) {
    __shared__ lit::Shared sh;
    __shared__ uint32_t scan[kLitThreads];
    LitX x{scan};
    lit::merge_summaries(x, S, sh, F);
}

// restoreState: the snapshot's components, one run after another (lit::load_components)
__global__ __launch_bounds__(kLitThreads) void k_bipl_load(lit::State S, const uint32_t* rk, const uint64_t* ro,
                                                           uint32_t runs, const uint32_t* rv, const uint8_t* rs) {
    __shared__ lit::Shared sh;
    __shared__ uint32_t scan[kLitThreads];
    LitX x{scan};
    lit::load_components(x, S, sh, rk, ro, runs, rv, rs);
}

// the live (component, vertex, sign) entries: sort keys vertex << 32 | key (emission order: by
// vertex, then key) with their signs, and the emission checksum (bip.hip's formula, per entry)
__global__ __launch_bounds__(256) void k_bipl_collect(lit::State S, uint32_t nodes, uint64_t* __restrict__ keys,
                                                      uint8_t* __restrict__ signs, unsigned long long* __restrict__ acc) {
    unsigned long long sum = 0;
    for (uint32_t nd = blockIdx.x * blockDim.x + threadIdx.x; nd < nodes; nd += gridDim.x * blockDim.x) {
        const uint32_t cs = S.node_cs[nd], c = lit::slot_of(cs);
        if (!S.comp_alive[c]) continue;
        const uint32_t v = S.node_v[nd], k = S.comp_key[c], sg = lit::sign_of(cs);
        sum += pair_mix(v, ((uint64_t)k << 1) | sg);
        if (keys) {
            const unsigned long long at = atomicAdd(&acc[1], 1ull);
            keys[at] = ((uint64_t)v << 32) | k;
            signs[at] = (uint8_t)sg;
        }
    }
    atomicAdd(&acc[0], sum);
}

template <typename IdT>
__global__ __launch_bounds__(256) void k_bipl_split(const uint64_t* __restrict__ keys, const uint8_t* __restrict__ sg_in,
                                                    uint64_t n, IdT* __restrict__ v, IdT* __restrict__ k,
                                                    uint8_t* __restrict__ sg) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        v[i] = (IdT)(keys[i] >> 32);
        k[i] = (IdT)(keys[i] & 0xFFFFFFFFu);
        sg[i] = sg_in[i];
    }
}

static unsigned bgrid(uint64_t items, uint64_t per, unsigned capb) {
    uint64_t b = (items + per - 1) / per;
    if (b == 0) b = 1;
    return (unsigned)(b < capb ? b : capb);
}

}  // namespace gsgpu

using namespace gsgpu;

// device state of a GS_BIP_REFERENCE_LITERAL summary (bip_literal.hpp), in one allocation
struct LitDev {
    void* mem = nullptr;
    lit::State S{};
    lit::Ctl* hctl = nullptr;                     // pinned mirror of S.ctl
};

struct gs_bip {
    uint32_t cap = 0, id_bits = 64;
    int device = 0;
    LitDev* lit = nullptr;                     // GS_BIP_REFERENCE_LITERAL: the literal engine's state
    hipStream_t own = nullptr, stream = nullptr;
    uint32_t* w = nullptr;
    uint32_t* flags = nullptr;                 // [0] range error, [1] not bipartite
    unsigned long long* dscr = nullptr;        // reductions
    unsigned long long* hscr = nullptr;        // pinned mirror
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    void* stage = nullptr;
    size_t stage_bytes = 0;
    uint64_t edges_since_reset = 0;
    bool compressed = true;
};

namespace {

BipArgs bargs(gs_bip_t* h) { return BipArgs{h->w, h->cap, h->flags}; }

int bcheck(gs_bip_t* h) { return h ? GS_OK : fail(GS_ERR_INVALID, "null handle"); }

int bensure(void** p, size_t* have, size_t need) {
    if (*have >= need) return GS_OK;
    if (*p) { GS_HIP(hipFree(*p)); *p = nullptr; *have = 0; }
    if (hipMalloc(p, need) != hipSuccess) { (void)hipGetLastError(); return fail(GS_ERR_NOMEM, "hipMalloc(%zu) failed", need); }
    *have = need;
    return GS_OK;
}

// literal engine: its control words to the host, errors mapped to GS_ERR_* (the range flag is
// cleared once reported, as the union-find's is)
int lsync(gs_bip_t* h, int* bipartite) {
    lit::Ctl* c = h->lit->hctl;
    GS_HIP(hipMemcpyAsync(c, h->lit->S.ctl, sizeof(lit::Ctl), hipMemcpyDeviceToHost, h->stream));
    GS_HIP(hipStreamSynchronize(h->stream));
    if (bipartite) *bipartite = c->ok ? 1 : 0;
    if (c->err & lit::kErrCapacity)
        return fail(GS_ERR_CAPACITY, "reference-literal Candidates: entry capacity exhausted (%u nodes, %u components, %u "
                    "arena slots; gs_bip_create_ex entry_capacity)", h->lit->S.E, h->lit->S.C, h->lit->S.A);
    if (c->err & lit::kErrThrows)
        return fail(GS_ERR_INVALID, "reference-literal Candidates: Candidates.merge would throw here (an empty mergeBy "
                    "list, Candidates.java:156)");
    if (c->skipped) {
        GS_HIP(hipMemsetAsync(reinterpret_cast<char*>(h->lit->S.ctl) + offsetof(lit::Ctl, skipped), 0, sizeof(uint32_t), h->stream));
        return fail(GS_ERR_RANGE, "a vertex id outside [0, %u) was folded; such edges were skipped", h->cap);
    }
    return GS_OK;
}

// reads the flags; GS_ERR_RANGE if an out-of-range id was folded since the last check
int bsync(gs_bip_t* h, int* bipartite) {
    if (h->lit) return lsync(h, bipartite);
    uint32_t* hf = reinterpret_cast<uint32_t*>(h->hscr + 6);
    GS_HIP(hipMemcpyAsync(hf, h->flags, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
    GS_HIP(hipStreamSynchronize(h->stream));
    if (bipartite) *bipartite = hf[1] ? 0 : 1;
    if (hf[0]) {
        GS_HIP(hipMemsetAsync(h->flags, 0, sizeof(uint32_t), h->stream));
        return fail(GS_ERR_RANGE, "a vertex id outside [0, %u) was folded; such edges were skipped", h->cap);
    }
    return GS_OK;
}

int bcompress(gs_bip_t* h) {
    if (h->lit || h->compressed) return GS_OK;        // (the literal summary needs no compression)
    hipLaunchKernelGGL(k_bip_compress, dim3(bgrid(h->cap, 256, 16384)), dim3(256), 0, h->stream, h->w, h->cap);
    GS_HIP(hipGetLastError());
    h->compressed = true;
    return GS_OK;
}

template <typename IdT, bool AOS>
void bfold_launch(gs_bip_t* h, const IdT* a, const IdT* b, uint64_t n) {
    // young-forest split as for CC: few edges in flight while the forest is being built
    const uint64_t young = h->cap / 4;
    uint64_t off = 0;
    while (off < n) {
        uint64_t m = n - off;
        if (h->edges_since_reset < young)
            m = std::min(m, std::max<uint64_t>(std::min<uint64_t>(1ull << 18, young - h->edges_since_reset), 1));
        const IdT* pa = a + (AOS ? 2 * off : off);
        const IdT* pb = AOS ? nullptr : b + off;
        const dim3 grid(bgrid((m + 3) / 4, 256, 16384));
        const bool vec = std::is_same<IdT, uint32_t>::value && !AOS &&
                         ((reinterpret_cast<uintptr_t>(pa) | reinterpret_cast<uintptr_t>(pb)) & 15) == 0;
        if (vec) hipLaunchKernelGGL((k_bip_fold<IdT, AOS, true>), grid, dim3(256), 0, h->stream, pa, pb, m, bargs(h));
        else hipLaunchKernelGGL((k_bip_fold<IdT, AOS, false>), grid, dim3(256), 0, h->stream, pa, pb, m, bargs(h));
        h->edges_since_reset += m;
        off += m;
    }
}

int bfold(gs_bip_t* h, const void* a, const void* b, uint64_t n, bool aos) {
    GS_TRY(bcheck(h));
    if (n == 0) return GS_OK;
    if (!a || (!aos && !b)) return fail(GS_ERR_INVALID, "gs_bip_fold: null edge buffer");
    DeviceGuard g(h->device);
    h->compressed = false;
    const size_t esz = h->id_bits / 8;
    auto launch = [&](const void* x, const void* y, uint64_t m) {
        if (h->lit) {                                  // one workgroup, edge after edge
            if (h->id_bits == 32)
                hipLaunchKernelGGL(k_bipl_fold<uint32_t>, dim3(1), dim3(kLitThreads), 0, h->stream, h->lit->S,
                                   (const uint32_t*)x, (const uint32_t*)y, m, aos ? 1 : 0);
            else
                hipLaunchKernelGGL(k_bipl_fold<int64_t>, dim3(1), dim3(kLitThreads), 0, h->stream, h->lit->S,
                                   (const int64_t*)x, (const int64_t*)y, m, aos ? 1 : 0);
            return;
        }
        if (h->id_bits == 32) {
            if (aos) bfold_launch<uint32_t, true>(h, (const uint32_t*)x, nullptr, m);
            else bfold_launch<uint32_t, false>(h, (const uint32_t*)x, (const uint32_t*)y, m);
        } else {
            if (aos) bfold_launch<int64_t, true>(h, (const int64_t*)x, nullptr, m);
            else bfold_launch<int64_t, false>(h, (const int64_t*)x, (const int64_t*)y, m);
        }
    };
    if (is_device_pointer(a) && (aos || is_device_pointer(b))) {
        launch(a, b, n);
        GS_HIP(hipGetLastError());
        return GS_OK;
    }
    const uint64_t chunk = 1ull << 22;
    GS_TRY(bensure(&h->stage, &h->stage_bytes, chunk * esz * 2));
    for (uint64_t off = 0; off < n; off += chunk) {
        const uint64_t m = std::min(n - off, chunk);
        char* s0 = static_cast<char*>(h->stage);
        char* s1 = s0 + chunk * esz;
        if (aos) {
            GS_HIP(hipMemcpyAsync(s0, static_cast<const char*>(a) + off * esz * 2, m * esz * 2, hipMemcpyHostToDevice, h->stream));
        } else {
            GS_HIP(hipMemcpyAsync(s0, static_cast<const char*>(a) + off * esz, m * esz, hipMemcpyHostToDevice, h->stream));
            GS_HIP(hipMemcpyAsync(s1, static_cast<const char*>(b) + off * esz, m * esz, hipMemcpyHostToDevice, h->stream));
        }
        launch(s0, s1, m);
        GS_HIP(hipGetLastError());
    }
    return GS_OK;
}

// literal summary: every live (vertex, key, sign) entry, ordered by vertex then key (a vertex may
// belong to several components, see bip_literal.hpp); nothing when failed
int lemit(gs_bip_t* h, void* vertices, void* keys, uint8_t* signs, uint64_t cap, uint64_t* n_out) {
    int ok = 1;
    GS_TRY(lsync(h, &ok));
    const lit::Ctl c = *h->lit->hctl;
    const uint64_t total = ok ? c.live_entries : 0;
    *n_out = total;
    const uint64_t wn = std::min<uint64_t>(total, cap);
    if (wn) {
        size_t sort_bytes = 0;
        GS_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                   (const uint8_t*)nullptr, (uint8_t*)nullptr, (int)total, 0, 64, h->stream));
        const size_t kb = ((size_t)total * 8 + 255) & ~(size_t)255, sb = ((size_t)total + 255) & ~(size_t)255;
        const size_t esz = h->id_bits / 8;
        const size_t ob = ((size_t)wn * (2 * esz + 1) + 255) & ~(size_t)255;
        GS_TRY(bensure(&h->tmp, &h->tmp_bytes, 256 + 2 * kb + 2 * sb + ob + sort_bytes));
        char* base = static_cast<char*>(h->tmp);
        auto* acc = reinterpret_cast<unsigned long long*>(base);
        auto* ki = reinterpret_cast<uint64_t*>(base + 256);
        auto* ko = reinterpret_cast<uint64_t*>(base + 256 + kb);
        auto* si = reinterpret_cast<uint8_t*>(base + 256 + 2 * kb);
        auto* so = reinterpret_cast<uint8_t*>(base + 256 + 2 * kb + sb);
        char* out = base + 256 + 2 * kb + 2 * sb;
        void* st = out + ob;
        GS_HIP(hipMemsetAsync(acc, 0, 2 * sizeof(unsigned long long), h->stream));
        hipLaunchKernelGGL(k_bipl_collect, dim3(bgrid(c.n_nodes, 256, 1024)), dim3(256), 0, h->stream, h->lit->S,
                           c.n_nodes, ki, si, acc);
        GS_HIP(hipGetLastError());
        GS_HIP(hipcub::DeviceRadixSort::SortPairs(st, sort_bytes, (const uint64_t*)ki, ko, (const uint8_t*)si, so,
                                                   (int)total, 0, 64, h->stream));
        const bool dev = is_device_pointer(vertices) && is_device_pointer(keys) && is_device_pointer(signs);
        void* vo = dev ? vertices : out;
        void* kout = dev ? keys : out + wn * esz;
        uint8_t* sg = dev ? signs : reinterpret_cast<uint8_t*>(out + 2 * wn * esz);
        if (h->id_bits == 32)
            hipLaunchKernelGGL(k_bipl_split<uint32_t>, dim3(bgrid(wn, 256, 1024)), dim3(256), 0, h->stream,
                               (const uint64_t*)ko, (const uint8_t*)so, wn, (uint32_t*)vo, (uint32_t*)kout, sg);
        else
            hipLaunchKernelGGL(k_bipl_split<int64_t>, dim3(bgrid(wn, 256, 1024)), dim3(256), 0, h->stream,
                               (const uint64_t*)ko, (const uint8_t*)so, wn, (int64_t*)vo, (int64_t*)kout, sg);
        GS_HIP(hipGetLastError());
        if (!dev) {
            GS_HIP(hipMemcpyAsync(vertices, vo, wn * esz, hipMemcpyDeviceToHost, h->stream));
            GS_HIP(hipMemcpyAsync(keys, kout, wn * esz, hipMemcpyDeviceToHost, h->stream));
            GS_HIP(hipMemcpyAsync(signs, sg, wn, hipMemcpyDeviceToHost, h->stream));
        }
        GS_HIP(hipStreamSynchronize(h->stream));
    }
    if (total > cap) return fail(GS_ERR_CAPACITY, "gs_bip_emit_pairs: %llu entries, capacity %llu",
                                 (unsigned long long)total, (unsigned long long)cap);
    return GS_OK;
}

}  // namespace

extern "C" {

int gs_bip_create(gs_bip_t** out, uint64_t vertex_capacity, uint32_t id_bits, int device) {
    return gs_bip_create_ex(out, vertex_capacity, id_bits, device, 0u, 0ull);
}

int gs_bip_create_ex(gs_bip_t** out, uint64_t vertex_capacity, uint32_t id_bits, int device, uint32_t flags,
                     uint64_t entry_capacity) {
    if (!out) return fail(GS_ERR_INVALID, "gs_bip_create: null out");
    if (flags & ~(uint32_t)GS_BIP_REFERENCE_LITERAL) return fail(GS_ERR_INVALID, "gs_bip_create_ex: unknown flags 0x%x", flags);
    *out = nullptr;
    if (id_bits != 32 && id_bits != 64) return fail(GS_ERR_INVALID, "gs_bip_create: id_bits must be 32 or 64");
    if (vertex_capacity == 0 || vertex_capacity > kBipMaxCap)
        return fail(GS_ERR_INVALID, "gs_bip_create: vertex_capacity must be in [1, 2^31-1]");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return fail(GS_ERR_HIP, "gs_bip_create: no HIP device available");
    }
    if (device < 0 || device >= ndev) return fail(GS_ERR_INVALID, "gs_bip_create: device %d of %d", device, ndev);
    DeviceGuard g(device);
    gs_bip_t* h = new gs_bip_t();
    h->cap = (uint32_t)vertex_capacity;
    h->id_bits = id_bits;
    h->device = device;
    auto bail = [&](int rc) { gs_bip_destroy(h); return rc; };
    if (hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking) != hipSuccess) return bail(fail(GS_ERR_HIP, "hipStreamCreate failed"));
    h->stream = h->own;
    if (hipMalloc(&h->dscr, 8 * sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc(&h->hscr, 8 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return bail(fail(GS_ERR_NOMEM, "gs_bip_create: scratch allocation failed"));
    }
    if (flags & GS_BIP_REFERENCE_LITERAL) {
        // the literal engine: nodes E (component memberships ever made between resets), as many
        // component slots, an arena of 4 E member slots (component arrays double as they grow)
        const uint64_t E = entry_capacity ? entry_capacity : std::max<uint64_t>(16ull * h->cap, 4096);
        if (E > 0x7FFFFFFFull / 4) return bail(fail(GS_ERR_INVALID, "gs_bip_create_ex: entry_capacity too large"));
        h->lit = new LitDev();
        lit::State& S = h->lit->S;
        S.cap = h->cap;
        S.E = (uint32_t)E;
        S.C = (uint32_t)E;
        S.A = (uint32_t)(4 * E);
        const size_t cap = h->cap;
        size_t off = 0;
        auto take = [&](size_t bytes) { const size_t at = off; off += (bytes + 255) & ~(size_t)255; return at; };
        const size_t o_vhead = take(cap * 4), o_kslot = take(cap * 4), o_sv = take(cap * 4), o_keys = take(cap * 4),
                     o_ss = take(cap), o_ncs = take(E * 4), o_nv = take(E * 4), o_nn = take(E * 4),
                     o_ck = take(E * 4), o_ca = take(E * 4), o_cb = take(E * 4), o_csz = take(E * 4), o_ccap = take(E * 4),
                     o_cnt = take(E * 4), o_tch = take(E * 4), o_mw = take(E * 8), o_mws = take(E * 8),
                     o_arena = take(4 * E * 4), o_ctl = take(sizeof(lit::Ctl));
        if (hipMalloc(&h->lit->mem, off) != hipSuccess ||
            hipHostMalloc(&h->lit->hctl, sizeof(lit::Ctl), hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            return bail(fail(GS_ERR_NOMEM, "gs_bip_create_ex: %zu bytes for the reference-literal summary", off));
        }
        char* m = static_cast<char*>(h->lit->mem);
        S.vhead = (int32_t*)(m + o_vhead);
        S.kslot = (int32_t*)(m + o_kslot);
        S.sv = (uint32_t*)(m + o_sv);
        S.keys = (uint32_t*)(m + o_keys);
        S.ss = (uint8_t*)(m + o_ss);
        S.node_cs = (uint32_t*)(m + o_ncs);
        S.node_v = (uint32_t*)(m + o_nv);
        S.node_next = (int32_t*)(m + o_nn);
        S.comp_key = (uint32_t*)(m + o_ck);
        S.comp_alive = (uint32_t*)(m + o_ca);
        S.comp_base = (uint32_t*)(m + o_cb);
        S.comp_size = (uint32_t*)(m + o_csz);
        S.comp_cap = (uint32_t*)(m + o_ccap);
        S.cnt = (uint32_t*)(m + o_cnt);
        S.touched = (uint32_t*)(m + o_tch);
        S.mw = (uint64_t*)(m + o_mw);
        S.mws = (uint64_t*)(m + o_mws);
        S.arena = (int32_t*)(m + o_arena);
        S.ctl = (lit::Ctl*)(m + o_ctl);
    } else if (hipMalloc(&h->w, (size_t)h->cap * 4) != hipSuccess || hipMalloc(&h->flags, 16) != hipSuccess) {
        (void)hipGetLastError();
        return bail(fail(GS_ERR_NOMEM, "gs_bip_create: allocation of %u words failed", h->cap));
    }
    int rc = gs_bip_reset(h);
    if (rc != GS_OK) return bail(rc);
    if (hipStreamSynchronize(h->stream) != hipSuccess) return bail(fail(GS_ERR_HIP, "stream sync failed"));
    *out = h;
    return GS_OK;
}

int gs_bip_destroy(gs_bip_t* h) {
    if (!h) return GS_OK;
    DeviceGuard g(h->device);
    if (h->own) (void)hipStreamSynchronize(h->own);
    if (h->stream && h->stream != h->own) (void)hipStreamSynchronize(h->stream);
    for (void* p : {(void*)h->w, (void*)h->flags, (void*)h->dscr, h->tmp, h->stage})
        if (p) (void)hipFree(p);
    if (h->hscr) (void)hipHostFree(h->hscr);
    if (h->lit) {
        if (h->lit->mem) (void)hipFree(h->lit->mem);
        if (h->lit->hctl) (void)hipHostFree(h->lit->hctl);
        delete h->lit;
    }
    if (h->own) (void)hipStreamDestroy(h->own);
    delete h;
    return GS_OK;
}

int gs_bip_reset(gs_bip_t* h) {
    GS_TRY(bcheck(h));
    DeviceGuard g(h->device);
    h->edges_since_reset = 0;
    if (h->lit) {                                      // new Candidates(true): no component, f0 true
        lit::State& S = h->lit->S;
        GS_HIP(hipMemsetAsync(S.vhead, 0xFF, (size_t)S.cap * 4, h->stream));
        GS_HIP(hipMemsetAsync(S.kslot, 0xFF, (size_t)S.cap * 4, h->stream));
        GS_HIP(hipMemsetAsync(S.cnt, 0, (size_t)S.C * 4, h->stream));
        lit::Ctl c{};
        c.ok = 1;
        *h->lit->hctl = c;                             // (pinned: the copy reads it when it runs)
        GS_HIP(hipMemcpyAsync(S.ctl, h->lit->hctl, sizeof(c), hipMemcpyHostToDevice, h->stream));
        GS_HIP(hipStreamSynchronize(h->stream));       // (the pinned word is reused by lsync)
        return GS_OK;
    }
    GS_HIP(hipMemsetAsync(h->w, 0xFF, (size_t)h->cap * 4, h->stream));
    GS_HIP(hipMemsetAsync(h->flags, 0, 16, h->stream));
    h->edges_since_reset = 0;
    h->compressed = true;
    return GS_OK;
}

int gs_bip_set_stream(gs_bip_t* h, void* s) {
    GS_TRY(bcheck(h));
    h->stream = static_cast<hipStream_t>(s);
    return GS_OK;
}

int gs_bip_fold(gs_bip_t* h, const void* src, const void* dst, uint64_t n) { return bfold(h, src, dst, n, false); }
int gs_bip_fold_pairs(gs_bip_t* h, const void* pairs, uint64_t n) { return bfold(h, pairs, nullptr, n, true); }

int gs_bip_merge(gs_bip_t* into, gs_bip_t* from) {
    GS_TRY(bcheck(into));
    GS_TRY(bcheck(from));
    if (into == from) return GS_OK;
    if (into->device != from->device) return fail(GS_ERR_UNSUPPORTED, "gs_bip_merge: summaries on different devices");
    if (from->cap > into->cap) return fail(GS_ERR_RANGE, "gs_bip_merge: source capacity %u exceeds target %u", from->cap, into->cap);
    if ((into->lit == nullptr) != (from->lit == nullptr))
        return fail(GS_ERR_UNSUPPORTED, "gs_bip_merge: a reference-literal and an intended-semantics summary do not mix");
    DeviceGuard g(into->device);
    hipEvent_t e = nullptr;
    if (from->stream != into->stream) {
        GS_HIP(hipEventCreate(&e));
        GS_HIP(hipEventRecord(e, from->stream));
        GS_HIP(hipStreamWaitEvent(into->stream, e, 0));
    }
    into->compressed = false;
    if (into->lit)
        hipLaunchKernelGGL(k_bipl_merge, dim3(1), dim3(kLitThreads), 0, into->stream, into->lit->S, from->lit->S);
    else
        hipLaunchKernelGGL(k_bip_merge, dim3(bgrid(from->cap, 256, 16384)), dim3(256), 0, into->stream,
                           (const uint32_t*)from->w, from->cap, (const uint32_t*)from->flags, bargs(into));
    GS_HIP(hipGetLastError());
    if (e) {
        GS_HIP(hipEventRecord(e, into->stream));
        GS_HIP(hipStreamWaitEvent(from->stream, e, 0));
        GS_HIP(hipEventDestroy(e));
    }
    return GS_OK;
}

int gs_bip_close_window(gs_bip_t* h) {
    GS_TRY(bcheck(h));
    DeviceGuard g(h->device);
    return bcompress(h);
}

int gs_bip_status(gs_bip_t* h, int* bipartite, uint64_t* n_vertices, uint64_t* n_components) {
    uint64_t sum = 0;
    return gs_bip_checksum(h, &sum, bipartite, n_vertices, n_components);
}

// literal summary: (checksum over live entries, ok, entries, components); a failed summary is empty
int lstats(gs_bip_t* h, uint64_t* checksum, int* bipartite, uint64_t* n_entries, uint64_t* n_components) {
    int ok = 1;
    GS_TRY(lsync(h, &ok));
    const lit::Ctl c = *h->lit->hctl;
    uint64_t sum = 0;
    if (ok && c.n_nodes) {
        GS_HIP(hipMemsetAsync(h->dscr, 0, 2 * sizeof(unsigned long long), h->stream));
        hipLaunchKernelGGL(k_bipl_collect, dim3(bgrid(c.n_nodes, 256, 1024)), dim3(256), 0, h->stream, h->lit->S,
                           c.n_nodes, (uint64_t*)nullptr, (uint8_t*)nullptr, h->dscr);
        GS_HIP(hipGetLastError());
        GS_HIP(hipMemcpyAsync(h->hscr, h->dscr, sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream));
        GS_HIP(hipStreamSynchronize(h->stream));
        sum = h->hscr[0];
    }
    if (bipartite) *bipartite = ok;
    if (checksum) *checksum = ok ? sum : 0;
    if (n_entries) *n_entries = ok ? c.live_entries : 0;
    if (n_components) *n_components = ok ? c.live_comps : 0;
    return GS_OK;
}

int gs_bip_checksum(gs_bip_t* h, uint64_t* checksum, int* bipartite, uint64_t* n_vertices, uint64_t* n_components) {
    GS_TRY(bcheck(h));
    DeviceGuard g(h->device);
    if (h->lit) return lstats(h, checksum, bipartite, n_vertices, n_components);
    GS_TRY(bcompress(h));
    GS_HIP(hipMemsetAsync(h->dscr, 0, 3 * sizeof(unsigned long long), h->stream));
    hipLaunchKernelGGL(k_bip_stats, dim3(bgrid(h->cap, 256, 4096)), dim3(256), 0, h->stream, (const uint32_t*)h->w, h->cap, h->dscr);
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(h->hscr, h->dscr, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream));
    int bip = 1;
    GS_TRY(bsync(h, &bip));
    if (bipartite) *bipartite = bip;
    if (checksum) *checksum = h->hscr[2];
    if (n_vertices) *n_vertices = h->hscr[0];
    if (n_components) *n_components = h->hscr[1];
    return GS_OK;
}

int gs_bip_emit_pairs(gs_bip_t* h, void* vertices, void* keys, uint8_t* signs, uint64_t cap, uint64_t* n_out) {
    GS_TRY(bcheck(h));
    if (!n_out) return fail(GS_ERR_INVALID, "gs_bip_emit_pairs: null n_out");
    if (cap && (!vertices || !keys || !signs)) return fail(GS_ERR_INVALID, "gs_bip_emit_pairs: null output");
    DeviceGuard g(h->device);
    if (h->lit) return lemit(h, vertices, keys, signs, cap, n_out);
    GS_TRY(bcompress(h));
    const uint32_t nt = (uint32_t)((h->cap + kBipTile - 1) / kBipTile);
    const size_t esz = h->id_bits / 8;
    const size_t cnt_b = ((size_t)nt * 4 + 255) & ~(size_t)255, off_b = ((size_t)(nt + 1) * 8 + 255) & ~(size_t)255;
    GS_TRY(bensure(&h->tmp, &h->tmp_bytes, cnt_b + off_b));
    uint32_t* cnt = static_cast<uint32_t*>(h->tmp);
    uint64_t* off = reinterpret_cast<uint64_t*>(static_cast<char*>(h->tmp) + cnt_b);
    hipLaunchKernelGGL(k_bip_count, dim3(nt), dim3(256), 0, h->stream, (const uint32_t*)h->w, h->cap, cnt);
    hipLaunchKernelGGL(k_bip_scan, dim3(1), dim3(1024), 0, h->stream, (const uint32_t*)cnt, off, nt);
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(h->hscr, off + nt, 8, hipMemcpyDeviceToHost, h->stream));
    GS_TRY(bsync(h, nullptr));
    const uint64_t total = h->hscr[0];
    *n_out = total;
    const uint64_t wn = total < cap ? total : cap;
    if (wn) {
        const bool dev = is_device_pointer(vertices) && is_device_pointer(keys) && is_device_pointer(signs);
        void* vo = vertices;
        void* ko = keys;
        uint8_t* so = signs;
        if (!dev) {
            GS_TRY(bensure(&h->tmp, &h->tmp_bytes, cnt_b + off_b + wn * (2 * esz + 1)));
            off = reinterpret_cast<uint64_t*>(static_cast<char*>(h->tmp) + cnt_b);
            cnt = static_cast<uint32_t*>(h->tmp);
            hipLaunchKernelGGL(k_bip_count, dim3(nt), dim3(256), 0, h->stream, (const uint32_t*)h->w, h->cap, cnt);
            hipLaunchKernelGGL(k_bip_scan, dim3(1), dim3(1024), 0, h->stream, (const uint32_t*)cnt, off, nt);
            vo = static_cast<char*>(h->tmp) + cnt_b + off_b;
            ko = static_cast<char*>(vo) + wn * esz;
            so = static_cast<uint8_t*>(ko) + wn * esz;
        }
        if (h->id_bits == 32)
            hipLaunchKernelGGL(k_bip_scatter<uint32_t>, dim3(nt), dim3(256), 0, h->stream, (const uint32_t*)h->w, h->cap,
                               (const uint64_t*)off, (uint32_t*)vo, (uint32_t*)ko, so, wn);
        else
            hipLaunchKernelGGL(k_bip_scatter<int64_t>, dim3(nt), dim3(256), 0, h->stream, (const uint32_t*)h->w, h->cap,
                               (const uint64_t*)off, (int64_t*)vo, (int64_t*)ko, so, wn);
        GS_HIP(hipGetLastError());
        if (!dev) {
            GS_HIP(hipMemcpyAsync(vertices, vo, wn * esz, hipMemcpyDeviceToHost, h->stream));
            GS_HIP(hipMemcpyAsync(keys, ko, wn * esz, hipMemcpyDeviceToHost, h->stream));
            GS_HIP(hipMemcpyAsync(signs, so, wn, hipMemcpyDeviceToHost, h->stream));
        }
    }
    GS_TRY(bsync(h, nullptr));
    if (total > cap) return fail(GS_ERR_CAPACITY, "gs_bip_emit_pairs: %llu vertices, capacity %llu",
                                 (unsigned long long)total, (unsigned long long)cap);
    return GS_OK;
}

// restoreState (the Merger's ListCheckpointed state, SummaryAggregation.java:121-135): the summary
// becomes the snapshot's. A literal summary is loaded entry by entry (its components may share
// vertices, so no set of edges rebuilds it); an intended one is rebuilt from one parity edge per
// vertex, relative to its component key's own sign (a reversed merge can leave a key signed false,
// Candidates.java:155-182): a vertex signed unlike its key gets (v, key), one signed like it (other
// than the key) an edge to a vertex of the component signed the other way, a lone key its
// self-loop; a failed snapshot is the odd cycle 0-1-2 there (Candidates.fail(): empty, f0 false).
int gs_bip_restore(gs_bip_t* h, int bipartite, const void* vertices, const void* keys, const uint8_t* signs, uint64_t n) {
    GS_TRY(bcheck(h));
    if (n && (!vertices || !keys || !signs)) return fail(GS_ERR_INVALID, "gs_bip_restore: null entry array");
    DeviceGuard g(h->device);
    const size_t esz = h->id_bits / 8;
    std::vector<int64_t> v(n), k(n);
    std::vector<uint8_t> sg(n);
    if (n) {
        std::vector<char> raw(n * esz);
        auto get = [&](const void* src, size_t bytes, void* dst) -> int {
            if (is_device_pointer(src)) GS_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
            else std::memcpy(dst, src, bytes);
            return GS_OK;
        };
        for (int which = 0; which < 2; ++which) {
            GS_TRY(get(which ? keys : vertices, n * esz, raw.data()));
            std::vector<int64_t>& o = which ? k : v;
            for (uint64_t i = 0; i < n; ++i) {
                if (esz == 4) { uint32_t x; std::memcpy(&x, raw.data() + 4 * i, 4); o[i] = x; }
                else std::memcpy(&o[i], raw.data() + 8 * i, 8);
            }
        }
        GS_TRY(get(signs, n, sg.data()));
        for (uint64_t i = 0; i < n; ++i) {
            if (v[i] < 0 || v[i] >= (int64_t)h->cap || k[i] < 0 || k[i] >= (int64_t)h->cap)
                return fail(GS_ERR_INVALID, "gs_bip_restore: entry %llu (vertex %lld, key %lld) outside [0, %u)",
                            (unsigned long long)i, (long long)v[i], (long long)k[i], h->cap);
            sg[i] = sg[i] ? 1 : 0;
        }
    }
    GS_TRY(gs_bip_reset(h));
    if (h->lit) {
        if (!bipartite) {                              // Candidates.fail(): no component, f0 false
            lit::Ctl c = *h->lit->hctl;
            c.ok = 0;
            *h->lit->hctl = c;
            GS_HIP(hipMemcpyAsync(h->lit->S.ctl, h->lit->hctl, sizeof(c), hipMemcpyHostToDevice, h->stream));
            GS_HIP(hipStreamSynchronize(h->stream));
            return GS_OK;
        }
        if (n == 0) return GS_OK;
        std::vector<uint64_t> ord(n);
        for (uint64_t i = 0; i < n; ++i) ord[i] = i;
        std::sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) { return k[a] != k[b] ? k[a] < k[b] : v[a] < v[b]; });
        std::vector<uint32_t> rk, rv(n);
        std::vector<uint64_t> ro;
        std::vector<uint8_t> rs(n);
        for (uint64_t j = 0; j < n; ++j) {
            const uint64_t i = ord[j];
            if (j && k[i] == k[ord[j - 1]] && v[i] == v[ord[j - 1]])
                return fail(GS_ERR_INVALID, "gs_bip_restore: vertex %lld twice in component %lld", (long long)v[i], (long long)k[i]);
            if (!j || k[i] != k[ord[j - 1]]) {
                rk.push_back((uint32_t)k[i]);
                ro.push_back(j);
            }
            rv[j] = (uint32_t)v[i];
            rs[j] = sg[i];
        }
        ro.push_back(n);
        const lit::State& S = h->lit->S;
        if (n > S.E || rk.size() > S.C)
            return fail(GS_ERR_CAPACITY, "gs_bip_restore: %llu entries in %zu components, the summary holds %u / %u "
                        "(gs_bip_create_ex entry_capacity)", (unsigned long long)n, rk.size(), S.E, S.C);
        const size_t b_rk = (rk.size() * 4 + 255) & ~(size_t)255, b_ro = (ro.size() * 8 + 255) & ~(size_t)255,
                     b_rv = ((size_t)n * 4 + 255) & ~(size_t)255;
        GS_TRY(bensure(&h->tmp, &h->tmp_bytes, b_rk + b_ro + b_rv + n));
        char* base = static_cast<char*>(h->tmp);
        GS_HIP(hipMemcpy(base, rk.data(), rk.size() * 4, hipMemcpyHostToDevice));
        GS_HIP(hipMemcpy(base + b_rk, ro.data(), ro.size() * 8, hipMemcpyHostToDevice));
        GS_HIP(hipMemcpy(base + b_rk + b_ro, rv.data(), (size_t)n * 4, hipMemcpyHostToDevice));
        GS_HIP(hipMemcpy(base + b_rk + b_ro + b_rv, rs.data(), n, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_bipl_load, dim3(1), dim3(kLitThreads), 0, h->stream, h->lit->S, (const uint32_t*)base,
                           (const uint64_t*)(base + b_rk), (uint32_t)rk.size(), (const uint32_t*)(base + b_rk + b_ro),
                           (const uint8_t*)(base + b_rk + b_ro + b_rv));
        GS_HIP(hipGetLastError());
        return lsync(h, nullptr);
    }
    std::vector<int64_t> src, dst;
    if (!bipartite) {
        if (h->cap < 3) return fail(GS_ERR_INVALID, "gs_bip_restore: a failed snapshot needs vertex_capacity >= 3");
        src = {0, 1, 2};
        dst = {1, 2, 0};
    } else {
        std::unordered_map<int64_t, uint8_t> ksign;   // component key -> the key vertex's own sign
        std::unordered_map<int64_t, int64_t> other;   // component key -> a vertex signed unlike the key
        for (uint64_t i = 0; i < n; ++i)
            if (v[i] == k[i]) ksign[k[i]] = sg[i];
        for (uint64_t i = 0; i < n; ++i) {
            auto ks = ksign.find(k[i]);
            if (ks == ksign.end())
                return fail(GS_ERR_INVALID, "gs_bip_restore: component key %lld is not among the vertices", (long long)k[i]);
            if (sg[i] != ks->second) other.emplace(k[i], v[i]);
        }
        src.reserve(n);
        dst.reserve(n);
        for (uint64_t i = 0; i < n; ++i) {
            src.push_back(v[i]);
            if (sg[i] != ksign[k[i]]) dst.push_back(k[i]);
            else if (v[i] != k[i]) {
                auto o = other.find(k[i]);
                if (o == other.end())
                    return fail(GS_ERR_INVALID, "gs_bip_restore: component %lld has vertices on one side only", (long long)k[i]);
                dst.push_back(o->second);
            } else dst.push_back(v[i]);
        }
    }
    if (!src.empty()) {
        if (esz == 4) {
            std::vector<uint32_t> a(src.begin(), src.end()), b(dst.begin(), dst.end());
            GS_TRY(bfold(h, a.data(), b.data(), a.size(), false));
            GS_HIP(hipStreamSynchronize(h->stream));   // (the staged copies read the host vectors)
        } else {
            GS_TRY(bfold(h, src.data(), dst.data(), src.size(), false));
            GS_HIP(hipStreamSynchronize(h->stream));
        }
    }
    GS_TRY(gs_bip_close_window(h));
    return bsync(h, nullptr);
}

int gs_bip_sync(gs_bip_t* h) {
    GS_TRY(bcheck(h));
    DeviceGuard g(h->device);
    return bsync(h, nullptr);
}

}  // extern "C"
