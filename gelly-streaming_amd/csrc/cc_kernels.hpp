// cc_kernels.hpp — device code for streaming Connected Components on gfx950 (wave64).
//
// State: one dense uint32 parent[] per summary (HBM-resident, vertex_capacity words).
//   parent[v] == kInvalid      v is not in the summary (DisjointSet.matches has no key v)
//   parent[v] == v             v is a root
//   parent[v] <  v             v hangs below parent[v]
// Hooking always puts the LARGER root under the SMALLER one (atomicCAS on the larger root's
// word), so parent[v] <= v holds for every seen v and every root is the minimum id of its tree:
// after full compression parent[] *is* the canonical (min-id) label array the reference's
// emissions canonicalise to. DisjointSet.java:92-118 decides by rank instead; its trees differ,
// its components (and hence canonical labels) do not.
//
// Visibility (8 XCDs, per-XCD L2s not coherent with each other, per-CU L1s never refreshed by
// other CUs' stores): plain loads of parent[] may return a stale (older) word. Every older value
// of parent[x] is an ancestor of x (or x itself, or kInvalid), so a stale read can only shorten a
// walk. EVERY store to parent[] / mark[] inside a launch where other workgroups also write is a
// device-scope atomic, executed at the memory side: hooks are atomicCAS (a failed hook retries
// from the true parent), path halving is a no-return atomicMin (parents only ever decrease), marks
// are atomicOr. A plain store would sit in the writer's XCD L2 as a dirty line and, written back
// later, could overwrite a hook that another XCD made meanwhile on the same line; at RMAT-22 scale
// that lost unions (tests/test_gpu_parity.py::test_full_size_rmat_properties). Plain stores are
// used only where one workgroup owns every word of the line it writes (k_compress, k_export).
#pragma once

#include "common.hpp"

namespace gsgpu {

// Root of x, given px = a parent[x] value already read. Walks with intermediate pointer jumping
// (each visited word gets its grandparent) and stops at the first word that is not strictly
// smaller than its index: a root, or a stale kInvalid read from L1 of a vertex another CU has
// just initialised (treated as a root; a hook on it is then decided by the CAS, which sees the
// true word). A non-root's parent is always < its index, so px >= x covers both cases and no
// walk ever indexes parent[kInvalid].
// halve = false: a read-only walk (no stores into words other walks share: in a young forest the
// halving atomics on hub ancestors serialise at the memory-side atomic unit).
__device__ __forceinline__ uint32_t find_root(uint32_t* __restrict__ parent, uint32_t x, uint32_t px, bool halve = true) {
    if (px >= x) return x;
    uint32_t prev = x, cur = px, next;
    while (cur > (next = parent[cur])) {
        if (halve) __hip_atomic_fetch_min(&parent[prev], next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        prev = cur;
        cur = next;
    }
    return cur;
}

__device__ __forceinline__ void set_mark(uint32_t* __restrict__ mark, uint32_t v) {
    __hip_atomic_fetch_or(&mark[v >> 5], 1u << (v & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Measured and dropped (profiles/r02_g, r02_i): a new vertex hooked straight under the giant's
// root setting its gbits bit instead (no close visit: closes -240 us per step) made the steady fold
// 12 us slower per window — atomics into the bitmap the filter is reading push its lines out of
// the L2s; skipping both bits left those vertices out of the filter (+4 us per steady window).
// first touch: v's bit in the seen bitmap. sbits == nullptr: not kept by this launch (big young
// folds: the next close is a full pass that rebuilds the bitmap from parent[], cc_api.hip
// launch_fold) — one device-scope atomic less per new vertex
__device__ __forceinline__ void set_seen(uint32_t* __restrict__ sbits, uint32_t v) {
    if (sbits) set_mark(sbits, v);
}

// Read-only root walk (no writes) for find() on const state.
__device__ __forceinline__ uint32_t find_root_ro(const uint32_t* __restrict__ parent, uint32_t x) {
    uint32_t cur = x, next;
    while (cur > (next = parent[cur])) cur = next;
    return cur;
}

// First touch of v (makeSet, DisjointSet.java:53-56): kInvalid -> v, and v's bit in the seen
// bitmap (read by the incremental close). Returns v's parent word.
__device__ __forceinline__ uint32_t make_set(uint32_t* __restrict__ parent, uint32_t* __restrict__ sbits,
                                             uint32_t v, uint32_t pv) {
    if (pv != kInvalid) return pv;
    const uint32_t old = atomicCAS(&parent[v], kInvalid, v);
    if (old != kInvalid) return old;
    set_seen(sbits, v);
    return v;
}

// union(u, v) given the parent words read by the caller. Returns the vertex the partial-summary
// export must carry (MARK: the root it hooked, or a self-loop's first touch; kInvalid if none):
// the caller appends it to the handle's hook log (log_append).
// per-thread diagnostic counters (GSGPU_FOLD_STATS=1 builds the STATS variant of k_fold)
struct FoldStats {
    uint32_t early = 0, hooks = 0, casfail = 0, inits = 0;
};

// hbits (or null): the hooked-root bitmap of a fold before any giant exists (k_compress: the full
// pass that must follow reads it instead of every vertex's grandparent) — a root that stops being a
// root here gets its bit
// nl (or null): a logging fold (touch log, below) also collects the vertices this edge
// first-touches (at most two)
struct NewV {
    uint32_t a = kInvalid, b = kInvalid;
};
__device__ __forceinline__ void first_touch(uint32_t* __restrict__ sbits, NewV* nl, uint32_t x) {
    if (nl) {
        if (nl->a == kInvalid) nl->a = x;
        else nl->b = x;
    }
    set_seen(sbits, x);
}

template <bool MARK, bool STATS = false>
__device__ __forceinline__ uint32_t union_edge(uint32_t* __restrict__ parent, uint32_t* __restrict__ sbits,
                                               uint32_t u, uint32_t v, uint32_t pu, uint32_t pv,
                                               FoldStats* st = nullptr, bool halve = true,
                                               uint32_t* __restrict__ hbits = nullptr, NewV* nl = nullptr) {
    if (u == v) {                                   // union(u,u): makeSet only
        if (pu == kInvalid) {
            const uint32_t old = atomicCAS(&parent[u], kInvalid, u);
            if (old == kInvalid) {
                first_touch(sbits, nl, u);
                if (MARK) return u;
            }
        }
        return kInvalid;
    }
    // A side whose word was read as kInvalid is a fresh vertex: it is a root of its own, and if
    // it ends up the larger root it is hooked straight from kInvalid (one CAS instead of an
    // init CAS + a hook CAS). Only a fresh SMALLER root must be initialised before anything
    // hangs below it. The CAS decides in every case: a stale kInvalid read fails and retries.
    bool fu = pu == kInvalid, fv = pv == kInvalid;
    if (STATS) st->inits += fu + fv;
    if (!fu && !fv && pu == pv) {                   // common parent: already one component
        if (STATS) ++st->early;
        return kInvalid;
    }
    uint32_t ru = fu ? u : find_root(parent, u, pu, halve);
    uint32_t rv = fv ? v : find_root(parent, v, pv, halve);
    while (ru != rv) {
        const bool uhi = ru > rv;
        const uint32_t hi = uhi ? ru : rv, lo = uhi ? rv : ru;
        bool& hf = uhi ? fu : fv;                   // fresh flags follow their side
        bool& lf = uhi ? fv : fu;
        if (lf) {                                   // the smaller root must exist first
            const uint32_t old = atomicCAS(&parent[lo], kInvalid, lo);
            lf = false;
            if (old == kInvalid) {
                first_touch(sbits, nl, lo);
            } else if (old != lo) {                 // initialised and hooked meanwhile
                const uint32_t r = find_root(parent, old, parent[old], halve);
                if (uhi) rv = r; else ru = r;
                continue;
            }
        }
        const uint32_t expect = hf ? kInvalid : hi;
        const uint32_t old = atomicCAS(&parent[hi], expect, lo);
        if (old == expect) {                        // hooked: hi is no longer a root
            if (hf) first_touch(sbits, nl, hi);
            else if (hbits) set_mark(hbits, hi);    // (a fresh hi never had children: no mark)
            if (STATS) ++st->hooks;
            return MARK ? hi : kInvalid;
        }
        if (STATS) ++st->casfail;
        hf = false;
        if (old == hi) continue;                    // was fresh, became a root meanwhile
        if (old == kInvalid) { hf = true; continue; }   // defensive: never reached by a walk result
        // hi was hooked meanwhile: continue from its true parent (old < hi, strictly
        // decreasing, so the loop ends)
        const uint32_t r = find_root(parent, old, parent[old], halve);
        if (uhi) ru = r; else rv = r;
    }
    return kInvalid;
}


// Hook log (GS_CC_TRACK_MARKS): the vertices a partial-summary export carries, appended in
// launch order. Wave-aggregated: one atomicAdd on the log length per wave call (the active lanes'
// entries are written contiguously), so a window's few hooks cost no per-hook same-address atomic
// and the export reads just the log instead of scanning a V-bit bitmap. Works with any set of
// active lanes (ballots over the exec mask). Every vertex is hooked at most once and first-touched
// by a self-loop at most once between resets, so 2 x capacity entries never overflow.
template <int EPT>
__device__ __forceinline__ void log_append(uint32_t* __restrict__ log, unsigned long long* __restrict__ len,
                                           const uint32_t (&m)[EPT]) {
    const uint64_t lt = (1ull << __lane_id()) - 1;
    uint64_t masks[EPT];
    uint32_t total = 0;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        masks[k] = __ballot(m[k] != kInvalid);
        total += (uint32_t)__popcll(masks[k]);
    }
    if (total == 0) return;                          // uniform over the active lanes
    const uint64_t active = __ballot(1);
    const int leader = __ffsll((long long)active) - 1;
    uint32_t lo = 0, hi = 0;
    if ((int)__lane_id() == leader) {
        const unsigned long long b = atomicAdd(len, (unsigned long long)total);
        lo = (uint32_t)b;
        hi = (uint32_t)(b >> 32);
    }
    lo = __shfl(lo, leader, 64);
    hi = __shfl(hi, leader, 64);
    uint64_t pos = ((uint64_t)hi << 32) | lo;
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        if (m[k] != kInvalid) log[pos + __popcll(masks[k] & lt)] = m[k];
        pos += __popcll(masks[k]);
    }
}

// ---- list-mode closes (small windows) ----
// While the seen vertices outside the giant are few (config 5: ~10^4 of 2^24), a close visits a
// list of them (the NGL) plus the window's first touches (the touch log) instead of scanning three
// V-bit bitmaps: the close follows the window, not V.
// Touch log: one slot per fold wave (kSlotWords words, whole 128-B lines: word 0 the count, then up
// to 2 x 64 first touches), written by that wave alone with plain stores, no atomic (a returning
// atomic per wave put ~1 us on config 5's fold). The host numbers the slots of an interval's folds.
// A logging fold still sets the seen bits, so whether the close can take the list (below) is the
// close's own decision: a fold reads no control word (two more dependent loads at the head of a
// 6 us launch cost ~1 us).
// NGL: (vertex, label) pairs in kListSub sub-lists (sub-list = the close's workgroup index mod
// kListSub), appended one atomic per wave, so that the appends spread over kListSub count words. An
// entry whose label is still a root keeps it (parent[v] is that label since the last close): one
// read of parent[label] per entry instead of parent[v] then parent[parent[v]].
// Control words (one array per handle, ListCtl below), by close number c (interval c = the folds
// between close c-1 and close c):
//   NC(k, s)   entries of NGL sub-list s written by close c with (c + 1) % 3 == k
//   LVALID(k)  close c-1 built a complete NGL with a giant, expecting logging folds (list_next)
//   LOVF(k)    an NGL sub-list overflowed (the list is incomplete: no list close)
// Close c reads index c % 3, appends (c + 1) % 3 and zeroes what no launch before close c + 1
// reads: NC / LOVF at (c + 2) % 3.
constexpr uint32_t kListSub = 256;
constexpr uint32_t kSlotWords = 160;                 // 1 + 128 entries, rounded up to 5 lines
struct ListCtl {
    __host__ __device__ static constexpr uint32_t NC(uint32_t k) { return k * kListSub; }
    __host__ __device__ static constexpr uint32_t LVALID(uint32_t k) { return 3 * kListSub + 32 * k; }
    __host__ __device__ static constexpr uint32_t LOVF(uint32_t k) { return 3 * kListSub + 128 + 32 * k; }
    static constexpr uint32_t kWords = 3 * kListSub + 256;
};

// Appends the lanes' entries (m[k].x != kInvalid) to a sub-list of capacity cap: one atomicAdd per
// wave call (any set of active lanes). Entries past cap are dropped and *ovf is set; the count keeps
// growing (readers take min(count, cap) and check ovf).
template <int N>
__device__ __forceinline__ void list_append(uint2* __restrict__ list, uint32_t* __restrict__ cnt, uint32_t cap,
                                            uint32_t* __restrict__ ovf, const uint2 (&m)[N]) {
    const uint64_t lt = (1ull << __lane_id()) - 1;
    uint64_t masks[N];
    uint32_t total = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        masks[k] = __ballot(m[k].x != kInvalid);
        total += (uint32_t)__popcll(masks[k]);
    }
    if (total == 0) return;                          // uniform over the active lanes
    const uint64_t active = __ballot(1);
    const int leader = __ffsll((long long)active) - 1;
    uint32_t base = 0;
    if ((int)__lane_id() == leader) {
        base = atomicAdd(cnt, total);
        if (base + total > cap) atomicOr(ovf, 1u);
    }
    uint32_t pos = __shfl(base, leader, 64);
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const uint32_t at = pos + (uint32_t)__popcll(masks[k] & lt);
        if (m[k].x != kInvalid && at < cap) list[at] = m[k];
        pos += (uint32_t)__popcll(masks[k]);
    }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct RangeCheck {
    uint32_t cap;
    uint32_t* err;
};

template <typename IdT>
__device__ __forceinline__ bool id_ok(IdT x, uint32_t cap) {
    return static_cast<uint64_t>(x) < static_cast<uint64_t>(cap) &&
           !(sizeof(IdT) == 8 && static_cast<int64_t>(x) < 0);
}

constexpr int kFoldThreads = 256;
constexpr int kEdgesPerThread = 4;          // default; k_fold takes EPT as a template parameter

// Giant-component filter (Afforest's "skip the largest component", made streaming): after every
// close_window, gbits[v] = 1 iff v's canonical label == *giant, a root picked by sampling
// (k_pick_giant). Components only ever merge until reset, so two set bits always mean "already
// one component" and the edge needs no parent[] access at all. The bitmap is V/8 bytes (8 MiB at
// 2^26 vertices: L2 / Infinity-Cache resident) where parent[] is V*4 bytes (HBM-bound gathers).
struct FoldArgs {
    uint64_t n;
    uint32_t* parent;
    uint32_t* mark;                       // hook log (GS_CC_TRACK_MARKS, marking on), or null
    uint32_t* sbits;
    const uint32_t* gbits;
    const uint32_t* giant;
    RangeCheck rc;
    unsigned long long* stats;   // STATS: [valid, filtered, early, hooks, casfail, inits]
    uint32_t halve = 1;          // path halving in root walks (find_root)
    unsigned long long* work = nullptr;   // k_fold: dynamic chunk counter (young forest), or null
    unsigned long long* mark_len = nullptr;   // MARK: the hook log's length word (mark = the log)
    uint32_t* cbits = nullptr;   // ring folds: vertices claimed straight under the giant root (k_compress)
    uint32_t* hbits = nullptr;   // hooked-root bitmap, used by the kernel only while no giant exists
    // logging fold (k_fold, one edge per thread, one pass): the touch-log slot of this launch's
    // wave 0; in the kernel, tlog is the wave's own slot and tcnt its entry count in LDS
    uint32_t* tlog = nullptr;
    uint32_t* tcnt = nullptr;
    uint32_t combine = 0;        // pair / survivor folds: wave-combined hooks of one root word (combine_hooks)
};

// A wave's first touches (t[k] != kInvalid) appended to its touch-log slot: ballots over the active
// lanes, the running count in LDS (every lane of a wave calls this at most once per launch).
template <int N>
__device__ __forceinline__ void slot_append(uint32_t* __restrict__ slot, uint32_t* tcnt, const uint32_t (&t)[N]) {
    const uint64_t lt = (1ull << __lane_id()) - 1;
    uint64_t masks[N];
    uint32_t total = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        masks[k] = __ballot(t[k] != kInvalid);
        total += (uint32_t)__popcll(masks[k]);
    }
    if (total == 0) return;
    uint32_t pos = *tcnt;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        if (t[k] != kInvalid) slot[1 + pos + __popcll(masks[k] & lt)] = t[k];
        pos += (uint32_t)__popcll(masks[k]);
    }
    const uint64_t active = __ballot(1);
    if ((int)__lane_id() == __ffsll((long long)active) - 1) *tcnt = pos;
}

// ---- LDS hot set (steady state) ----
// The filter's two gbits lookups per edge miss L2 half the time (an 8 MiB bitmap against a 4 MiB
// L2 per XCD) and the Infinity-Cache transfers of those misses bound the steady fold. The most
// frequent endpoints of a power-law stream are few: a 128 KiB exact set of giant-component
// members, copied into every workgroup's LDS at launch, answers ~1/3 of the lookups of an RMAT-26
// window from LDS (tools/hot_lab.hip: 268 -> 225 us per 2^24 edges).
// Layout: 2^14 buckets x 4 slots of 16-bit remainders. With ids < 2^B (B = hot_bits, 20..29),
// h = v * kHotMul mod 2^B (odd multiplier: a bijection), bucket = h >> (B - 14), slot value =
// (h mod 2^(B-14)) + 1; (bucket, slot value) <-> v is one-to-one, so membership is exact. 0 = empty.
// Exactness (and k_compress clearing the table when the giant becomes another component) is
// needed for CORRECTNESS, not only speed: a hit stands in for v's gbits bit, a hit on both
// endpoints drops the edge, and a hit on one endpoint makes the survivor's union start from the
// giant root instead of parent[v] (union_group_g). The same holds for the warm set.
// Entries are only ever added (a 0 half-word CASed to a remainder) and every entry is a vertex
// whose gbits bit was set, i.e. a member of the giant component; components only merge until
// reset, so an entry stays a member while the giant is the same component (k_pick_giant clears
// the table when a re-sample picks another one). Filling: each steady fold launch inserts the
// filter-confirmed endpoints of its first kHotSampleEdges edges into free slots; hubs appear
// first in any prefix of a power-law stream, so the table fills with them.
constexpr int kHotBucketBits = 14;
constexpr uint32_t kHotBuckets = 1u << kHotBucketBits;
constexpr uint32_t kHotMul = 0x9E3779B1u;
constexpr int kHotThreads = 1024;
constexpr uint64_t kHotSampleEdges = 1u << 18;

__device__ __forceinline__ uint32_t hot_hash(uint32_t v, uint32_t B) {
    return (v * kHotMul) & ((B >= 32) ? ~0u : ((1u << B) - 1));
}

// Slot formats. 4 x 16 bits (any B up to 29), or, when the remainder fits 12 bits (B <= 26),
// 5 x 12 bits packed in the bucket's 64 bits: 80 K entries instead of 64 K (an ideal
// frequency-ordered set answers 35.3 % instead of 32.4 % of an RMAT-26 window's lookups). The
// one remainder that does not fit (r + 1 = 4096) can never enter: 1 id in 4096.
// A probe in two halves (bucket index + slot value, then the compare), so a thread's LDS bucket
// reads all issue before the first compare. five is uniform: both formats are compared and
// selected without a branch.
__device__ __forceinline__ uint32_t hot_bucket(uint32_t v, uint32_t B, uint32_t& r) {
    const uint32_t h = hot_hash(v, B);
    const uint32_t rb = B - kHotBucketBits;
    r = (h & ((1u << rb) - 1)) + 1;
    return h >> rb;
}
// Any slot == r, by the SWAR zero-field test on x ^ (r in every field): ((z - ones) & ~z & highs)
// is non-zero iff some field of z is zero (a borrow can only flag fields above a true zero
// field, so "any" is exact). Empty slots (0) never equal r >= 1; r = 4096 does not fit 12 bits
// and never matches (it never enters either).
__device__ __forceinline__ bool hot_match(uint2 w, uint32_t r, bool five) {
    const uint64_t x = ((uint64_t)w.y << 32) | w.x;
    constexpr uint64_t kOnes5 = 0x001001001001001ull, kHigh5 = 0x800800800800800ull;
    constexpr uint64_t kOnes4 = 0x0001000100010001ull, kHigh4 = 0x8000800080008000ull;
    const uint64_t ones = five ? kOnes5 : kOnes4, high = five ? kHigh5 : kHigh4;
    const uint64_t z = x ^ ((uint64_t)r * ones);
    return (((z - ones) & ~z & high) != 0) & (!five | (r <= 0xFFFu));
}

// add v to the global table if a slot of its bucket is free (a full bucket drops it)
__device__ inline void hot_insert(uint2* gtab, uint32_t v, uint32_t B, bool five) {
    const uint32_t h = hot_hash(v, B);
    const uint32_t rb = B - kHotBucketBits;
    const uint32_t r = (h & ((1u << rb) - 1)) + 1;
    if (five) {
        if (r > 0xFFFu) return;
        unsigned long long* p = reinterpret_cast<unsigned long long*>(gtab + (h >> rb));
        unsigned long long x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int attempt = 0; attempt < 6; ++attempt) {
            int empty = -1;
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const uint32_t fk = (uint32_t)(x >> (12 * k)) & 0xFFFu;
                if (fk == r) return;
                if (fk == 0 && empty < 0) empty = k;
            }
            if (empty < 0) return;                           // bucket full
            const unsigned long long want = x | ((unsigned long long)r << (12 * empty));
            const unsigned long long old = atomicCAS(p, x, want);
            if (old == x) return;
            x = old;
        }
        return;
    }
    uint32_t* words = reinterpret_cast<uint32_t*>(gtab + (h >> rb));
#pragma unroll
    for (int wi = 0; wi < 2; ++wi) {
        uint32_t x = __hip_atomic_load(&words[wi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int attempt = 0; attempt < 4; ++attempt) {
            const uint32_t lo = x & 0xFFFFu, hi = x >> 16;
            if (lo == r || hi == r) return;
            if (lo && hi) break;                             // this word is full
            const uint32_t want = lo ? (x | (r << 16)) : (x | r);
            const uint32_t old = atomicCAS(&words[wi], x, want);
            if (old == x) return;
            x = old;
        }
    }
}

// Admission: a sampled giant member enters the hot set on its second sighting. `cand` is a
// direct-mapped table of the last sampled id per slot (overwritten on collision), so an id gets
// in only if it recurs before another sampled id lands on its slot: ids are admitted roughly in
// order of frequency, the hubs within the first sampled window. Plain racing stores are fine
// here: any value in a slot is only a candidate.
constexpr uint32_t kHotCandBits = 20;                // 2^20 candidate slots (4 MiB)
struct HotArgs {
    uint2* table;       // global master copy (kHotBuckets uint2), nullptr = no hot set
    uint32_t bits;      // B: every id < 2^B
    uint32_t* cand;     // 2^kHotCandBits candidate slots
    uint64_t sample_edges = kHotSampleEdges;   // admission offers endpoints of a launch's first edges
    uint32_t* budget = nullptr;                // admitting launches left (device word, see below)
    uint32_t periodic = 0;                     // the host's periodic refresh: admit in this launch
    uint32_t five = 0;                         // slot format: 5 x 12 bits (B <= 26) instead of 4 x 16
    uint32_t thresh = 2;                       // sightings before admission (> 2 needs B <= 26;
                                               // the host passes 3: steady window 233 -> 229 us)
    uint32_t* warm = nullptr;                  // warm set (2^warm_bits words), nullptr = none
    uint32_t warm_bits = 0;                    // log2(warm buckets), B - 8 <= warm_bits <= B
    const uint32_t* warm_valid = nullptr;      // device word: warm set built for the current giant
    uint32_t* wkeys = nullptr;                 // warm build: endpoint keys, 512 per wave step (count launches only)
    unsigned long long* wctl = nullptr;        // warm build: edges counted (written by count launches)
    uint64_t count_edges = 0;                  // count this launch's first edges (if !*warm_valid)
    uint32_t clocks = 0;                       // GSGPU_RING_CLOCKS: launch k_fold_ring's CLK instance
};

// ---- warm set (L2-resident second tier) ----
// Ids ranked ~80K..2M by frequency answer ~45 % of an RMAT-26 window's lookups (top 80K: 38 %,
// top 2M: 82 %), but do not fit LDS. The warm set holds them in a global table small enough to
// stay in every XCD's 4 MiB L2 next to the bitmap lines (2 MiB at 2^26 ids), one 4-B word per
// probe: 2^wb buckets x 4 slots of 8 bits, h = v * kWarmMul mod 2^B (odd multiplier: a
// bijection), bucket = h >> (B - wb), slot value = (h mod 2^(B - wb)) + 1; exact like the hot set. An LDS miss
// probes it before gbits, so a warm hit costs an L2 hit instead of (half the time) an
// Infinity-Cache line fill. Built from endpoint counts of one ring launch's
// first count_edges edges (LDS misses confirmed in the giant), hottest first (k_warm_part below);
// valid (hot.warm_valid) while the giant is the same component, like the hot set.
constexpr uint32_t kWarmMul = 0x85EBCA6Bu;
// wb = log2(buckets); remainders of B - wb <= 8 bits, slot value r = rem + 1 in [1, 256]: the one
// value that does not fit a byte (256: 1 id in 256 when B - wb = 8) never enters nor matches.
__device__ __forceinline__ uint32_t warm_hash(uint32_t v, uint32_t B) { return (v * kWarmMul) & ((1u << B) - 1); }
// A warm probe in two halves (word index + slot value, then the compare on the loaded word), so
// the probes of a thread's LDS misses are all in flight together (written as one `hit || probe`
// expression, the short-circuit put each load in a branch of its own with its wait inside: one L2
// round trip after the other, 8 per thread and pass of the ring fold)
__device__ __forceinline__ uint32_t warm_word(uint32_t v, uint32_t B, uint32_t wb, uint32_t& r) {
    const uint32_t h = warm_hash(v, B);
    const uint32_t rb = B - wb;
    r = (h & ((1u << rb) - 1)) + 1;
    return h >> rb;
}
__device__ __forceinline__ bool warm_match(uint32_t w, uint32_t r) {
    const uint32_t x = w ^ (r * 0x01010101u);
    return (r <= 0xFFu) & (((x - 0x01010101u) & ~x & 0x80808080u) != 0);   // no short-circuit branch
}
// Admission cadence. Offering a launch's first 2^18 edges costs ~28 us per RMAT-26 window (the
// candidate table's atomics); the hubs are stable, so a launch admits only while *budget > 0
// (kHotAdmitLaunches after reset or after k_compress clears the set for a new giant) or when the
// host's periodic refresh (every kHotAdmitEvery ring launches) asks: steady window 266 -> 240 us.
constexpr uint32_t kHotAdmitLaunches = 4;           // 8 -> 4: windows 2-12 -110 us, steady = (r02_ax/ay)
// every 64th (was 16th): 0.4-0.8 % faster per step on RMAT-26 (round-1 sweep: 16 / 32 / 64 /
// never = 18.77 / 18.68 / 18.65 / 18.61 ms); a refresh is kept for streams whose hubs drift
constexpr uint32_t kHotAdmitEvery = 64;

__device__ __forceinline__ void hot_admit(const HotArgs& hot, uint32_t v) {
    uint32_t* slot = &hot.cand[(uint32_t)(splitmix64(v) >> (64 - kHotCandBits))];
    const uint32_t x = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (hot.thresh > 2 && hot.bits <= 26) {          // slot = id << 6 | sightings
        if ((x >> 6) == v) {
            const uint32_t c = (x & 63u) + 1;
            if (c >= hot.thresh) hot_insert(hot.table, v, hot.bits, hot.five != 0);
            else __hip_atomic_store(slot, (v << 6) | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(slot, (v << 6) | 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    if (x == v) hot_insert(hot.table, v, hot.bits, hot.five != 0);
    else __hip_atomic_store(slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Filter of one thread's EPT edges (ids already range-checked and zeroed where !ok): ok[k]
// becomes false for an edge whose endpoints are both in the giant component. HOT: probe the LDS
// hot set `tab` before gbits, and (insert) offer the gbits-confirmed endpoints for admission.
// warm: probe the warm set for LDS misses first; count: add the LDS misses found in the giant to
// the warm build's counters.
// Raw buffer resource over [p, p + bytes) (gfx9 dword3: 32-bit data format); a lane whose offset
// is >= bytes (kNoLoad) makes no memory request and reads 0. The filter's correctness depends on
// that out-of-range behaviour, and dword3 is encoded differently on gfx10+: build for gfx9 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "buffer_rsrc: dword3 0x00020000 is the gfx9 (CDNA) encoding; libgsgpu is built for gfx950"
#endif
constexpr uint32_t kNoLoad = 0xFFFFFFFFu;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* p, uint64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)(bytes < kNoLoad ? bytes : kNoLoad), 0x00020000);
}

template <bool STATS, int EPT, bool HOT>
__device__ __forceinline__ void filter_group(const FoldArgs& f, const uint32_t (&u)[EPT], const uint32_t (&v)[EPT],
                                             bool (&ok)[EPT], const uint2* tab, const HotArgs& hot, bool insert,
                                             bool warm, uint64_t count_slot, uint32_t (&gflag)[EPT]) {
    bool hu[EPT], hv[EPT];       // LDS hot-set hits
    bool mu[EPT], mv[EPT];       // known giant members without a gbits load (LDS or warm hits)
    uint32_t wu[EPT], wv[EPT];
    if (HOT) {
        // every LDS bucket read of the group, then the compares
        uint2 bu[EPT], bv[EPT];
        uint32_t ru[EPT], rv[EPT];
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            bu[k] = tab[hot_bucket(u[k], hot.bits, ru[k])];
            bv[k] = tab[hot_bucket(v[k], hot.bits, rv[k])];
        }
        const bool five = hot.five != 0;
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            hu[k] = hot_match(bu[k], ru[k], five);
            hv[k] = hot_match(bv[k], rv[k], five);
        }
    } else {
#pragma unroll
        for (int k = 0; k < EPT; ++k) hu[k] = hv[k] = false;
    }
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        mu[k] = hu[k];
        mv[k] = hv[k];
    }
    if (HOT && warm) {
        // the warm words of every LDS miss in flight together, then the compares
        uint32_t xu[EPT], xv[EPT], ru[EPT], rv[EPT];
        // buffer loads: an LDS hit's lane gets an out-of-range offset (no memory request, 0
        // returned), so the loads need no branch and the waits count them exactly
        const __amdgpu_buffer_rsrc_t wr = buffer_rsrc(hot.warm, 4ull << hot.warm_bits);
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const uint32_t iu = warm_word(u[k], hot.bits, hot.warm_bits, ru[k]);
            const uint32_t iv = warm_word(v[k], hot.bits, hot.warm_bits, rv[k]);
            xu[k] = __builtin_amdgcn_raw_buffer_load_b32(wr, hu[k] ? kNoLoad : iu << 2, 0, 0);
            xv[k] = __builtin_amdgcn_raw_buffer_load_b32(wr, hv[k] ? kNoLoad : iv << 2, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            mu[k] = hu[k] | warm_match(xu[k], ru[k]);
            mv[k] = hv[k] | warm_match(xv[k], rv[k]);
        }
    }
    if (HOT) {                                       // branch-free, as the warm probes
        const __amdgpu_buffer_rsrc_t gr = buffer_rsrc(f.gbits, (((uint64_t)f.rc.cap + 31) >> 5) << 2);
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const uint32_t xu = __builtin_amdgcn_raw_buffer_load_b32(gr, mu[k] ? kNoLoad : (u[k] >> 5) << 2, 0, 0);
            const uint32_t xv = __builtin_amdgcn_raw_buffer_load_b32(gr, mv[k] ? kNoLoad : (v[k] >> 5) << 2, 0, 0);
            wu[k] = mu[k] ? ~0u : xu;
            wv[k] = mv[k] ? ~0u : xv;
        }
    } else {
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            wu[k] = mu[k] ? ~0u : f.gbits[u[k] >> 5];
            wv[k] = mv[k] ? ~0u : f.gbits[v[k] >> 5];
        }
    }

    if (HOT && STATS) {
        uint32_t nh = 0, nw = 0;
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            nh += (ok[k] && hu[k]) + (ok[k] && hv[k]);
            nw += (ok[k] && mu[k] && !hu[k]) + (ok[k] && mv[k] && !hv[k]);
        }
        if (nh) atomicAdd(&f.stats[6], (unsigned long long)nh);
        if (nw) atomicAdd(&f.stats[7], (unsigned long long)nw);
    }
    if (HOT && insert) {
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            if (ok[k] && !hu[k] && ((wu[k] >> (u[k] & 31)) & 1u)) hot_admit(hot, u[k]);
            if (ok[k] && !hv[k] && ((wv[k] >> (v[k] & 31)) & 1u)) hot_admit(hot, v[k]);
        }
    }
    if (HOT && count_slot != ~0ull) {                // uniform: a warm count launch's sampled edges
        // the wave's 4 x 64 edges own keys [count_slot * 512, +512): endpoints that count as
        // u32x4 stores, kInvalid for the rest (no atomics: a shared length word would take one
        // same-address atomic per wave step, 0.3 ms per count launch)
        uint32_t m[2 * EPT];
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            m[2 * k] = (ok[k] && !hu[k] && ((wu[k] >> (u[k] & 31)) & 1u)) ? u[k] : kInvalid;
            m[2 * k + 1] = (ok[k] && !hv[k] && ((wv[k] >> (v[k] & 31)) & 1u)) ? v[k] : kInvalid;
        }
        u32x4* dst = reinterpret_cast<u32x4*>(hot.wkeys + count_slot * (128 * EPT) + (threadIdx.x & 63) * (2 * EPT));
#pragma unroll
        for (int q = 0; q < EPT / 2; ++q) dst[q] = u32x4{m[4 * q], m[4 * q + 1], m[4 * q + 2], m[4 * q + 3]};
    }
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        gflag[k] = ((wu[k] >> (u[k] & 31)) & 1u) | (((wv[k] >> (v[k] & 31)) & 1u) << 1);
        ok[k] = ok[k] && gflag[k] != 3u;
    }
}

// Parent gathers and unions of the edges with ok[k] (all issued before any dependent step).
// Pair folds (f.combine: a received partial summary's (v, R) pairs, the Merger's survivors): the
// pairs of one sender component all name its root R, and while R's component is not yet joined to
// the receiver's every lane whose v has the smaller root CASes the same word (R's root) — one
// succeeds, the rest fail and re-walk, serialised at the memory-side atomic unit (the all-gather's
// window-1 merge at ~2.3 G pairs/s, window 5's at 0.6: profiles/r05_allgather_sim_p8.txt). Within a
// wave the lanes whose unions hook the same root H are combined first: the lane holding the
// smallest other root Lmin keeps union(H, Lmin); a lane whose other root is Lmin too has nothing
// left (the same union); any other lane's union(H, lo) becomes union(lo, Lmin) — the same
// components joined, over distinct words. One CAS on H per wave instead of one per lane.
// Every lane of a live union leaves here holding its two ROOTS (fresh = its parent word kInvalid),
// so union_edge does not walk again. Ballots and shuffles read only active lanes' values except in
// the min reduction, whose result is checked against the lanes (no owner: nothing combined).
__device__ __forceinline__ void combine_hooks(uint32_t* __restrict__ parent, bool halve, bool live, uint32_t& u,
                                              uint32_t& v, uint32_t& pu, uint32_t& pv, bool& skip) {
    skip = false;
    const bool fu = pu == kInvalid, fv = pv == kInvalid;
    if (live && (u == v || (!fu && !fv && pu == pv))) live = false;    // self-loop / common parent: union_edge's
    uint32_t ru = 0, rv = 0;
    if (live) {
        ru = fu ? u : find_root(parent, u, pu, halve);
        rv = fv ? v : find_root(parent, v, pv, halve);
        if (ru == rv) {                                                 // one component already
            live = false;
            skip = true;
        }
    }
    const uint32_t hi = ru > rv ? ru : rv, lo = ru > rv ? rv : ru;
    const bool fhi = ru > rv ? fu : fv, flo = ru > rv ? fv : fu;       // fresh: the root is the vertex
    if (live) {
        u = hi;
        pu = fhi ? kInvalid : hi;
        v = lo;
        pv = flo ? kInvalid : lo;
    }
    const uint64_t lm = __ballot(live);
    if (!lm) return;                                                    // uniform
    const uint32_t H = __shfl(hi, __ffsll((long long)lm) - 1, 64);
    const bool same = live && hi == H;
    if (__popcll(__ballot(same)) < 2) return;                           // uniform
    uint32_t x = same ? lo : 0xFFFFFFFFu;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x = min(x, (uint32_t)__shfl_xor(x, off, 64));
    const uint64_t om = __ballot(same && lo == x);
    if (!om || !same) return;                                           // (om == 0: an inactive lane's value)
    if ((int)__lane_id() == __ffsll((long long)om) - 1) return;         // the owner: union(H, Lmin)
    if (lo == x) {                                                      // the owner's union
        skip = true;
        return;
    }
    // union(lo, Lmin): Lmin is a root, or fresh and initialised by the owner's union (H > Lmin); a
    // hook of lo under a not yet initialised Lmin is the transient union_edge already tolerates (a
    // walk stops at a kInvalid word; a CAS expecting Lmin there retries from kInvalid)
    u = lo;
    pu = flo ? kInvalid : lo;
    v = x;
    pv = x;
}

template <bool MARK, bool STATS, int EPT>
__device__ __forceinline__ void union_group(const FoldArgs& f, const uint32_t (&u)[EPT], const uint32_t (&v)[EPT],
                                            const bool (&ok)[EPT], FoldStats& st) {
    uint32_t pu[EPT], pv[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        pu[k] = ok[k] ? f.parent[u[k]] : 0u;
        pv[k] = ok[k] ? f.parent[v[k]] : 0u;
    }
    uint32_t m[EPT];
    if (f.tlog) {                                    // logging fold: first touches into the touch log too
        NewV nl[EPT];
#pragma unroll
        for (int k = 0; k < EPT; ++k)
            m[k] = ok[k] ? union_edge<MARK, STATS>(f.parent, f.sbits, u[k], v[k], pu[k], pv[k], &st,
                                                   f.halve == 1 || (f.halve > 1 && ((u[k] * 0x9E3779B1u) >> 29) == 0),
                                                   f.hbits, &nl[k]) : kInvalid;
        uint32_t t[2 * EPT];
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            t[2 * k] = nl[k].a;
            t[2 * k + 1] = nl[k].b;
        }
        slot_append<2 * EPT>(f.tlog, f.tcnt, t);
    } else if (f.combine) {                          // pair folds: combined hooks (combine_hooks)
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const bool halve = f.halve == 1 || (f.halve > 1 && ((u[k] * 0x9E3779B1u) >> 29) == 0);
            uint32_t cu = u[k], cv = v[k];
            bool skip;
            combine_hooks(f.parent, halve, ok[k], cu, cv, pu[k], pv[k], skip);
            m[k] = (ok[k] && !skip) ? union_edge<MARK, STATS>(f.parent, f.sbits, cu, cv, pu[k], pv[k], &st, halve, f.hbits)
                                    : kInvalid;
        }
    } else {
#pragma unroll
        for (int k = 0; k < EPT; ++k)
            m[k] = ok[k] ? union_edge<MARK, STATS>(f.parent, f.sbits, u[k], v[k], pu[k], pv[k], &st,
                                                   f.halve == 1 || (f.halve > 1 && ((u[k] * 0x9E3779B1u) >> 29) == 0),
                                                   f.hbits) : kInvalid;
    }
    if (MARK) log_append<EPT>(f.mark, f.mark_len, m);
}

// As union_group, for survivors whose giant flags are known (bit 0: u in the giant, bit 1: v): a
// giant member x was relabelled to the giant root gR by the last close and is no root (gR is), so
// its parent word can only have moved to an ancestor of gR since; gR stands in for the parent[x]
// read (the walk goes on from gR, halving with fetch_min, and the hook CAS decides as for any
// stale read). Saves one random parent[] gather per survivor with one endpoint in the giant
// (most survivors of windows 2-12: a first-touched vertex joining the giant). Ring fold only:
// in the young forest the giant root gR is hooked again and again, and every walk from a stand-in
// gR then halves a shared word (x = a hub, or gR's own word when the walk starts at gR):
// one same-address atomic per edge, window 1 1.3 -> 2.7 ms; taking gR itself for a root instead
// fails every hook CAS on gR's word once it is hooked (14 ms). A/B in profiles/r01_v12.
// An endpoint outside the giant next to one inside is first claimed straight under gR (below):
// windows 2-12 -158 us, steady -2.5 us per window (profiles/r02_ab_experiments.txt r02_aa).
template <bool MARK, bool STATS, int EPT>
__device__ __forceinline__ void union_group_g(const FoldArgs& f, const uint32_t (&u)[EPT], const uint32_t (&v)[EPT],
                                              const bool (&ok)[EPT], const uint32_t (&gflag)[EPT], uint32_t gR,
                                              FoldStats& st, uint32_t* marks_out = nullptr) {
    uint32_t pu[EPT], pv[EPT];
    // one endpoint in the giant, the other x > gR: claim x straight under gR with a CAS from
    // kInvalid instead of gathering parent[x] first. Success = x was never touched, and hanging a
    // fresh singleton below any giant member (gR < x keeps parent[x] < x) is its union with the
    // giant; failure returns parent[x], the word the gather would have read.
    bool claimed[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        const bool cu = ok[k] && gflag[k] == 2u && u[k] > gR;      // v in the giant, u outside
        const bool cv = ok[k] && gflag[k] == 1u && v[k] > gR;      // u in the giant, v outside
        pu[k] = !ok[k] ? 0u : (gflag[k] & 1u) ? gR : cu ? atomicCAS(&f.parent[u[k]], kInvalid, gR) : f.parent[u[k]];
        pv[k] = !ok[k] ? 0u : (gflag[k] & 2u) ? gR : cv ? atomicCAS(&f.parent[v[k]], kInvalid, gR) : f.parent[v[k]];
        claimed[k] = (cu && pu[k] == kInvalid) || (cv && pv[k] == kInvalid);
    }
    uint32_t m[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        if (claimed[k]) {
            const uint32_t x = (gflag[k] == 2u) ? u[k] : v[k];
            // a claimed vertex is a depth-1 child of gR, the root the next incremental close labels
            // the giant with: that close only sets its gbits bit (cbits, no parent[] read); a close
            // that is a full pass reads every parent[] word anyway. Without cbits: the seen bit.
            if (f.cbits) set_mark(f.cbits, x);
            else set_seen(f.sbits, x);
            if (STATS) { ++st.inits; ++st.hooks; }
            m[k] = MARK ? x : kInvalid;
        } else {
            m[k] = ok[k] ? union_edge<MARK, STATS>(f.parent, f.sbits, u[k], v[k], pu[k], pv[k], &st, f.halve != 0, f.hbits) : kInvalid;
        }
    }
    if (MARK && marks_out) {                         // the caller appends them (ring_flush_final)
#pragma unroll
        for (int k = 0; k < EPT; ++k) marks_out[k] = m[k];
    } else if (MARK) {
        log_append<EPT>(f.mark, f.mark_len, m);
    }
}

// union_group_g for k_fold's small mature folds (f.claim): the same claims and gR stand-ins, plus
// the touch log of a logging fold (first touches, claims included). A separate copy so that the
// ring fold's code is not touched.
template <bool MARK, bool STATS, int EPT>
__device__ __forceinline__ void union_group_gl(const FoldArgs& f, const uint32_t (&u)[EPT], const uint32_t (&v)[EPT],
                                               const bool (&ok)[EPT], const uint32_t (&gflag)[EPT], uint32_t gR,
                                               FoldStats& st) {
    uint32_t pu[EPT], pv[EPT];
    bool claimed[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        const bool cu = ok[k] && gflag[k] == 2u && u[k] > gR;      // v in the giant, u outside
        const bool cv = ok[k] && gflag[k] == 1u && v[k] > gR;      // u in the giant, v outside
        pu[k] = !ok[k] ? 0u : (gflag[k] & 1u) ? gR : cu ? atomicCAS(&f.parent[u[k]], kInvalid, gR) : f.parent[u[k]];
        pv[k] = !ok[k] ? 0u : (gflag[k] & 2u) ? gR : cv ? atomicCAS(&f.parent[v[k]], kInvalid, gR) : f.parent[v[k]];
        claimed[k] = (cu && pu[k] == kInvalid) || (cv && pv[k] == kInvalid);
    }
    uint32_t m[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        if (claimed[k]) {
            const uint32_t x = (gflag[k] == 2u) ? u[k] : v[k];
            set_seen(f.sbits, x);                    // (a first touch: the seen bit, and the log)
            if (STATS) { ++st.inits; ++st.hooks; }
        }
    }
    if (f.tlog) {
        NewV nl[EPT];
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            if (claimed[k]) {
                nl[k].a = (gflag[k] == 2u) ? u[k] : v[k];
                m[k] = MARK ? nl[k].a : kInvalid;
            } else {
                m[k] = ok[k] ? union_edge<MARK, STATS>(f.parent, f.sbits, u[k], v[k], pu[k], pv[k], &st, f.halve != 0,
                                                       f.hbits, &nl[k]) : kInvalid;
            }
        }
        uint32_t t[2 * EPT];
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            t[2 * k] = nl[k].a;
            t[2 * k + 1] = nl[k].b;
        }
        slot_append<2 * EPT>(f.tlog, f.tcnt, t);
    } else if (f.combine) {                          // pair folds: combined hooks (combine_hooks)
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            uint32_t cu = u[k], cv = v[k];
            bool skip;
            combine_hooks(f.parent, f.halve != 0, ok[k] && !claimed[k], cu, cv, pu[k], pv[k], skip);
            if (claimed[k]) m[k] = MARK ? ((gflag[k] == 2u) ? u[k] : v[k]) : kInvalid;
            else m[k] = (ok[k] && !skip) ? union_edge<MARK, STATS>(f.parent, f.sbits, cu, cv, pu[k], pv[k], &st, f.halve != 0, f.hbits)
                                         : kInvalid;
        }
    } else {
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            if (claimed[k]) m[k] = MARK ? ((gflag[k] == 2u) ? u[k] : v[k]) : kInvalid;
            else m[k] = ok[k] ? union_edge<MARK, STATS>(f.parent, f.sbits, u[k], v[k], pu[k], pv[k], &st, f.halve != 0, f.hbits)
                              : kInvalid;
        }
    }
    if (MARK) log_append<EPT>(f.mark, f.mark_len, m);
}

// Filter, parent gathers and unions of one thread's EPT edges (ids already range-checked;
// ok[k] false = nothing to do for edge k).
template <bool MARK, bool STATS, int EPT>
__device__ __forceinline__ void fold_group(const FoldArgs& f, bool filt, uint32_t (&u)[EPT], uint32_t (&v)[EPT],
                                           bool (&ok)[EPT], FoldStats& st, uint32_t claim_gR) {
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        if (!ok[k]) { u[k] = 0; v[k] = 0; }
    }
    uint32_t nvalid = 0, nfilt = 0;
    if (STATS) for (int k = 0; k < EPT; ++k) nvalid += ok[k];
    uint32_t gflag[EPT];
    if (filt) filter_group<STATS, EPT, false>(f, u, v, ok, nullptr, HotArgs{nullptr, 0, nullptr}, false, false, ~0ull, gflag);
    if (EPT == 1 && filt && claim_gR != kInvalid) union_group_gl<MARK, STATS, EPT>(f, u, v, ok, gflag, claim_gR, st);
    else union_group<MARK, STATS, EPT>(f, u, v, ok, st);
    if (STATS) {
        for (int k = 0; k < EPT; ++k) nfilt += ok[k];
        atomicAdd(&f.stats[0], (unsigned long long)nvalid);
        atomicAdd(&f.stats[1], (unsigned long long)(nvalid - nfilt));   // filtered (skipped)
    }
}

// One thread's EPT edges starting at edge g * EPT: load, range-check, filter, union.
template <typename IdT, bool AOS, bool MARK, bool VEC, int EPT, bool STATS>
__device__ __forceinline__ void fold_edges_at(const IdT* __restrict__ a, const IdT* __restrict__ b, const FoldArgs& f,
                                              bool filt, uint64_t g, FoldStats& st, uint32_t claim_gR) {
    const uint64_t n = f.n;
    const uint64_t e0 = g * EPT;
    uint32_t u[EPT], v[EPT];
    bool ok[EPT];
    bool bad = false;
    if (VEC && e0 + EPT <= n) {
#pragma unroll
        for (int q = 0; q < EPT / 4; ++q) {
            const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a) + g * (EPT / 4) + q);
            const u32x4 y = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b) + g * (EPT / 4) + q);
            u[4 * q + 0] = x.x; u[4 * q + 1] = x.y; u[4 * q + 2] = x.z; u[4 * q + 3] = x.w;
            v[4 * q + 0] = y.x; v[4 * q + 1] = y.y; v[4 * q + 2] = y.z; v[4 * q + 3] = y.w;
        }
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            ok[k] = u[k] < f.rc.cap && v[k] < f.rc.cap;
            bad |= !ok[k];
        }
    } else {
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const uint64_t e = e0 + k;
            IdT x = 0, y = 0;
            if (e < n) {
                if (AOS) {
                    x = __builtin_nontemporal_load(&a[2 * e]);
                    y = __builtin_nontemporal_load(&a[2 * e + 1]);
                } else {
                    x = __builtin_nontemporal_load(&a[e]);
                    y = __builtin_nontemporal_load(&b[e]);
                }
            }
            const bool in = e < n;
            const bool good = in && id_ok<IdT>(x, f.rc.cap) && id_ok<IdT>(y, f.rc.cap);
            bad |= in && !good;
            ok[k] = good;
            u[k] = static_cast<uint32_t>(x);
            v[k] = static_cast<uint32_t>(y);
        }
    }
    if (bad) atomicOr(f.rc.err, 1u);
    fold_group<MARK, STATS, EPT>(f, filt, u, v, ok, st, claim_gR);
}

// UpdateCC over a batch. Each thread takes EPT consecutive edges per pass: endpoint reads are
// coalesced and nontemporal (the edge stream is read once and must not evict parent[] / gbits
// from L2 / Infinity Cache), 16 B per lane when VEC; the filter and parent[] gathers of the
// edges are issued back to back before any dependent step; then the unions run.
// f.work != nullptr (young forest, one launch per batch): workgroups take the next blockDim
// groups from the counter *f.work in stream order, so about grid x blockDim x EPT edges are in
// flight at any time (what bounds the hub contention) without a launch boundary per chunk.
template <typename IdT, bool AOS, bool MARK, bool VEC, int EPT = kEdgesPerThread, bool STATS = false>
__global__ __launch_bounds__(kFoldThreads) void k_fold(const IdT* __restrict__ a, const IdT* __restrict__ b,
                                                       FoldArgs f, uint32_t claim) {
    const uint64_t n = f.n;
    const bool filt = *f.giant != kInvalid;          // wave-uniform
    // no giant yet: the close after this launch is a full pass (k_compress: the slot this launch
    // reads has built == giant == kInvalid, so it cannot be incremental), which rebuilds the seen
    // bitmap from parent[] — first touches skip their seen-bit atomic (Erdos-Renyi windows before the
    // giant forms: ~1 M memory-side atomics per 2^20-edge window)
    if (!filt) f.sbits = nullptr;
    else f.hbits = nullptr;                          // (hooked roots are marked only before a giant)
    // small mature folds (claim): survivors next to the giant claim under the root gbits were built
    // for, as in the ring fold (ids < 2^31)
    const uint32_t claim_gR = (claim && filt && f.rc.cap <= 0x80000000u) ? f.giant[1] : kInvalid;
    // logging fold (ListCtl): this wave's touch-log slot
    __shared__ uint32_t s_tcnt[kFoldThreads / 64];
    const uint32_t wave = threadIdx.x >> 6;
    if (f.tlog) {
        f.tlog += ((size_t)blockIdx.x * (kFoldThreads / 64) + wave) * kSlotWords;
        f.tcnt = &s_tcnt[wave];
        if ((threadIdx.x & 63) == 0) s_tcnt[wave] = 0;
    }
    FoldStats st;
    const uint64_t groups = (n + EPT - 1) / EPT;
    if (f.work) {
        __shared__ unsigned long long s_base;
        for (;;) {
            if (threadIdx.x == 0) s_base = atomicAdd(f.work, (unsigned long long)blockDim.x);
            __syncthreads();
            const uint64_t base = s_base;
            __syncthreads();
            if (base >= groups) break;
            const uint64_t g = base + threadIdx.x;
            if (g < groups) fold_edges_at<IdT, AOS, MARK, VEC, EPT, STATS>(a, b, f, filt, g, st, claim_gR);
        }
    } else {
        const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
        for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += stride)
            fold_edges_at<IdT, AOS, MARK, VEC, EPT, STATS>(a, b, f, filt, g, st, claim_gR);
    }
    if (f.tlog && (threadIdx.x & 63) == 0) f.tlog[0] = s_tcnt[wave];   // every slot's count, 0 included
    if (STATS) {
        atomicAdd(&f.stats[2], (unsigned long long)st.early);
        atomicAdd(&f.stats[3], (unsigned long long)st.hooks);
        atomicAdd(&f.stats[4], (unsigned long long)st.casfail);
        atomicAdd(&f.stats[5], (unsigned long long)st.inits);
    }
}

// Steady-state UpdateCC (mature forest, aligned uint32 SoA device edges): one 1024-thread
// workgroup per CU (the hot set takes 128 KiB of its LDS, the survivor rings 16 KiB) streams the
// edges, 16 B per lane, and filters each through the LDS hot set and gbits. A wave keeps its
// survivors (edges not known to lie inside the giant) in a wave-private LDS ring and unions them
// 64 at a time, one per lane, whenever the ring holds a wave's worth, while the CU's other waves
// keep streaming: the unions' latency chains (parent walks, CAS) overlap the lookups, and run on
// full waves instead of a few lanes of a filter pass (unions inline in the filter pass: 280 us
// per steady RMAT-26 window; survivors queued for a second launch: 252 + 18-107 us; ring: 259 us).
constexpr int kRingCap = 128;                       // pairs per wave: 16 waves x 1 KiB of LDS
// Ring entries carry the survivor's giant flags in bit 31 of each id (ids < 2^31 when gR != kInvalid,
// see k_fold_ring).
template <bool MARK, bool STATS>
__device__ __forceinline__ void ring_flush(const FoldArgs& f, uint2* ring, uint32_t& cnt, uint32_t keep, FoldStats& st,
                                           uint32_t gR) {
    const int lane = threadIdx.x & 63;
    // the ring is written and read by different lanes of this wave: order those LDS accesses
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    while (cnt > keep) {                            // uniform
        const uint32_t take = min(cnt - keep, 64u);
        const uint32_t at = cnt - take;
        const bool ok1 = (uint32_t)lane < take;
        const uint2 e = ok1 ? ring[at + lane] : make_uint2(0u, 0u);
        const uint32_t u[1] = {e.x & 0x7FFFFFFFu}, v[1] = {e.y & 0x7FFFFFFFu};
        const uint32_t gf[1] = {(e.x >> 31) | ((e.y >> 31) << 1)};
        const bool ok[1] = {ok1};
        union_group_g<MARK, STATS, 1>(f, u, v, ok, gf, gR, st);
        cnt = at;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// The last flush of every wave's ring at the end of k_fold_ring. With the hook log on (MARK), the
// marks of the whole workgroup go into the log with ONE global atomic: at a launch's end every wave
// of the chip flushes at once, and a log append per wave (4096 returning atomics on one word)
// serialised there (~46 us per launch). All threads of the workgroup must call it.
template <bool MARK, bool STATS>
__device__ __forceinline__ void ring_flush_final(const FoldArgs& f, uint2* ring, uint32_t cnt, FoldStats& st, uint32_t gR,
                                                 uint32_t* s_cnt, unsigned long long* s_base) {
    if (!MARK) {
        ring_flush<MARK, STATS>(f, ring, cnt, 0, st, gR);
        return;
    }
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) *s_cnt = 0u;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    uint32_t mk[2] = {kInvalid, kInvalid};           // the ring holds at most 2 x 64 entries here
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        if (cnt == 0) break;                         // uniform
        const uint32_t take = min(cnt, 64u);
        const uint32_t at = cnt - take;
        const bool ok1 = (uint32_t)lane < take;
        const uint2 e = ok1 ? ring[at + lane] : make_uint2(0u, 0u);
        const uint32_t u[1] = {e.x & 0x7FFFFFFFu}, v[1] = {e.y & 0x7FFFFFFFu};
        const uint32_t gf[1] = {(e.x >> 31) | ((e.y >> 31) << 1)};
        const bool ok[1] = {ok1};
        union_group_g<MARK, STATS, 1>(f, u, v, ok, gf, gR, st, &mk[it]);
        cnt = at;
    }
    __syncthreads();                                 // s_cnt is zeroed
    const uint64_t lt = (1ull << lane) - 1;
    const uint64_t b0 = __ballot(mk[0] != kInvalid), b1 = __ballot(mk[1] != kInvalid);
    const uint32_t c = (uint32_t)__popcll(b0) + (uint32_t)__popcll(b1);
    uint32_t off = 0;
    if (lane == 0 && c) off = atomicAdd(s_cnt, c);   // LDS: the wave's place in the workgroup's batch
    off = __shfl(off, 0, 64);
    __syncthreads();
    if (threadIdx.x == 0) *s_base = *s_cnt ? atomicAdd(f.mark_len, (unsigned long long)*s_cnt) : 0ull;
    __syncthreads();
    const unsigned long long base = *s_base + off;
    if (mk[0] != kInvalid) f.mark[base + __popcll(b0 & lt)] = mk[0];
    if (mk[1] != kInvalid) f.mark[base + __popcll(b0) + __popcll(b1 & lt)] = mk[1];
}

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// 16-B copy of WORDS 32-bit words global -> LDS by a 1024-thread workgroup, 8 loads in flight per
// thread before any store: the element loop it replaces (load, wait, store) waited one round trip
// per step, 16 of them to fill the hot set at every ring launch
constexpr uint32_t kFillThreads = 1024;
// 16-B copy of `words` 32-bit words global -> LDS by the whole workgroup, 8 loads in flight per
// thread before any store (a load-store loop waits one round trip per step); zero past `avail`
template <uint32_t WORDS, uint32_t THREADS = kFillThreads>
__device__ __forceinline__ void lds_fill(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, uint64_t avail) {
    constexpr uint32_t kVecs = WORDS / 4;
    const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
    u32x4* d4 = reinterpret_cast<u32x4*>(dst);
    for (uint32_t v0 = 0; v0 < kVecs; v0 += 8 * THREADS) {
        u32x4 q[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t vi = v0 + j * THREADS + threadIdx.x;
            q[j] = (vi < kVecs && 4ull * vi + 4 <= avail) ? s4[vi] : u32x4{0u, 0u, 0u, 0u};
            if (vi < kVecs && 4ull * vi < avail && 4ull * vi + 4 > avail) {       // a partial last vector
                const uint32_t* w = src + 4ull * vi;
                q[j] = u32x4{w[0], 4ull * vi + 1 < avail ? w[1] : 0u, 4ull * vi + 2 < avail ? w[2] : 0u, 0u};
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t vi = v0 + j * THREADS + threadIdx.x;
            if (vi < kVecs) d4[vi] = q[j];
        }
    }
}



// 4 consecutive ids of an aligned SoA stream, loaded raw (load) and range-checked as uint32 where
// they are used (unpack): int64 ids take two 16-B loads; a negative or >= cap id fails the range
// check either way. Split so the ring fold can issue a group's loads one pass ahead.
template <typename IdT>
struct Raw4 {
    u32x4 q{0u, 0u, 0u, 0u};
    __device__ __forceinline__ void load(const IdT* __restrict__ p, uint64_t g) {
        q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p) + g);
    }
    __device__ __forceinline__ void unpack(uint32_t (&x)[4], bool (&ok)[4], uint32_t cap) const {
        x[0] = q.x; x[1] = q.y; x[2] = q.z; x[3] = q.w;
#pragma unroll
        for (int k = 0; k < 4; ++k) ok[k] = ok[k] && x[k] < cap;
    }
};
template <>
struct Raw4<int64_t> {
    u64x2 q0{0ull, 0ull}, q1{0ull, 0ull};
    __device__ __forceinline__ void load(const int64_t* __restrict__ p, uint64_t g) {
        q0 = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(p) + 2 * g);
        q1 = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(p) + 2 * g + 1);
    }
    __device__ __forceinline__ void unpack(uint32_t (&x)[4], bool (&ok)[4], uint32_t cap) const {
        const uint64_t y[4] = {q0.x, q0.y, q1.x, q1.y};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ok[k] = ok[k] && y[k] < (uint64_t)cap;
            x[k] = (uint32_t)y[k];
        }
    }
};

// GSGPU_RING_CLOCKS only (the CLK instance of k_fold_ring; production launches the one without):
// per-workgroup clocks (wall_clock64) of the last k_fold_ring launch — entry, hot set in LDS, every
// wave's main loop done, final flush done (report_ring_clocks prints them)
constexpr uint32_t kRingPhaseGroups = 4096;
__device__ unsigned long long g_ring_phase[kRingPhaseGroups][4];

template <typename IdT, bool MARK, bool STATS, bool CLK = false>
__global__ __launch_bounds__(kHotThreads) void k_fold_ring(const IdT* __restrict__ a, const IdT* __restrict__ b,
                                                           FoldArgs f, HotArgs hot) {
    __shared__ __attribute__((aligned(16))) uint2 tab[kHotBuckets];
    __shared__ uint2 rings[kHotThreads / 64][kRingCap];
    const uint64_t n = f.n;
    const bool clocks = CLK && threadIdx.x == 0 && blockIdx.x < kRingPhaseGroups;
    if (clocks) g_ring_phase[blockIdx.x][0] = wall_clock64();
    const bool filt = *f.giant != kInvalid;          // uniform
    if (!filt) f.sbits = nullptr;                    // the next close is a full pass (k_fold)
    else f.hbits = nullptr;
    if (filt) lds_fill<2 * kHotBuckets>(reinterpret_cast<uint32_t*>(tab), reinterpret_cast<const uint32_t*>(hot.table), 2 * kHotBuckets);
    // the root gbits were built for (= the giant's label at the last close); survivors' giant
    // flags use it in place of a parent[] read (union_group_g). Off (kInvalid) without a filter
    // or for ids >= 2^31 (the ring's flag bit)
    const uint32_t gR = (filt && f.rc.cap <= 0x80000000u) ? f.giant[1] : kInvalid;
    // admitting launch? (read before workgroup 0's decrement may land: a workgroup that reads the
    // decremented budget only skips this launch's admission, which is a heuristic anyway)
    const uint32_t budget = hot.budget ? *hot.budget : 1u;
    const uint64_t sample_edges = (hot.periodic || budget) ? hot.sample_edges : 0;
    const bool warm_ok = filt && hot.warm && *hot.warm_valid != 0;                        // uniform
    const uint64_t count_edges = (filt && hot.wkeys && hot.warm_valid && *hot.warm_valid == 0) ? hot.count_edges : 0;
    __syncthreads();
    if (clocks) g_ring_phase[blockIdx.x][1] = wall_clock64();
    if (blockIdx.x == 0 && threadIdx.x == 0 && hot.budget && budget) *hot.budget = budget - 1;
    if (blockIdx.x == 0 && threadIdx.x == 0 && hot.wkeys)            // key slots written below
        *hot.wctl = (min(count_edges, n / 4 * 4) + 255) / 256 * 256;
    const int lane = threadIdx.x & 63;
    uint2* const ring = rings[threadIdx.x >> 6];
    uint32_t cnt = 0;                                // wave-uniform ring fill
    FoldStats st;
    const uint64_t groups = n / 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t nvalid = 0, nkept = 0;
    // one wave round: 64 groups of 4 edges from g0 — filter, then ring or union in place
    auto wave_round = [&](const uint64_t g0) {
        const uint64_t g = g0 + lane;
        uint32_t u[4] = {0, 0, 0, 0}, v[4] = {0, 0, 0, 0};
        bool ok[4] = {false, false, false, false};
        uint32_t gf[4] = {0u, 0u, 0u, 0u};
        if (g < groups) {
            bool oka[4] = {true, true, true, true}, okb[4] = {true, true, true, true};
            Raw4<IdT> ra, rb;
            ra.load(a, g);
            rb.load(b, g);
            ra.unpack(u, oka, f.rc.cap);
            rb.unpack(v, okb, f.rc.cap);
            bool bad = false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                ok[k] = oka[k] && okb[k];
                bad |= !ok[k];
                if (!ok[k]) { u[k] = 0; v[k] = 0; }
            }
            if (bad) atomicOr(f.rc.err, 1u);
        }
        if (STATS) for (int k = 0; k < 4; ++k) nvalid += ok[k];
        if (filt) filter_group<STATS, 4, true>(f, u, v, ok, tab, hot, g * 4 < sample_edges, warm_ok,
                                               g0 * 4 < count_edges ? g0 / 64 : ~0ull, gf);
        if (gR == kInvalid) {
#pragma unroll
            for (int k = 0; k < 4; ++k) gf[k] = 0u;
        }
        const uint32_t c = (uint32_t)ok[0] + ok[1] + ok[2] + ok[3];
        if (STATS) nkept += c;
        uint32_t incl = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        const uint32_t wtot = __shfl(incl, 63, 64);
        if (wtot == 0) return;                       // uniform
        if (wtot > kRingCap / 2) {                   // young window: union in place
            union_group_g<MARK, STATS, 4>(f, u, v, ok, gf, gR, st);
            return;
        }
        if (cnt + wtot > kRingCap) ring_flush<MARK, STATS>(f, ring, cnt, kRingCap - wtot, st, gR);
        uint32_t pos = cnt + incl - c;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!ok[k]) continue;
            ring[pos] = make_uint2(u[k] | ((gf[k] & 1u) << 31), v[k] | ((gf[k] >> 1) << 31));
            ++pos;
        }
        cnt += wtot;
        if (cnt >= 64) ring_flush<MARK, STATS>(f, ring, cnt, cnt - 64, st, gR);
    };
    for (uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); g0 < groups; g0 += stride)
        wave_round(g0);
    __shared__ uint32_t s_mcnt;
    __shared__ unsigned long long s_mbase;
    if (CLK) {
        __syncthreads();
        if (clocks) g_ring_phase[blockIdx.x][2] = wall_clock64();
    }
    ring_flush_final<MARK, STATS>(f, ring, cnt, st, gR, &s_mcnt, &s_mbase);
    if (CLK) {
        __syncthreads();
        if (clocks) g_ring_phase[blockIdx.x][3] = wall_clock64();
    }
    if (STATS) {
        atomicAdd(&f.stats[0], nvalid);
        atomicAdd(&f.stats[1], nvalid - nkept);
        atomicAdd(&f.stats[2], (unsigned long long)st.early);
        atomicAdd(&f.stats[3], (unsigned long long)st.hooks);
        atomicAdd(&f.stats[4], (unsigned long long)st.casfail);
        atomicAdd(&f.stats[5], (unsigned long long)st.inits);
    }
}

// ---- partition pre-filter (GS_MERGE_PREFILTER senders, comm.hip) ----
// SummaryBulkAggregation.java:76-83 folds every partition's slice with UpdateCC and ships the
// partial to the parallelism-1 Merger. Here a sending rank keeps no forest: it runs only the giant
// FILTER of the fold over its slice — against the giant bitmap and root the Merger (rank 0)
// broadcasts, plus this rank's own LDS hot set / L2 warm set admitted against that bitmap — and
// the survivors go to the Merger as plain (u, v) edges. A stale bitmap is safe: components only
// merge until reset, so two endpoints flagged in the broadcast giant stay in one component.
// Each workgroup collects its survivors in its region of a scratch buffer, then reserves its range
// of the count-headed output with ONE atomic and copies them there (order is free: union is
// commutative). Range errors set f.rc.err, like a fold. HOT: the hot / warm sets exist (ring-sized
// ids); otherwise gbits only.
template <typename IdT, bool HOT>
__global__ __launch_bounds__(kHotThreads) void k_filter_out(const IdT* __restrict__ a, const IdT* __restrict__ b,
                                                            FoldArgs f, HotArgs hot, uint2* __restrict__ regions,
                                                            uint64_t region, uint2* __restrict__ out,
                                                            unsigned long long* __restrict__ count, int aligned) {
    __shared__ __attribute__((aligned(16))) uint2 tab[HOT ? kHotBuckets : 1];
    __shared__ uint32_t s_pos;
    __shared__ unsigned long long s_base;
    const uint64_t n = f.n;
    const bool filt = *f.giant != kInvalid;          // uniform: a bitmap has been broadcast
    if (HOT && filt) lds_fill<2 * kHotBuckets>(reinterpret_cast<uint32_t*>(tab), reinterpret_cast<const uint32_t*>(hot.table), 2 * kHotBuckets);
    const uint32_t budget = (HOT && hot.budget) ? *hot.budget : 0u;
    const uint64_t sample_edges = (HOT && (hot.periodic || budget)) ? hot.sample_edges : 0;
    const bool warm_ok = HOT && filt && hot.warm && *hot.warm_valid != 0;
    const uint64_t count_edges = (HOT && filt && hot.wkeys && hot.warm_valid && *hot.warm_valid == 0) ? hot.count_edges : 0;
    if (threadIdx.x == 0) s_pos = 0;
    __syncthreads();
    if (HOT && blockIdx.x == 0 && threadIdx.x == 0 && hot.budget && budget) *hot.budget = budget - 1;
    if (HOT && blockIdx.x == 0 && threadIdx.x == 0 && hot.wkeys)
        *hot.wctl = (min(count_edges, n / 4 * 4) + 255) / 256 * 256;
    const int lane = threadIdx.x & 63;
    uint2* const reg = regions + (uint64_t)blockIdx.x * region;
    const uint64_t groups = (n + 3) / 4;             // a partial last group: its lanes past n are not ok
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const bool vec = (n & 3) == 0;
    // aligned: both streams 16-B aligned, so whole groups load as Raw4 (otherwise element loads)
    for (uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); g0 < groups; g0 += stride) {
        const uint64_t g = g0 + lane;
        uint32_t u[4] = {0, 0, 0, 0}, v[4] = {0, 0, 0, 0};
        bool ok[4] = {false, false, false, false};
        uint32_t gf[4];
        if (g < groups) {
            bool oka[4] = {true, true, true, true}, okb[4] = {true, true, true, true};
            if (aligned && (vec || g + 1 < groups)) {
                Raw4<IdT> ra, rb;
                ra.load(a, g);
                rb.load(b, g);
                ra.unpack(u, oka, f.rc.cap);
                rb.unpack(v, okb, f.rc.cap);
            } else {                                 // unaligned, or the ragged last group
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint64_t e = 4 * g + k;
                    const bool in = e < n;
                    const uint64_t x = in ? (uint64_t)a[e] : 0, y = in ? (uint64_t)b[e] : 0;
                    oka[k] = x < (uint64_t)f.rc.cap || !in;
                    okb[k] = y < (uint64_t)f.rc.cap || !in;
                    u[k] = (uint32_t)x;
                    v[k] = (uint32_t)y;
                }
            }
            bool bad = false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool in = 4 * g + k < n;
                ok[k] = in && oka[k] && okb[k];
                bad |= in && !(oka[k] && okb[k]);
                if (!ok[k]) { u[k] = 0; v[k] = 0; }
            }
            if (bad) atomicOr(f.rc.err, 1u);
        }
        if (filt) filter_group<false, 4, HOT>(f, u, v, ok, tab, hot, g * 4 < sample_edges, warm_ok,
                                              g0 * 4 < count_edges ? g0 / 64 : ~0ull, gf);
        const uint32_t c = (uint32_t)ok[0] + ok[1] + ok[2] + ok[3];
        uint32_t incl = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        const uint32_t wtot = __shfl(incl, 63, 64);
        if (wtot == 0) continue;                     // uniform
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&s_pos, wtot);   // LDS: the wave's place in the region
        uint32_t pos = __shfl(base, 0, 64) + incl - c;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!ok[k]) continue;
            reg[pos] = make_uint2(u[k], v[k]);
            ++pos;
        }
    }
    __syncthreads();
    const uint32_t total = s_pos;
    if (threadIdx.x == 0) s_base = total ? atomicAdd(count, (unsigned long long)total) : 0ull;
    __syncthreads();
    const unsigned long long at = s_base;
    for (uint32_t i = threadIdx.x; i < total; i += blockDim.x) out[at + i] = reg[i];
}

// A sending rank's filter state after the Merger's broadcast (its gbits already in place): the
// giant words go to the slot its filters read; the hot set (and warm set) are dropped when the
// giant's root differs from the one they were admitted for — another component, or a renamed root
// of the same one, which a rank without a forest cannot tell apart. owner = derr + 5 (owner, hot
// admission budget, warm set valid), as k_compress keeps them.
__global__ __launch_bounds__(1024) void k_install_giant(const uint32_t* __restrict__ in, uint32_t* __restrict__ slot,
                                                        uint32_t* __restrict__ owner, uint2* __restrict__ hot) {
    const uint32_t g = in[0];
    const bool clear = g != owner[0];                // uniform
    __syncthreads();                                 // every thread has read owner[0]
    if (clear && hot)
        for (uint32_t i = threadIdx.x; i < kHotBuckets; i += blockDim.x) hot[i] = make_uint2(0u, 0u);
    if (threadIdx.x == 0) {
        slot[0] = in[0];
        slot[1] = in[1];
        if (clear) {
            owner[0] = g;
            owner[1] = kHotAdmitLaunches;
            owner[2] = 0;
        }
    }
}

// Warm build without global counters (the count launch's per-endpoint atomicAdd into 2^B 16-bit
// counters cost ~390 us and four band scans of them ~400 us per RMAT-26 build): the count launch
// writes its LDS-miss giant endpoints into key slots (512 per wave step, kInvalid where none);
// k_warm_part scatters their hashes h = warm_hash(v) into 2^(B-16) buckets of 2^16 hash values
// (per-workgroup LDS histogram, one atomicAdd per (workgroup, bucket) for the bucket cursor);
// k_warm_count counts a bucket in LDS (2^16 16-bit counters = 128 KiB). A bucket's hash values
// are exactly those of warm buckets [b << (16 - rb), (b + 1) << (16 - rb)) (warm bucket = h >> rb,
// rb = B - wb <= 16), so the workgroup owns those table words: each is written once, with plain
// stores, holding its 4 most counted ids (count >= 2) — no CAS inserts, no count bands, and the
// exact top 4 per bucket instead of band order. Every kernel is a no-op while the set is valid
// (*valid), so the host schedules builds without reading it back.
constexpr uint32_t kWarmLocalBits = 16;              // hash values per bucket: 2^16
constexpr uint32_t kWarmPartTile = 1u << 16;          // keys per k_warm_part workgroup (64 per thread)
constexpr uint32_t kWarmMaxBuckets = 1u << 13;        // B <= 29

struct WarmBuild {
    uint32_t* keys;                  // key slots the count launch wrote
    unsigned long long* ctl;         // [0] edges the count launch counted (0: none, e.g. no giant yet)
    uint32_t* cur;                   // per-bucket fill (nbk words)
    uint16_t* part;                  // nbk buckets x cap local hash values
    uint64_t keys_cap;               // key slot capacity (2 x sampled edges)
    uint32_t cap;                    // bucket capacity, a multiple of 8 (keys past it are dropped: counts only rank)
    uint32_t B;                      // ids < 2^B
    uint32_t nbk;                    // 2^(B - 16) buckets
    uint32_t* warm;                  // the warm table
    uint32_t wb;                     // log2(warm table words), B - 16 <= wb
    const uint32_t* valid;
};

__global__ __launch_bounds__(1024) void k_warm_part(WarmBuild w) {
    if (*w.valid) return;                            // uniform
    __shared__ uint32_t hist[kWarmMaxBuckets];
    __shared__ uint32_t base[kWarmMaxBuckets];
    const uint64_t n = min(2 * w.ctl[0], w.keys_cap);    // a multiple of 512
    const uint64_t lo = (uint64_t)blockIdx.x * kWarmPartTile;
    const uint64_t hi = min(n, lo + kWarmPartTile);
    if (lo >= hi) return;                            // uniform
    const uint32_t mask = (w.B >= 32) ? ~0u : ((1u << w.B) - 1);
    for (uint32_t b = threadIdx.x; b < w.nbk; b += blockDim.x) hist[b] = 0u;
    // the tile's keys stay in registers: 16 x 16-B loads per thread, all issued before any use
    // (a dependent load per loop step made the two passes latency-bound: 133 -> 99 us per build)
    constexpr int kVec = kWarmPartTile / 4 / 1024;
    const u32x4* src = reinterpret_cast<const u32x4*>(w.keys + lo);
    const uint32_t nvec = (uint32_t)((hi - lo) / 4);
    uint32_t hv[4 * kVec];
#pragma unroll
    for (int j = 0; j < kVec; ++j) {
        const uint32_t vi = j * 1024 + threadIdx.x;
        const u32x4 q = vi < nvec ? src[vi] : u32x4{kInvalid, kInvalid, kInvalid, kInvalid};
        const uint32_t k4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) hv[4 * j + e] = k4[e] == kInvalid ? kInvalid : (k4[e] * kWarmMul) & mask;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4 * kVec; ++j)
        if (hv[j] != kInvalid) atomicAdd(&hist[hv[j] >> kWarmLocalBits], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < w.nbk; b += blockDim.x) {
        const uint32_t c = hist[b];
        base[b] = c ? atomicAdd(&w.cur[b], c) : 0u;
        hist[b] = 0u;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4 * kVec; ++j) {
        if (hv[j] == kInvalid) continue;
        const uint32_t b = hv[j] >> kWarmLocalBits;
        const uint32_t pos = base[b] + atomicAdd(&hist[b], 1u);
        if (pos < w.cap) w.part[(uint64_t)b * w.cap + pos] = (uint16_t)(hv[j] & 0xFFFFu);
    }
}

__global__ __launch_bounds__(1024) void k_warm_count(WarmBuild w) {
    if (*w.valid) return;                            // uniform
    constexpr uint32_t kWords = 1u << (kWarmLocalBits - 1);   // 2^16 16-bit counters
    __shared__ uint32_t cnt[kWords];
    const uint32_t b = blockIdx.x;
    const uint32_t m = min(w.cur[b], w.cap);
    for (uint32_t i = threadIdx.x; i < kWords; i += blockDim.x) cnt[i] = 0u;
    __syncthreads();
    // 8 hash values per 16-B load (w.cap is a multiple of 8), a thread's loads issued together
    const u32x4* p = reinterpret_cast<const u32x4*>(w.part + (uint64_t)b * w.cap);
    const uint32_t nv = (m + 7) / 8;
    for (uint32_t v0 = 0; v0 < nv; v0 += 4 * 1024) {
        u32x4 q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t vi = v0 + j * 1024 + threadIdx.x;
            q[j] = vi < nv ? p[vi] : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t vi = v0 + j * 1024 + threadIdx.x;
            const uint32_t w4[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                if (vi * 8 + e >= m) continue;
                const uint32_t li = (w4[e >> 1] >> ((e & 1) * 16)) & 0xFFFFu;
                const uint32_t sh = (li & 1u) << 4;
                // counts saturate near 1024: with at most 1024 racing adds past the check a
                // 16-bit half never carries into its neighbour's
                if (((cnt[li >> 1] >> sh) & 0xFFFFu) < 1024u) atomicAdd(&cnt[li >> 1], 1u << sh);
            }
        }
    }
    __syncthreads();
    // warm word t of this bucket: its 2^rb hash values are local [t << rb, (t + 1) << rb); slot
    // value r = low rb bits + 1 (r = 256 does not fit a byte and never enters; warm_match never
    // matches it). Four lanes per word each keep the top 4 of a quarter as packed (count << 16 | r)
    // keys, sorted; two bitonic merges over lanes ^1 and ^2 leave the word's top 4 (one lane per
    // word scanning all 2^rb counters: 167 us per build).
    const uint32_t rb = w.B - w.wb;
    const uint32_t words = 1u << (kWarmLocalBits - rb);
    const uint32_t qw = 1u << (rb - 3);              // counter words per quarter (2 counters each)
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t task = threadIdx.x; task < 4 * words; task += blockDim.x) {   // groups of 4 lanes stay whole
        const uint32_t t = task >> 2, q = task & 3;
        uint32_t top[4] = {0u, 0u, 0u, 0u};
        const uint32_t base = (t << (rb - 1)) + q * qw;
        for (uint32_t j = 0; j < qw; ++j) {
            const uint32_t jj = (j + lane) & (qw - 1);   // rotated start: lanes spread over banks
            const uint32_t c2 = cnt[base + jj];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t c = (c2 >> (16 * k)) & 0xFFFFu;
                const uint32_t r = 2 * (q * qw + jj) + k + 1;
                uint32_t x = (c >= 2u && r <= 0xFFu) ? ((c << 16) | r) : 0u;
#pragma unroll
                for (int i = 0; i < 4; ++i) {        // sorted insertion, descending
                    const uint32_t hi = max(top[i], x);
                    x = min(top[i], x);
                    top[i] = hi;
                }
            }
        }
#pragma unroll
        for (int off = 1; off <= 2; off <<= 1) {
            uint32_t o[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = __shfl_xor(top[i], off, 64);
#pragma unroll
            for (int i = 0; i < 4; ++i) top[i] = max(top[i], o[3 - i]);   // bitonic: the 4 largest
            uint32_t x0 = max(top[0], top[2]), x2 = min(top[0], top[2]);
            uint32_t x1 = max(top[1], top[3]), x3 = min(top[1], top[3]);
            top[0] = max(x0, x1);
            top[1] = min(x0, x1);
            top[2] = max(x2, x3);
            top[3] = min(x2, x3);
        }
        if (q == 0)
            w.warm[((uint64_t)b << (kWarmLocalBits - rb)) + t] =
                (top[0] & 0xFFu) | ((top[1] & 0xFFu) << 8) | ((top[2] & 0xFFu) << 16) | ((top[3] & 0xFFu) << 24);
    }
}

// End of a build (or of a scheduled check that found the set valid): valid again, counters zeroed.
// A build that counted nothing (no giant yet) leaves the set invalid, so a later count rebuilds it.
__global__ __launch_bounds__(1024) void k_warm_done(WarmBuild w, uint32_t* __restrict__ valid) {
    for (uint32_t b = threadIdx.x; b < w.nbk; b += blockDim.x) w.cur[b] = 0u;
    __syncthreads();
    if (threadIdx.x == 0) {
        const bool counted = w.ctl[0] != 0;
        w.ctl[0] = 0;
        *valid = (*valid || counted) ? 1u : 0u;
    }
}

// DisjointSet.merge(other) with other given as a dense parent array: union(v, other[v]) for
// every v in other (DisjointSet.java:127-131 iterates other.getMatches()).
template <bool MARK>
__global__ __launch_bounds__(256) void k_merge_dense(const uint32_t* __restrict__ other, uint32_t n_other,
                                                     uint32_t* __restrict__ parent, uint32_t* __restrict__ log,
                                                     unsigned long long* __restrict__ log_len,
                                                     uint32_t* __restrict__ sbits) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n_other; v += stride) {
        const uint32_t p = other[v];
        const uint32_t m[1] = {p == kInvalid ? kInvalid : union_edge<MARK>(parent, sbits, v, p, parent[v], parent[p])};
        if (MARK) log_append<1>(log, log_len, m);
    }
}

// Per-slot pair capacities of a slot fold (the gather exchange: every sender's slot has its own
// size); n == 0: every slot holds `hi` pairs
struct SlotCaps {
    uint32_t n = 0;
    uint64_t v[kMaxSlotCaps] = {};
};

// Folds received partial summaries laid out in slots (multi-GPU exchange, comm.hip): slot q =
// [uint64 count][cap pairs (v, root)], slot_words 32-bit words apart; pairs [lo, min(count, hi,
// caps[q]))) of every slot but `skip` are unioned (DisjointSet.merge over the pairs). The counts are
// read on the device, so the fold is enqueued before the host has seen them. Ids are
// range-checked (a peer's buffer). blockIdx.y = slot.
__global__ __launch_bounds__(256) void k_fold_slots(const uint32_t* __restrict__ slots, uint64_t slot_words, int skip,
                                                    uint64_t lo, uint64_t hi, FoldArgs f, SlotCaps caps) {
    const int q = blockIdx.y;
    if (q == skip) return;                           // uniform
    if (caps.n && caps.v[q] < hi) hi = caps.v[q];
    if (*f.giant == kInvalid) f.sbits = nullptr;     // the next close is a full pass (k_fold)
    const uint32_t* s = slots + (uint64_t)q * slot_words;
    const unsigned long long cnt = *reinterpret_cast<const unsigned long long*>(s);
    const uint64_t n = cnt < hi ? cnt : hi;
    const uint32_t* pairs = s + 2;
    FoldStats st;
    for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t u[1] = {pairs[2 * i]}, v[1] = {pairs[2 * i + 1]};
        const bool ok[1] = {u[0] < f.rc.cap && v[0] < f.rc.cap};
        union_group<false, false, 1>(f, u, v, ok, st);
    }
}

// Giant-component state (gs_cc_t::derr, cc_api.hip giant_state()): two slots of two words,
// double-buffered by close parity, plus the hot set's owner:
//   slot[0] giant: the root the next close builds gbits for (followed to its current root first);
//         kInvalid = none (no filter). The folds read the current slot's word: != kInvalid turns
//         the filter on.
//   slot[1] built: the root the last close built gbits for (kInvalid: none). A close whose
//         followed giant equals it may be incremental (that root was never hooked: roots only ever
//         become non-roots).
//   owner: the root of the component the hot set's entries belong to (kInvalid: none yet).
// Close c reads slot c & 1 and writes slot (c + 1) & 1, so no workgroup's store can overtake
// another workgroup's read within the launch. Components only merge until reset, so a sampled
// giant stays the component holding its old root; k_pick_giant re-samples before every
// kPickEvery-th close in case another component overtook it (and before the early closes while
// there is no giant yet).
constexpr int kPickSamples = 1024;
constexpr int kPickSlots = 2048;
constexpr int kPickEvery = 16;              // 8 -> 16: closes -40 us per step (r02_bg)

struct PickLds {
    uint32_t keys[kPickSlots];
    uint32_t cnt[kPickSlots];
    unsigned long long best[16];
    uint32_t seen_total;
};

// Labels (read-only root walks) of kPickSamples sampled vertex ids, counted in an LDS hash table
// by one whole workgroup; the most frequent label wins if it holds at least a quarter of the seen
// samples. Returns the pick (kInvalid: no giant) to every thread.
__device__ uint32_t sample_giant(const uint32_t* __restrict__ parent, uint32_t n, PickLds& L) {
    for (int i = threadIdx.x; i < kPickSlots; i += blockDim.x) { L.keys[i] = kInvalid; L.cnt[i] = 0; }
    if (threadIdx.x == 0) L.seen_total = 0;
    __syncthreads();
    uint32_t seen = 0;
    for (int i = threadIdx.x; i < kPickSamples; i += blockDim.x) {
        const uint32_t pos = (uint32_t)(splitmix64(0x5EED0000ull + i) % n);
        if (parent[pos] == kInvalid) continue;
        const uint32_t lab = find_root_ro(parent, pos);
        ++seen;
        uint32_t h = (lab * 2654435761u) & (kPickSlots - 1);
        for (;;) {
            const uint32_t old = atomicCAS(&L.keys[h], kInvalid, lab);
            if (old == kInvalid || old == lab) { atomicAdd(&L.cnt[h], 1u); break; }
            h = (h + 1) & (kPickSlots - 1);
        }
    }
    atomicAdd(&L.seen_total, seen);
    __syncthreads();
    unsigned long long mine = 0;                 // (count << 32) | key, max-reduced
    for (int i = threadIdx.x; i < kPickSlots; i += blockDim.x)
        if (L.cnt[i]) {
            const unsigned long long c = ((unsigned long long)L.cnt[i] << 32) | L.keys[i];
            mine = c > mine ? c : mine;
        }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_down(mine, off, 64);
        mine = o > mine ? o : mine;
    }
    if ((threadIdx.x & 63) == 0) L.best[threadIdx.x >> 6] = mine;
    __syncthreads();
    unsigned long long b = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) b = L.best[w] > b ? L.best[w] : b;
    const uint32_t c = (uint32_t)(b >> 32);
    const uint32_t g = (c >= 16 && 4 * c >= L.seen_total) ? (uint32_t)b : kInvalid;
    __syncthreads();                             // L is reused by the caller
    return g;
}

// As sample_giant, over labels a previous full-pass close recorded (samp[i] = the label of sample
// position i, kInvalid where unseen): no parent[] walks. Every workgroup of a launch reads the same
// samp and gets the same pick (the count order breaks ties by key).
__device__ uint32_t mode_of_samples(const uint32_t* __restrict__ samp, PickLds& L) {
    for (int i = threadIdx.x; i < kPickSlots; i += blockDim.x) { L.keys[i] = kInvalid; L.cnt[i] = 0; }
    if (threadIdx.x == 0) L.seen_total = 0;
    __syncthreads();
    uint32_t seen = 0;
    for (int i = threadIdx.x; i < kPickSamples; i += blockDim.x) {
        const uint32_t lab = samp[i];
        if (lab == kInvalid) continue;
        ++seen;
        uint32_t h = (lab * 2654435761u) & (kPickSlots - 1);
        for (;;) {
            const uint32_t old = atomicCAS(&L.keys[h], kInvalid, lab);
            if (old == kInvalid || old == lab) { atomicAdd(&L.cnt[h], 1u); break; }
            h = (h + 1) & (kPickSlots - 1);
        }
    }
    atomicAdd(&L.seen_total, seen);
    __syncthreads();
    unsigned long long mine = 0;
    for (int i = threadIdx.x; i < kPickSlots; i += blockDim.x)
        if (L.cnt[i]) {
            const unsigned long long c = ((unsigned long long)L.cnt[i] << 32) | L.keys[i];
            mine = c > mine ? c : mine;
        }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_down(mine, off, 64);
        mine = o > mine ? o : mine;
    }
    if ((threadIdx.x & 63) == 0) L.best[threadIdx.x >> 6] = mine;
    __syncthreads();
    unsigned long long b = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) b = L.best[w] > b ? L.best[w] : b;
    const uint32_t c = (uint32_t)(b >> 32);
    return (c >= 16 && 4 * c >= L.seen_total) ? (uint32_t)b : kInvalid;
}

// Sample positions a full-pass close records labels of: position i (< kPickSamples) sits at a hashed
// offset inside the i-th stride of 2^sb ids, sb = max(0, floor(log2 n) - 10).
__device__ __forceinline__ uint32_t samp_shift(uint32_t n) {
    const uint32_t lg = 31u - (uint32_t)__clz(n | 1u);
    return lg > 10u ? lg - 10u : 0u;
}
__device__ __forceinline__ bool is_sample(uint32_t v, uint32_t sb) {
    const uint32_t i = v >> sb;
    return i < (uint32_t)kPickSamples && (v & ((1u << sb) - 1u)) == ((uint32_t)splitmix64(0x5A3Dull + i) & ((1u << sb) - 1u));
}

// Sample the giant before a close into the slot that close reads (force: even if one is known).
// One workgroup.
__global__ __launch_bounds__(1024) void k_pick_giant(const uint32_t* __restrict__ parent, uint32_t n,
                                                    uint32_t* __restrict__ slot, int force) {
    if (!force && slot[0] != kInvalid) return;   // uniform
    __shared__ PickLds L;
    const uint32_t g = sample_giant(parent, n, L);
    if (threadIdx.x == 0) slot[0] = g;
}

// Merger emission: full compression. Afterwards parent[v] = root(v) = canonical label, and
// gbits is rebuilt for the current giant root. Only v's own thread writes parent[v], walking
// read-only: a path-halving store from another thread's walk could land after v's thread
// stored the root and put back an intermediate ancestor. A workgroup covers 1024 consecutive
// vertices (4 KiB of parent[], 128 B of gbits), so every line it stores to is its own.
//
// Incremental mode (the giant root g is the one the last close built gbits for): every vertex
// with its gbit set is a depth-1 child of g and stays so (g was never hooked, and a walk through
// g's children never writes), so only seen vertices outside the giant (sbits & ~gbits) are
// relabelled; the per-window cost drops from a 4-B read per vertex to two bitmap words per 32
// vertices plus the stragglers. The 32 vertices of a bitmap word are one thread's, as are their
// 128 B of parent[].
//
// Giant state (above): every workgroup follows the input slot's giant to its current root g
// itself (a short read-only walk), so a close needs no separate pick launch; workgroup 0 clears
// the hot set when g is another component than the hot set's owner, and writes g to the output
// slot as the next close's giant and the root gbits were built for.
// List-mode arguments of a close (ListCtl above); ctl == nullptr: no lists (sparse handles).
struct ListClose {
    uint32_t* ctl = nullptr;
    const uint2* ngl_in = nullptr;       // NGL read by this close (kListSub sub-lists of ngl_sub entries)
    uint2* ngl_out = nullptr;            // NGL this close writes
    uint32_t ngl_sub = 0;
    const uint32_t* tlog = nullptr;      // the touch log of the interval this close ends (nslots slots)
    uint32_t nslots = 0;
    uint32_t c3 = 0, n3 = 0, z3 = 0;     // close number mod 3, + 1, + 2
    uint32_t unlogged = 0;               // a fold of the interval did not log (or delta emission is on)
    uint32_t list_next = 0;              // build the NGL: the next interval's folds are expected to log
};

__global__ __launch_bounds__(256) void k_compress(uint32_t* __restrict__ parent, uint32_t n,
                                                  uint32_t* __restrict__ gbits, uint32_t* __restrict__ sbits,
                                                  const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                  uint32_t* __restrict__ owner, uint2* __restrict__ hot, int rebuild_seen,
                                                  uint32_t* __restrict__ cbits, uint32_t* __restrict__ dbits,
                                                  const uint32_t* __restrict__ samp_in, uint32_t* __restrict__ samp_out,
                                                  const uint32_t* __restrict__ hb_in, uint32_t* __restrict__ hb_next) {
    __shared__ uint32_t s_g, s_inc, s_clear, s_ren;
    __shared__ PickLds L;
    // no giant known (none picked yet, or a re-pick found none): the mode of the labels the last
    // full pass recorded at the sample positions, the same in every workgroup (a giant that forms
    // mid-stream, e.g. an Erdos-Renyi stream past average degree 1, gets its filter at the next
    // close instead of at the next host-side pick)
    uint32_t g_samp = kInvalid;
    if (samp_in && in[0] == kInvalid) g_samp = mode_of_samples(samp_in, L);      // uniform
    if (threadIdx.x == 0) {
        const uint32_t g0 = in[0] != kInvalid ? in[0] : g_samp;
        const uint32_t g = (g0 == kInvalid) ? kInvalid : find_root_ro(parent, g0);
        s_g = g;
        s_inc = (g != kInvalid && g == in[1] && !rebuild_seen) ? 1u : 0u;
        // the giant's root changed (a smaller id joined it) but it is the component gbits were
        // built for: the full pass labels its members g without walking (s_ren)
        s_ren = (!s_inc && g != kInvalid && in[1] != kInvalid && find_root_ro(parent, in[1]) == g) ? 1u : 0u;
        s_clear = 0;
        if (blockIdx.x == 0) {
            if (g != kInvalid) {
                const uint32_t o = *owner;
                s_clear = (o == kInvalid || find_root_ro(parent, o) != g) ? 1u : 0u;
                *owner = g;
            }
            out[0] = g;
            out[1] = g;
        }
    }
    __syncthreads();
    const uint32_t g = s_g;
    if (s_clear && hot) {                            // workgroup 0 only: the hot set belonged to another component
        for (uint32_t i = threadIdx.x; i < kHotBuckets; i += blockDim.x) hot[i] = make_uint2(0u, 0u);
        if (threadIdx.x == 0) {
            owner[1] = kHotAdmitLaunches;            // refill: the admission budget
            owner[2] = 0;                            // the warm set belonged to it too (rebuilt later)
        }
    }
    const int lane = threadIdx.x & 63;
    if (s_inc) {                                     // one bitmap word (32 vertices) per thread
        const uint32_t nwords = (uint32_t)((n + 31) >> 5);
        for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += gridDim.x * blockDim.x) {
            uint32_t cand = sbits[w] & ~gbits[w];
            // vertices claimed under the giant root since the last close: already labelled g
            uint32_t add = cbits ? cbits[w] : 0u;
            if (add) cbits[w] = 0u;
            // delta emission: every vertex this close may relabel (or that is new) is dirty
            if (dbits && (cand | add)) dbits[w] |= cand | add;
            // up to 8 stragglers at a time, their parent and grandparent reads issued back to
            // back (one at a time: a young Erdos-Renyi window's close, ~32 stragglers per word,
            // spent 121 us per 2^24 ids in dependent loads)
            while (cand) {
                uint32_t vb[8], p[8], gp[8];
                int m = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    vb[k] = cand ? (uint32_t)(__ffs(cand) - 1) : 32u;
                    if (cand) { cand &= cand - 1; ++m; }
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) p[k] = (k < m) ? parent[(w << 5) + vb[k]] : 0u;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint32_t v = (w << 5) + vb[k];
                    gp[k] = (k < m && p[k] != v) ? parent[p[k]] : p[k];
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    if (k >= m) continue;
                    const uint32_t v = (w << 5) + vb[k];
                    uint32_t lab = p[k];
                    if (p[k] != v && gp[k] != p[k]) {
                        lab = find_root_ro(parent, gp[k]);
                        parent[v] = lab;
                    }
                    add |= (lab == g) ? (1u << vb[k]) : 0u;
                }
            }
            if (add) gbits[w] |= add;
        }
    } else {
        const uint32_t sb = samp_shift(n);
        // Hooked-root bitmap (hb_in, non-null only when every fold since the last close marked the
        // roots it hooked, i.e. none had a giant to filter with, so this close cannot be incremental):
        // a vertex's parent p that was a root at the last close (every seen vertex pointed to one)
        // and is unmarked is still a root, so its grandparent read (a random 4-B read of parent[]
        // per seen vertex: HBM / Infinity-Cache bound, ~170 us per close of an Erdos-Renyi window
        // before the giant forms) becomes a bit test in a V/8-byte bitmap that stays in L2. Every
        // parent word written since the last close is a root at the time of writing (a hook's lo, a
        // claim's gR, a halving's grandparent), so "unmarked" is exact.
        const bool usehb = hb_in != nullptr && in[1] == kInvalid;
        // giant renamed (s_ren): a vertex whose gbits or cbits bit is set is in g's component (the bits
        // were built for, or claimed under, its old root in[1], now below g; members point at in[1] or
        // an ancestor of it): its label is g, no walk. (The 8 lanes of a bitmap word read it before
        // any of them writes it below: one wave, in order.)
        const bool ren = s_ren != 0;
        for (uint64_t blk = (uint64_t)blockIdx.x * 1024; blk < n; blk += (uint64_t)gridDim.x * 1024) {
            const uint32_t base = (uint32_t)blk + threadIdx.x * 4;
            uint32_t p[4];
            if ((uint64_t)base + 4 <= n) {
                const uint4 q = *reinterpret_cast<const uint4*>(parent + base);
                p[0] = q.x; p[1] = q.y; p[2] = q.z; p[3] = q.w;
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) p[k] = ((uint64_t)base + k < n) ? parent[base + k] : kInvalid;
            }
            uint32_t mem = 0;                        // rename: this thread's 4 member bits
            if (ren && base < n) mem = ((gbits[base >> 5] | (cbits ? cbits[base >> 5] : 0u)) >> (base & 31)) & 15u;
            bool need[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) need[k] = p[k] != kInvalid && p[k] != base + k && !((mem >> k) & 1u);
            if (usehb) {
                uint32_t hw[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) hw[k] = need[k] ? hb_in[p[k] >> 5] : 0u;
#pragma unroll
                for (int k = 0; k < 4; ++k) need[k] = need[k] && ((hw[k] >> (p[k] & 31)) & 1u);
            }
            uint32_t gp[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) gp[k] = need[k] ? parent[p[k]] : p[k];
            uint32_t nib = 0, seen = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t v = base + k;
                uint32_t lab = p[k];
                if ((mem >> k) & 1u) {                   // a renamed giant member
                    lab = g;
                    if (p[k] != g) parent[v] = g;
                } else if (p[k] != kInvalid && p[k] != v && gp[k] != p[k]) {   // depth >= 2: walk, store the root
                    lab = find_root_ro(parent, gp[k]);
                    parent[v] = lab;
                }
                nib |= (lab == g && lab != kInvalid) ? (1u << k) : 0u;
                seen |= (p[k] != kInvalid) ? (1u << k) : 0u;
                if (samp_out && v < n && is_sample(v, sb)) samp_out[v >> sb] = lab;   // kInvalid: unseen
            }
            uint32_t word = nib << (4 * (lane & 7));
            word |= __shfl_xor(word, 1, 64);
            word |= __shfl_xor(word, 2, 64);
            word |= __shfl_xor(word, 4, 64);
            if ((lane & 7) == 0 && base < n) gbits[base >> 5] = word;
            {                                        // the seen bitmap, exact again after every full pass
                uint32_t sw = seen << (4 * (lane & 7));
                sw |= __shfl_xor(sw, 1, 64);
                sw |= __shfl_xor(sw, 2, 64);
                sw |= __shfl_xor(sw, 4, 64);
                if ((lane & 7) == 0 && base < n) {
                    sbits[base >> 5] = sw;
                    if (cbits) cbits[base >> 5] = 0u;    // this pass labelled the claimed vertices too
                    if (dbits) dbits[base >> 5] = sw;    // a full pass may relabel any seen vertex
                    if (hb_next) hb_next[base >> 5] = 0u;   // the next window's hooked-root marks start empty
                }
            }
        }
    }
}


// k_compress_list: k_compress plus the list machinery (ListCtl): the list close, and NGL appends in
// the full and bitmap passes. A separate kernel: compiled into k_compress, that code cost one wave
// per SIMD of occupancy and slowed the headline's closes by ~40 % even where no list was used
// (profiles/r04_bisect). The host launches it only while lists are in use (the last close built an
// NGL or this one builds one), and clears the control words when it starts using it again.
__global__ __launch_bounds__(256) void k_compress_list(uint32_t* __restrict__ parent, uint32_t n,
                                                  uint32_t* __restrict__ gbits, uint32_t* __restrict__ sbits,
                                                  const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                  uint32_t* __restrict__ owner, uint2* __restrict__ hot, int rebuild_seen,
                                                  uint32_t* __restrict__ cbits, uint32_t* __restrict__ dbits,
                                                  const uint32_t* __restrict__ samp_in, uint32_t* __restrict__ samp_out,
                                                  const uint32_t* __restrict__ hb_in, uint32_t* __restrict__ hb_next,
                                                  ListClose lc) {
    __shared__ uint32_t s_g, s_inc, s_clear, s_ren;
    __shared__ PickLds L;
    // no giant known (none picked yet, or a re-pick found none): the mode of the labels the last
    // full pass recorded at the sample positions, the same in every workgroup (a giant that forms
    // mid-stream, e.g. an Erdos-Renyi stream past average degree 1, gets its filter at the next
    // close instead of at the next host-side pick)
    uint32_t g_samp = kInvalid;
    // the list-mode control words, loaded before any store of this kernel (independent of the
    // giant walk below)
    uint32_t c_lv = 0, c_lo = 0, c_nc = 0;
    const uint32_t sub = blockIdx.x & (kListSub - 1);
    if (lc.ctl) {
        c_lv = lc.ctl[ListCtl::LVALID(lc.c3)];
        c_lo = lc.ctl[ListCtl::LOVF(lc.c3)];
        c_nc = lc.ctl[ListCtl::NC(lc.c3) + sub];
    }
    if (samp_in && in[0] == kInvalid) g_samp = mode_of_samples(samp_in, L);      // uniform
    if (threadIdx.x == 0) {
        const uint32_t g0 = in[0] != kInvalid ? in[0] : g_samp;
        const uint32_t g = (g0 == kInvalid) ? kInvalid : find_root_ro(parent, g0);
        s_g = g;
        s_inc = (g != kInvalid && g == in[1] && !rebuild_seen) ? 1u : 0u;
        // the giant's root changed (a smaller id joined it) but it is the component gbits were
        // built for: the full pass labels its members g without walking (s_ren)
        s_ren = (!s_inc && g != kInvalid && in[1] != kInvalid && find_root_ro(parent, in[1]) == g) ? 1u : 0u;
        s_clear = 0;
        if (blockIdx.x == 0) {
            if (g != kInvalid) {
                const uint32_t o = *owner;
                s_clear = (o == kInvalid || find_root_ro(parent, o) != g) ? 1u : 0u;
                *owner = g;
            }
            out[0] = g;
            out[1] = g;
        }
    }
    if (threadIdx.x == 0) {
        // 0: full pass, 1: bitmap-incremental, 2: list (ListCtl: a complete NGL, and every fold of
        // the interval logged its first touches)
        if (lc.ctl) {
            if (s_inc && c_lv && !c_lo && !lc.unlogged) s_inc = 2u;
            if (blockIdx.x == 0) {
                lc.ctl[ListCtl::LVALID(lc.n3)] = (s_g != kInvalid && lc.list_next) ? 1u : 0u;
                lc.ctl[ListCtl::LOVF(lc.z3)] = 0u;
            }
        }
    }
    if (lc.ctl && blockIdx.x == 0) {
        for (uint32_t i = threadIdx.x; i < kListSub; i += blockDim.x) lc.ctl[ListCtl::NC(lc.z3) + i] = 0u;
    }
    __syncthreads();
    const uint32_t g = s_g;
    // this close writes the next NGL (seen vertices outside the giant) into sub-list blockIdx % kListSub
    const bool build = lc.ctl && lc.list_next && g != kInvalid;
    uint2* ngl_o = build ? lc.ngl_out + (size_t)sub * lc.ngl_sub : nullptr;
    uint32_t* ngl_c = build ? lc.ctl + ListCtl::NC(lc.n3) + sub : nullptr;
    uint32_t* ngl_v = build ? lc.ctl + ListCtl::LOVF(lc.n3) : nullptr;
    if (s_clear && hot) {                            // workgroup 0 only: the hot set belonged to another component
        for (uint32_t i = threadIdx.x; i < kHotBuckets; i += blockDim.x) hot[i] = make_uint2(0u, 0u);
        if (threadIdx.x == 0) {
            owner[1] = kHotAdmitLaunches;            // refill: the admission budget
            owner[2] = 0;                            // the warm set belonged to it too (rebuilt later)
        }
    }
    const int lane = threadIdx.x & 63;
    if (s_inc == 2u) {
        // list close: the last NGL (sub-list `sub` by the workgroups with that index mod kListSub)
        // and the interval's touch-log slots (one per wave, strided over the grid's waves). Their
        // labels may change (a hooked root); every other seen vertex is a giant member labelled g.
        // Stores: parent by fetch_min (lab < parent[v]), gbits by fetch_or (the items are
        // scattered: no thread owns their lines). Loops are wave-uniform.
        // p: v's parent word, or its label at the last close (an NGL entry: parent[v] still
        // points there unless that root was hooked since)
        auto visit = [&](uint32_t v, uint32_t p, bool have) {
            uint32_t lab = kInvalid;
            if (have) {
                lab = p;
                if (p != v) {
                    const uint32_t gp = parent[p];
                    if (gp != p) {
                        lab = find_root_ro(parent, gp);
                        __hip_atomic_fetch_min(&parent[v], lab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                } else {
                    const uint32_t q = parent[v];        // a root then: hooked since?
                    if (q != v) {
                        lab = find_root_ro(parent, q);
                        __hip_atomic_fetch_min(&parent[v], lab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                if (lab == g) __hip_atomic_fetch_or(&gbits[v >> 5], 1u << (v & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const uint2 m[1] = {make_uint2((have && lab != g) ? v : kInvalid, lab)};
            if (build) list_append<1>(ngl_o, ngl_c, lc.ngl_sub, ngl_v, m);
        };
        const uint32_t wpb = blockDim.x >> 6, wv = threadIdx.x >> 6;
        const uint32_t part = blockIdx.x / kListSub, nparts = gridDim.x / kListSub;
        const uint32_t cn = min(c_nc, lc.ngl_sub);
        const uint2* li = lc.ngl_in + (size_t)sub * lc.ngl_sub;
        for (uint32_t i0 = part * blockDim.x + wv * 64; i0 < cn; i0 += nparts * blockDim.x) {
            const uint32_t i = i0 + lane;
            const uint2 e = i < cn ? li[i] : make_uint2(0u, 0u);
            visit(e.x, e.y, i < cn);
        }
        // slots: the waves of the workgroups past the first kListSub (those have no NGL share
        // unless the NGL is long); a slot's count and first 64 entries are loaded together
        const uint32_t w0 = gridDim.x > kListSub ? kListSub : 0u;
        for (uint32_t sl = (blockIdx.x - w0) * wpb + wv; blockIdx.x >= w0 && sl < lc.nslots; sl += (gridDim.x - w0) * wpb) {
            const uint32_t* slot = lc.tlog + (size_t)sl * kSlotWords;
            const uint32_t c0 = slot[0];
            const uint32_t e0 = slot[1 + lane];
            const uint32_t sc = min(c0, 2u * 64u);
            const uint32_t p0 = (uint32_t)lane < sc ? parent[e0] : 0u;
            visit(e0, p0, (uint32_t)lane < sc);
            if (sc > 64) {
                const uint32_t e1 = slot[65 + lane];
                const bool h1 = 64u + lane < sc;
                visit(e1, h1 ? parent[e1] : 0u, h1);
            }
        }
    } else if (s_inc) {                              // one bitmap word (32 vertices) per thread
        const uint32_t nwords = (uint32_t)((n + 31) >> 5);
        for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += gridDim.x * blockDim.x) {
            uint32_t cand = sbits[w] & ~gbits[w];
            // vertices claimed under the giant root since the last close: already labelled g
            uint32_t add = cbits ? cbits[w] : 0u;
            if (add) cbits[w] = 0u;
            // delta emission: every vertex this close may relabel (or that is new) is dirty
            if (dbits && (cand | add)) dbits[w] |= cand | add;
            // up to 8 stragglers at a time, their parent and grandparent reads issued back to
            // back (one at a time: a young Erdos-Renyi window's close, ~32 stragglers per word,
            // spent 121 us per 2^24 ids in dependent loads)
            while (cand) {
                uint32_t vb[8], p[8], gp[8];
                int m = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    vb[k] = cand ? (uint32_t)(__ffs(cand) - 1) : 32u;
                    if (cand) { cand &= cand - 1; ++m; }
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) p[k] = (k < m) ? parent[(w << 5) + vb[k]] : 0u;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint32_t v = (w << 5) + vb[k];
                    gp[k] = (k < m && p[k] != v) ? parent[p[k]] : p[k];
                }
                uint2 ng[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    ng[k] = make_uint2(kInvalid, 0u);
                    if (k >= m) continue;
                    const uint32_t v = (w << 5) + vb[k];
                    uint32_t lab = p[k];
                    if (p[k] != v && gp[k] != p[k]) {
                        lab = find_root_ro(parent, gp[k]);
                        parent[v] = lab;
                    }
                    add |= (lab == g) ? (1u << vb[k]) : 0u;
                    if (lab != g) ng[k] = make_uint2(v, lab);
                }
                if (build) list_append<8>(ngl_o, ngl_c, lc.ngl_sub, ngl_v, ng);
            }
            if (add) gbits[w] |= add;
        }
    } else {
        const uint32_t sb = samp_shift(n);
        // Hooked-root bitmap (hb_in, non-null only when every fold since the last close marked the
        // roots it hooked, i.e. none had a giant to filter with, so this close cannot be incremental):
        // a vertex's parent p that was a root at the last close (every seen vertex pointed to one)
        // and is unmarked is still a root, so its grandparent read (a random 4-B read of parent[]
        // per seen vertex: HBM / Infinity-Cache bound, ~170 us per close of an Erdos-Renyi window
        // before the giant forms) becomes a bit test in a V/8-byte bitmap that stays in L2. Every
        // parent word written since the last close is a root at the time of writing (a hook's lo, a
        // claim's gR, a halving's grandparent), so "unmarked" is exact.
        const bool usehb = hb_in != nullptr && in[1] == kInvalid;
        // giant renamed (s_ren): a vertex whose gbits or cbits bit is set is in g's component (the bits
        // were built for, or claimed under, its old root in[1], now below g; members point at in[1] or
        // an ancestor of it): its label is g, no walk. (The 8 lanes of a bitmap word read it before
        // any of them writes it below: one wave, in order.)
        const bool ren = s_ren != 0;
        for (uint64_t blk = (uint64_t)blockIdx.x * 1024; blk < n; blk += (uint64_t)gridDim.x * 1024) {
            const uint32_t base = (uint32_t)blk + threadIdx.x * 4;
            uint32_t p[4];
            if ((uint64_t)base + 4 <= n) {
                const uint4 q = *reinterpret_cast<const uint4*>(parent + base);
                p[0] = q.x; p[1] = q.y; p[2] = q.z; p[3] = q.w;
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) p[k] = ((uint64_t)base + k < n) ? parent[base + k] : kInvalid;
            }
            uint32_t mem = 0;                        // rename: this thread's 4 member bits
            if (ren && base < n) mem = ((gbits[base >> 5] | (cbits ? cbits[base >> 5] : 0u)) >> (base & 31)) & 15u;
            bool need[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) need[k] = p[k] != kInvalid && p[k] != base + k && !((mem >> k) & 1u);
            if (usehb) {
                uint32_t hw[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) hw[k] = need[k] ? hb_in[p[k] >> 5] : 0u;
#pragma unroll
                for (int k = 0; k < 4; ++k) need[k] = need[k] && ((hw[k] >> (p[k] & 31)) & 1u);
            }
            uint32_t gp[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) gp[k] = need[k] ? parent[p[k]] : p[k];
            uint32_t nib = 0, seen = 0;
            uint2 ng[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t v = base + k;
                uint32_t lab = p[k];
                if ((mem >> k) & 1u) {                   // a renamed giant member
                    lab = g;
                    if (p[k] != g) parent[v] = g;
                } else if (p[k] != kInvalid && p[k] != v && gp[k] != p[k]) {   // depth >= 2: walk, store the root
                    lab = find_root_ro(parent, gp[k]);
                    parent[v] = lab;
                }
                nib |= (lab == g && lab != kInvalid) ? (1u << k) : 0u;
                seen |= (p[k] != kInvalid) ? (1u << k) : 0u;
                ng[k] = make_uint2((p[k] != kInvalid && lab != g) ? v : kInvalid, lab);
                if (samp_out && v < n && is_sample(v, sb)) samp_out[v >> sb] = lab;   // kInvalid: unseen
            }
            if (build) list_append<4>(ngl_o, ngl_c, lc.ngl_sub, ngl_v, ng);
            uint32_t word = nib << (4 * (lane & 7));
            word |= __shfl_xor(word, 1, 64);
            word |= __shfl_xor(word, 2, 64);
            word |= __shfl_xor(word, 4, 64);
            if ((lane & 7) == 0 && base < n) gbits[base >> 5] = word;
            {                                        // the seen bitmap, exact again after every full pass
                uint32_t sw = seen << (4 * (lane & 7));
                sw |= __shfl_xor(sw, 1, 64);
                sw |= __shfl_xor(sw, 2, 64);
                sw |= __shfl_xor(sw, 4, 64);
                if ((lane & 7) == 0 && base < n) {
                    sbits[base >> 5] = sw;
                    if (cbits) cbits[base >> 5] = 0u;    // this pass labelled the claimed vertices too
                    if (dbits) dbits[base >> 5] = sw;    // a full pass may relabel any seen vertex
                    if (hb_next) hb_next[base >> 5] = 0u;   // the next window's hooked-root marks start empty
                }
            }
        }
    }
}

// wave64 / block reductions
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
    return x;
}

// n_vertices, n_components (roots) and the emission checksum over a (compressed) parent array.
template <bool CHECKSUM>
__global__ __launch_bounds__(256) void k_stats(const uint32_t* __restrict__ parent, uint32_t n,
                                               unsigned long long* __restrict__ out) {
    unsigned long long seen = 0, roots = 0, h = 0;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += stride) {
        const uint32_t p = parent[v];
        if (p == kInvalid) continue;
        ++seen;
        roots += (p == v);
        if (CHECKSUM) h += pair_mix(v, p);
    }
    __shared__ unsigned long long red[3][4];
    seen = wave_sum(seen); roots = wave_sum(roots);
    if (CHECKSUM) h = wave_sum(h);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) { red[0][wid] = seen; red[1][wid] = roots; red[2][wid] = h; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0, r = 0, c = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { s += red[0][w]; r += red[1][w]; c += red[2][w]; }
        atomicAdd(&out[0], s);
        atomicAdd(&out[1], r);
        if (CHECKSUM) atomicAdd(&out[2], c);
    }
}

// DisjointSet.find for a batch of ids. Read-only walk (the label array is not modified).
template <typename IdT>
__global__ __launch_bounds__(256) void k_find(const IdT* __restrict__ ids, IdT* __restrict__ roots, uint64_t n,
                                              const uint32_t* __restrict__ parent, uint32_t cap) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const IdT x = ids[i];
        IdT r = static_cast<IdT>(-1);
        if (id_ok<IdT>(x, cap)) {
            const uint32_t p = parent[static_cast<uint32_t>(x)];
            if (p != kInvalid) r = static_cast<IdT>(find_root_ro(parent, static_cast<uint32_t>(x)));
        }
        roots[i] = r;
    }
}

// dense emission for 64-bit ids: labels[v] = parent[v] or -1
__global__ __launch_bounds__(256) void k_widen(const uint32_t* __restrict__ parent, int64_t* __restrict__ out, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += stride) {
        const uint32_t p = parent[v];
        out[v] = p == kInvalid ? -1 : static_cast<int64_t>(p);
    }
}

// ---- ordered compaction of (vertex, label) for emit_pairs: tile = 256 threads x 16 vertices
constexpr int kTileThreads = 256;
constexpr int kTilePerThread = 16;
constexpr uint32_t kTile = kTileThreads * kTilePerThread;

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t x, uint32_t* total) {
    __shared__ uint32_t wsum[kTileThreads / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t incl = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kTileThreads / 64; ++w) {
        if (w < wid) wbase += wsum[w];
        tot += wsum[w];
    }
    __syncthreads();
    *total = tot;
    return wbase + incl - x;
}

__global__ __launch_bounds__(kTileThreads) void k_tile_count(const uint32_t* __restrict__ parent, uint32_t n,
                                                             uint32_t* __restrict__ tile_count) {
    const uint64_t base = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kTilePerThread;
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < kTilePerThread; ++k) {
        const uint64_t v = base + k;
        c += (v < n && parent[v] != kInvalid);
    }
    uint32_t tot;
    (void)block_exclusive_scan(c, &tot);
    if (threadIdx.x == 0) tile_count[blockIdx.x] = tot;
}

// Exclusive scan of tile counts in one 1024-thread block; offsets are uint64, off[ntiles] = the sum
// (also to *total_host, a pinned word, if given). Up to kScanLdsTiles tiles the counts go through
// LDS: coalesced loads in, each thread scans a run of consecutive tiles there (wave shuffles across
// runs), offsets (< 2^32: at most vertex_capacity pairs) back in place, coalesced stores out. One CU
// reading lane-strided runs straight from memory issued 64 line requests per load instruction
// (~25 us at 16384 tiles); larger summaries keep that path.
constexpr uint32_t kScanLdsTiles = 16384;
__global__ __launch_bounds__(1024) void k_tile_scan(const uint32_t* __restrict__ cnt, uint64_t* __restrict__ off,
                                                    uint32_t ntiles, unsigned long long* __restrict__ total_host) {
    __shared__ uint32_t sc[kScanLdsTiles];
    __shared__ unsigned long long wsum[16];
    const bool lds = ntiles <= kScanLdsTiles;
    if (lds) {                                   // 16 loads in flight per thread, not one at a time
        constexpr uint32_t kU = kScanLdsTiles / 1024;
        uint32_t x[kU];
#pragma unroll
        for (uint32_t j = 0; j < kU; ++j) x[j] = cnt[min(j * 1024 + threadIdx.x, ntiles - 1)];
#pragma unroll
        for (uint32_t j = 0; j < kU; ++j)
            if (j * 1024 + threadIdx.x < ntiles) sc[j * 1024 + threadIdx.x] = x[j];
        __syncthreads();
    }
    const uint32_t per = (ntiles + blockDim.x - 1) / blockDim.x;
    const uint32_t lo = min(threadIdx.x * per, ntiles), hi = min(lo + per, ntiles);
    unsigned long long s = 0;
    for (uint32_t i = lo; i < hi; ++i) s += lds ? sc[i] : cnt[i];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long incl = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    unsigned long long base = 0, tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        if (w < wid) base += wsum[w];
        tot += wsum[w];
    }
    unsigned long long run = base + incl - s;
    if (lds) {
        for (uint32_t i = lo; i < hi; ++i) { const uint32_t x = sc[i]; sc[i] = (uint32_t)run; run += x; }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < ntiles; i += blockDim.x) off[i] = sc[i];
    } else {
        for (uint32_t i = lo; i < hi; ++i) { off[i] = run; run += cnt[i]; }
    }
    if (threadIdx.x == 0) {
        off[ntiles] = tot;
        if (total_host) *total_host = tot;
    }
}

template <typename IdT>
__global__ __launch_bounds__(kTileThreads) void k_tile_scatter(const uint32_t* __restrict__ parent, uint32_t n,
                                                               const uint64_t* __restrict__ off, IdT* __restrict__ vout,
                                                               IdT* __restrict__ lout, uint64_t cap) {
    const uint64_t base = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kTilePerThread;
    uint32_t p[kTilePerThread];
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < kTilePerThread; ++k) {
        const uint64_t v = base + k;
        p[k] = (v < n) ? parent[v] : kInvalid;
        c += (p[k] != kInvalid);
    }
    uint32_t tot;
    uint64_t pos = off[blockIdx.x] + block_exclusive_scan(c, &tot);
#pragma unroll
    for (int k = 0; k < kTilePerThread; ++k) {
        if (p[k] == kInvalid) continue;
        if (pos < cap) { vout[pos] = static_cast<IdT>(base + k); lout[pos] = static_cast<IdT>(p[k]); }
        ++pos;
    }
}

// ---- delta emission (gs_cc_emit_delta): same tiles as emit_pairs; a vertex is emitted when it is
// dirty (a close may have relabelled it since the last delta) and its label differs from the one
// last emitted (elab). A thread's 16 vertices are half a dirty word; clean halves read nothing else.
__device__ __forceinline__ uint32_t delta_bits(const uint32_t* __restrict__ dbits, uint64_t base) {
    return (dbits[base >> 5] >> (base & 16)) & 0xFFFFu;
}

// Pass 1 (nothing consumed): a tile's changed pairs into its own staging region (tile t at
// t * kTile of sv / sl, in vertex order), their number into tile_count[t]. A thread's 16 vertices
// are half a dirty word; it loads only the 16-B quads of parent / elab holding dirty vertices.
// kDeltaTiles tiles per workgroup, their loads issued together (one dbits + one quad latency per
// workgroup instead of per tile: the kernel is latency-bound, 8 workgroups per CU at a time).
constexpr int kDeltaTiles = 2;
template <typename IdT>
__global__ __launch_bounds__(kTileThreads) void k_delta_stage(const uint32_t* __restrict__ parent, uint32_t n,
                                                              const uint32_t* __restrict__ elab,
                                                              const uint32_t* __restrict__ dbits, uint32_t ntiles,
                                                              uint32_t* __restrict__ tile_count,
                                                              IdT* __restrict__ sv, IdT* __restrict__ sl) {
    uint64_t base[kDeltaTiles];
    uint32_t d[kDeltaTiles], hit[kDeltaTiles], c[kDeltaTiles];
    uint32_t p[kDeltaTiles][kTilePerThread];
#pragma unroll
    for (int u = 0; u < kDeltaTiles; ++u) {
        const uint32_t t = blockIdx.x * kDeltaTiles + u;
        base[u] = (uint64_t)t * kTile + (uint64_t)threadIdx.x * kTilePerThread;
        d[u] = (t < ntiles && base[u] < n) ? delta_bits(dbits, base[u]) : 0u;
    }
#pragma unroll
    for (int u = 0; u < kDeltaTiles; ++u) {
        hit[u] = 0;
        c[u] = 0;
        if (d[u] && base[u] + kTilePerThread <= n) {
            const uint4* p4 = reinterpret_cast<const uint4*>(parent + base[u]);
            const uint4* e4 = reinterpret_cast<const uint4*>(elab + base[u]);
#pragma unroll
            for (int q = 0; q < kTilePerThread / 4; ++q) {
                uint4 a = make_uint4(kInvalid, kInvalid, kInvalid, kInvalid), e = a;
                if ((d[u] >> (4 * q)) & 0xFu) { a = p4[q]; e = e4[q]; }
                const uint32_t pa[4] = {a.x, a.y, a.z, a.w}, ea[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int k = 4 * q + j;
                    p[u][k] = pa[j];
                    if (((d[u] >> k) & 1u) && pa[j] != kInvalid && pa[j] != ea[j]) { hit[u] |= 1u << k; ++c[u]; }
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < kTilePerThread; ++k) {
                const uint64_t v = base[u] + k;
                p[u][k] = kInvalid;
                if (((d[u] >> k) & 1u) && v < n) {
                    p[u][k] = parent[v];
                    if (p[u][k] != kInvalid && p[u][k] != elab[v]) { hit[u] |= 1u << k; ++c[u]; }
                }
            }
        }
    }
#pragma unroll
    for (int u = 0; u < kDeltaTiles; ++u) {
        const uint32_t t = blockIdx.x * kDeltaTiles + u;
        uint32_t tot;
        uint64_t pos = (uint64_t)t * kTile + block_exclusive_scan(c[u], &tot);
#pragma unroll
        for (int k = 0; k < kTilePerThread; ++k) {
            if (!((hit[u] >> k) & 1u)) continue;
            sv[pos] = static_cast<IdT>(base[u] + k);
            sl[pos] = static_cast<IdT>(p[u][k]);
            ++pos;
        }
        if (threadIdx.x == 0 && t < ntiles) tile_count[t] = tot;
    }
}

// Pass 3, only if the whole delta fits cap (off[ntiles] = its size; uniform, so an overflow consumes
// nothing and the next delta still holds these pairs): tile t's pairs to out[off[t]..], elab updated,
// the tile's 128 dirty words (its own line) cleared. One workgroup per tile.
template <typename IdT>
__global__ __launch_bounds__(256) void k_delta_pack(const IdT* __restrict__ sv, const IdT* __restrict__ sl,
                                                    const uint32_t* __restrict__ tile_count,
                                                    const uint64_t* __restrict__ off, uint32_t ntiles, uint64_t cap,
                                                    uint32_t* __restrict__ elab, uint32_t* __restrict__ dbits, uint32_t n,
                                                    IdT* __restrict__ vout, IdT* __restrict__ lout,
                                                    uint64_t* __restrict__ total_out) {
    // the size also to the output slot's own word (async emissions: the copy kernel reads it there,
    // after the next emission may already have reused off[])
    if (total_out && blockIdx.x == 0 && threadIdx.x == 0) *total_out = off[ntiles];
    if (off[ntiles] > cap) return;
    const uint32_t t = blockIdx.x;
    const uint32_t c = tile_count[t];
    const uint64_t o = off[t], src = (uint64_t)t * kTile;
    for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) {
        const IdT v = sv[src + i], l = sl[src + i];
        vout[o + i] = v;
        lout[o + i] = l;
        elab[static_cast<uint64_t>(v)] = static_cast<uint32_t>(l);
    }
    const uint64_t w = (uint64_t)t * (kTile / 32) + threadIdx.x;
    if (threadIdx.x < kTile / 32 && w < ((uint64_t)n + 31) / 32) dbits[w] = 0u;
}

// Async emission, last step (gs_cc_emit_delta_async into device or pinned host buffers): the packed
// pairs (*total of them, nothing if that exceeds cap) to the caller's buffers — pinned host memory
// through its device mapping, 16 B per lane where the buffers allow (a wave writes 1 KiB
// contiguously). Launched with a few workgroups on a stream of its own: it overlaps the next
// window's fold, and a full-width grid of PCIe writers slowed that fold by ~20 %.
template <typename IdT>
__device__ __forceinline__ void copy_ids(const IdT* __restrict__ src, IdT* __restrict__ dst, uint64_t n) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    uint64_t head = 0;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
        constexpr uint64_t kPer = 16 / sizeof(IdT);
        const uint64_t nv = n / kPer;
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(dst);
        constexpr int kU = 4;                                     // 4 loads in flight per thread
        uint64_t i = tid;
        for (; i + (kU - 1) * nt < nv; i += kU * nt) {
            uint4 q[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) q[u] = s4[i + u * nt];
#pragma unroll
            for (int u = 0; u < kU; ++u) d4[i + u * nt] = q[u];
        }
        for (; i < nv; i += nt) d4[i] = s4[i];
        head = nv * kPer;
    }
    for (uint64_t i = head + tid; i < n; i += nt) dst[i] = src[i];
}

template <typename IdT>
__global__ __launch_bounds__(256) void k_delta_copy(const IdT* __restrict__ sv, const IdT* __restrict__ sl,
                                                    const uint64_t* __restrict__ total, uint64_t cap,
                                                    IdT* __restrict__ vout, IdT* __restrict__ lout,
                                                    unsigned long long* __restrict__ count_out) {
    const uint64_t n = *total;
    if (blockIdx.x == 0 && threadIdx.x == 0) *count_out = n;
    if (n > cap) return;
    copy_ids(sv, vout, n);
    copy_ids(sl, lout, n);
}

// Partial-summary export (multi-GPU CombineCC): every pending hook-log entry v (a root hooked
// since the last export, or a self-loop first touch) becomes the pair (v, root(v)). Roots, not
// the parent words at hook time: the receiver's unions then all point at the few component minima
// its own forest already holds (short walks, no hook chains to contend on). ctr = [length, read
// cursor]; the pending entries are [cursor, length); *count receives their number; at most cap
// pairs are written, the rest stay pending (the last workgroup advances the cursor). One thread per entry: the export
// costs O(hooks) instead of a scan of a V-bit mark bitmap (23 us per RMAT-26 window).
__global__ __launch_bounds__(256) void k_export_log(const uint32_t* __restrict__ log, unsigned long long* __restrict__ ctr,
                                                    const uint32_t* __restrict__ parent, uint32_t* __restrict__ pairs,
                                                    uint64_t cap, unsigned long long* __restrict__ count) {
    const unsigned long long len = ctr[0], rd = ctr[1];
    const unsigned long long n = len - rd;
    const unsigned long long take = n < cap ? n : cap;
    if (blockIdx.x == 0 && threadIdx.x == 0) *count = n;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < take;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const uint32_t v = log[rd + i];
        pairs[2 * i] = v;
        pairs[2 * i + 1] = find_root_ro(parent, v);
    }
    // consume what was written, by the last workgroup to finish (ctr[2] counts finished workgroups;
    // each has read ctr before it counts itself): an emptied log restarts at 0. (Was a second
    // one-thread launch, ~5 us per exchanged window.)
    __syncthreads();
    if (threadIdx.x == 0 && len >= rd) {             // (the condition orders the ctr reads first)
        const unsigned long long done = atomicAdd(&ctr[2], 1ull);
        if (done == gridDim.x - 1) {
            if (rd + take == len) { ctr[0] = 0; ctr[1] = 0; }
            else ctr[1] = rd + take;
            ctr[2] = 0;
        }
    }
}

}  // namespace gsgpu
