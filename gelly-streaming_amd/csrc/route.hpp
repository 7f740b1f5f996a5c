// route.hpp — the routed steady fold (UpdateCC past the young forest, DisjointSet.java:92-118 via
// ConnectedComponents.java:83-85): the giant-component filter answered from LDS, never from L2.
//
// Why: k_fold_ring's filter does one random 4-B lookup per endpoint that misses the LDS hot set
// (~22.6 M per RMAT-26 2^24-edge window), each one L2 request; random 4-B requests run at ~260 G/s
// on L2 hits and ~59 G/s on misses chip-wide (tools/request_lab.hip), so the filter, not the bytes,
// bounds the kernel. Here every lookup that leaves a CU's hot set is routed to
// the workgroup that holds the vertex's slice of gbits in LDS; what crosses the chip are
// coalesced list writes and reads (bytes, at stream rate), not random requests.
//
//   A  k_sift: streams the edges through the LDS hot set (exact set of giant members). An edge whose
//      endpoints both hit is dropped. Otherwise it becomes a SINGLE x (4 B: the other endpoint is a
//      known giant member) listed for part(x), or a DOUBLE (u, v) (8 B: neither known) listed for
//      part(u); part(x) = x >> 20, 2^20 ids = 128 KiB of gbits. A wave sorts its entries by part in
//      LDS (counting sort) so each part's run leaves as one coalesced store.
//   B  k_probe<true>: workgroup b owns part b % parts, whose gbits slice it copies into LDS. A single
//      x: in the giant -> dropped, else a survivor (x joins the giant). A double: u outside the
//      giant -> survivor (u, v); inside -> v becomes a single for part(v), listed for C (decided in
//      place when part(v) is this part).
//   C  k_probe<false>: B's singles, as B's.
//   U  k_union_surv: the survivors (~0.5 M of a late window's 16.8 M edges) are unioned, one per
//      lane (union_group_g: a giant member's parent read is replaced by the giant root gR).
// Lists are per (producer workgroup, part) regions with LDS cursors (no global atomics). A list
// entry past its region's capacity is decided in place from global gbits (a skewed stream degrades
// to the old filter, never to a wrong answer); survivors past a workgroup's region go to one shared
// overflow list (each edge yields at most one survivor, so n entries always suffice).
// Correctness rests on the same facts as k_fold_ring: gbits bit v = label(v) == gR at the last
// close, hot-set entries are members of that component, and components only merge until reset, so
// a "both in the giant" edge is already one component and x's union with any giant member is its
// union with gR.
#pragma once

#include "cc_kernels.hpp"

namespace gsgpu {

constexpr uint32_t kPartBits = 20;                       // ids per part: 2^20 = 128 KiB of gbits in LDS
constexpr uint32_t kPartWords = 1u << (kPartBits - 5);
constexpr uint32_t kRouteMaxParts = 64;                  // one part cursor per lane: ids < 2^26
constexpr int kSiftWaves = 15;                           // 128 KiB hot set + 15 x 2 KiB staging in LDS
constexpr int kSiftThreads = 64 * kSiftWaves;
constexpr int kProbeWaves = 16;
constexpr int kProbeThreads = 64 * kProbeWaves;
constexpr uint32_t kSurvFlag = 0x80000000u;              // survivor entry: endpoint known in the giant

struct RouteArgs {
    uint32_t* qs;                // A singles   [grid][parts][cap]
    uint2* qd;                   // A doubles   [grid][parts][cap]
    uint32_t* qc;                // B -> C singles [grid][parts][cap]
    uint32_t* cnt;               // list lengths [3][grid][parts] (qs, qd, qc)
    uint2* surv;                 // survivors [3][grid][scap] (A, B, C)
    uint32_t* scnt;              // survivor counts [3][grid]
    uint2* over;                 // survivor overflow [ocap]
    unsigned long long* ocount;  // overflow count of this launch (zeroed by the previous launch)
    unsigned long long* onext;   // the next launch's overflow count (zeroed here)
    unsigned long long* admit;   // this launch admits into the hot set (written by A for B and C)
    uint64_t cap, scap, ocap;
    uint32_t parts;              // 2^(B - kPartBits), <= kRouteMaxParts
    uint32_t gwords;             // gbits words
    uint32_t grid;               // workgroups of every routed kernel (a multiple of parts)
    uint32_t exp;                // timing lab only (GSGPU_ROUTE_EXP, wrong results on purpose): bit 0 = A
                                 // stores no list entry, bit 1 = A skips the sort, bit 2 = A skips the probes;
                                 // (results unchanged) bit 3 = list and survivor counts on stderr, bit 4 =
                                 // the field-by-field hot-set match
};

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }

// exclusive prefix sum over the wave's 64 lanes (all lanes active)
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t& total) {
    const int lane = lane_id();
    uint32_t incl = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    total = __shfl(incl, 63, 64);
    return incl - x;
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ bool gbit(const uint32_t* __restrict__ gbits, uint32_t v) {
    return (gbits[v >> 5] >> (v & 31)) & 1u;
}

// Survivor append (any set of active lanes): the wave's survivors go to this workgroup's region of
// kind `kind` at an LDS cursor; past the region, to the shared overflow list.
__device__ __forceinline__ void surv_push(const RouteArgs& r, int kind, uint32_t* lsurv, bool keep, uint2 e,
                                          uint32_t* err) {
    const uint64_t m = __ballot(keep);
    if (m == 0) return;
    const uint64_t act = __ballot(1);
    const int leader = __ffsll((long long)act) - 1;
    uint32_t base = 0;
    if ((int)lane_id() == leader) base = atomicAdd(lsurv, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    if (!keep) return;
    const uint64_t pos = base + __popcll(m & ((1ull << lane_id()) - 1));
    if (pos < r.scap) {
        r.surv[((uint64_t)kind * r.grid + blockIdx.x) * r.scap + pos] = e;
    } else {
        const unsigned long long o = atomicAdd(r.ocount, 1ull);
        if (o < r.ocap) r.over[o] = e;
        else atomicOr(err, 4u);                       // impossible: at most one survivor per edge
    }
}

// Per-wave counting sort of up to 4 x 64 entries by part, then one coalesced store per part run.
// Every lane calls with its K candidate entries (val[k] valid where part[k] < parts); the stage
// holds K x 64 x W words: first the histogram (64 words), then, once it is read, the sorted
// entries (W words each) over it. Lists: region of
// part p of this workgroup = base + p * cap, cursor lcur[p] (LDS, shared by the workgroup's waves).
// Returns, per entry, whether it spilled (its list was full): the caller decides those in place.
template <int K, int W>
__device__ __forceinline__ void wave_route(uint32_t* __restrict__ st, uint32_t* __restrict__ lcur,
                                           uint32_t* __restrict__ list, uint64_t cap, uint32_t parts,
                                           const uint32_t (&part)[K], const uint32_t (&val0)[K],
                                           const uint32_t (&val1)[K], bool (&spill)[K], bool store = true) {
    const uint32_t lane = lane_id();
    st[lane] = 0u;
    wave_lds_sync();
    uint32_t rank[K];
#pragma unroll
    for (int k = 0; k < K; ++k) rank[k] = part[k] < parts ? atomicAdd(&st[part[k]], 1u) : 0u;
    wave_lds_sync();
    const uint32_t c = st[lane];                     // lanes >= parts read 0 (never incremented)
    uint32_t total;
    const uint32_t b = wave_excl_scan(c, total);    // this lane's part: first slot in the stage
    const uint32_t o = c ? atomicAdd(&lcur[lane], c) : 0u;   // list offset of the wave's run
    wave_lds_sync();
    uint32_t* const sv = st;                         // sorted entries over the (read) histogram
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t pk = part[k] < parts ? part[k] : 0u;
        const uint32_t slot = __shfl(b, (int)pk, 64) + rank[k];
        if (part[k] < parts) {
            sv[W * slot] = val0[k];
            if (W == 2) sv[W * slot + 1] = val1[k];
        }
    }
    wave_lds_sync();
    // copy-out: the lanes take the sorted entries in order; a part's run lands contiguously
    uint32_t sp[K];
#pragma unroll
    for (int k = 0; k < K; ++k) sp[k] = 0u;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const uint32_t i = (uint32_t)j * 64 + lane;
        const bool live = i < total;
        const uint32_t x0 = live ? sv[W * i] : 0u;
        const uint32_t x1 = (live && W == 2) ? sv[W * i + 1] : 0u;
        const uint32_t p = live ? (x0 >> kPartBits) : 0u;
        const uint32_t pb = __shfl(b, (int)p, 64), po = __shfl(o, (int)p, 64);
        const uint64_t at = (uint64_t)po + (i - pb);
        if (live && store) {
            if (at < cap) {
                if (W == 2) reinterpret_cast<uint2*>(list)[(uint64_t)p * cap + at] = make_uint2(x0, x1);
                else list[(uint64_t)p * cap + at] = x0;
            } else {
                sp[j] = 1u;
            }
        }
    }
    wave_lds_sync();
    // spilled entries back to their owners' k slots: rare; the caller re-decides them by value
#pragma unroll
    for (int k = 0; k < K; ++k) spill[k] = false;
    uint32_t any = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) any |= sp[j];
    if (__ballot(any != 0) == 0) return;            // uniform: the common case
    // mark spilled sorted slots in the stage (histogram area is free now), owners check theirs
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const uint32_t i = (uint32_t)j * 64 + lane;
        if (i < total) sv[W * i] = sp[j] ? kInvalid : sv[W * i];
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t pk = part[k] < parts ? part[k] : 0u;
        const uint32_t slot = __shfl(b, (int)pk, 64) + rank[k];
        spill[k] = part[k] < parts && sv[W * slot] == kInvalid;
    }
    wave_lds_sync();
}

// As wave_route, for A's singles and doubles together (one histogram of 2 x 64 keys, one sort):
// key = part for a single x (entry (x, kInvalid), stored as 4 B into lists_s), 64 + part for a double
// (u, v) (8 B into lists_d). The stage holds 256 uint2 (2 KiB).
__device__ __forceinline__ void wave_route2(uint2* __restrict__ st, uint32_t* __restrict__ lcur_s, uint32_t* __restrict__ lcur_d,
                                            uint32_t* __restrict__ lists_s, uint2* __restrict__ lists_d, uint64_t cap,
                                            uint32_t parts, const uint32_t (&key)[4], const uint32_t (&x0)[4],
                                            const uint32_t (&x1)[4], bool (&spill)[4], bool store) {
    const uint32_t lane = lane_id();
    uint32_t* const hist = reinterpret_cast<uint32_t*>(st);      // 128 counters over the stage
    hist[lane] = 0u;
    hist[64 + lane] = 0u;
    wave_lds_sync();
    uint32_t rank[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) rank[k] = key[k] != kInvalid ? atomicAdd(&hist[key[k]], 1u) : 0u;
    wave_lds_sync();
    const uint32_t cs = hist[lane], cd = hist[64 + lane];
    uint32_t ts, td;
    const uint32_t bs = wave_excl_scan(cs, ts);
    const uint32_t bd = ts + wave_excl_scan(cd, td);  // doubles after every single
    const uint32_t total = ts + td;
    const uint32_t os = cs ? atomicAdd(&lcur_s[lane], cs) : 0u;
    const uint32_t od = cd ? atomicAdd(&lcur_d[lane], cd) : 0u;
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t kk = key[k] != kInvalid ? key[k] : 0u;
        const uint32_t b1 = __shfl(bs, (int)(kk & 63), 64), b2 = __shfl(bd, (int)(kk & 63), 64);   // every lane
        const uint32_t b = kk < 64 ? b1 : b2;
        if (key[k] != kInvalid) st[b + rank[k]] = make_uint2(x0[k], kk < 64 ? kInvalid : x1[k]);
    }
    wave_lds_sync();
    uint32_t sp = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t i = (uint32_t)j * 64 + lane;
        const bool live = i < total;
        const uint2 e = live ? st[i] : make_uint2(0u, 0u);
        const bool single = e.y == kInvalid;
        const uint32_t p = live ? (e.x >> kPartBits) : 0u;
        const uint32_t b1 = __shfl(bs, (int)p, 64), b2 = __shfl(bd, (int)p, 64);           // every lane
        const uint32_t o1 = __shfl(os, (int)p, 64), o2 = __shfl(od, (int)p, 64);
        const uint32_t b = single ? b1 : b2, o = single ? o1 : o2;
        const uint64_t at = (uint64_t)o + (i - b);
        if (live && store) {
            if (at < cap) {
                if (single) lists_s[(uint64_t)p * cap + at] = e.x;
                else lists_d[(uint64_t)p * cap + at] = e;
            } else {
                sp |= 1u << j;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) spill[k] = false;
    if (__ballot(sp != 0) == 0) {                    // uniform: the common case
        wave_lds_sync();
        return;
    }
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t i = (uint32_t)j * 64 + lane;
        if ((sp >> j) & 1u) st[i].x = kInvalid;
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t kk = key[k] != kInvalid ? key[k] : 0u;
        const uint32_t b1 = __shfl(bs, (int)(kk & 63), 64), b2 = __shfl(bd, (int)(kk & 63), 64);   // every lane
        const uint32_t b = kk < 64 ? b1 : b2;
        spill[k] = key[k] != kInvalid && st[b + rank[k]].x == kInvalid;
    }
    wave_lds_sync();
}

// A: stream + LDS hot set + per-part lists. One workgroup per CU, persistent over the batch.
template <typename IdT>
__global__ __launch_bounds__(kSiftThreads) void k_sift(const IdT* __restrict__ a, const IdT* __restrict__ b,
                                                       FoldArgs f, HotArgs hot, RouteArgs r) {
    __shared__ __attribute__((aligned(16))) uint2 tab[kHotBuckets];
    __shared__ __attribute__((aligned(16))) uint2 stage[kSiftWaves][256];
    __shared__ uint32_t lcur_s[kRouteMaxParts], lcur_d[kRouteMaxParts];
    __shared__ uint32_t lsurv;
    const uint64_t n = f.n;
    const bool filt = *f.giant != kInvalid;          // uniform
    if (filt) lds_fill<2 * kHotBuckets, kSiftThreads>(reinterpret_cast<uint32_t*>(tab),
                                                      reinterpret_cast<const uint32_t*>(hot.table), 2 * kHotBuckets);
    for (uint32_t p = threadIdx.x; p < kRouteMaxParts; p += blockDim.x) { lcur_s[p] = 0u; lcur_d[p] = 0u; }
    if (threadIdx.x == 0) lsurv = 0u;
    const uint32_t budget = hot.budget ? *hot.budget : 1u;
    const uint32_t gR = filt ? f.giant[1] : kInvalid;
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (hot.budget && budget) *hot.budget = budget - 1;
        *r.admit = (hot.periodic || budget) ? 1ull : 0ull;      // B and C admit into the hot set
        *r.onext = 0ull;                                        // the next launch's overflow count
    }
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    uint2* const st = stage[wave];
    uint32_t* const lists_s = r.qs + (uint64_t)blockIdx.x * r.parts * r.cap;
    uint2* const lists_d = r.qd + (uint64_t)blockIdx.x * r.parts * r.cap;
    const bool five = hot.five != 0;
    const uint64_t groups = n / 4;
    const uint64_t stride = (uint64_t)gridDim.x * kSiftThreads;
    // the next wave step's edges are loaded while this one is decided (16 B per lane per array)
    uint64_t g0 = ((uint64_t)blockIdx.x * kSiftWaves + wave) * 64;
    Raw4<IdT> ra, rb;
    if (g0 + lane < groups) {
        ra.load(a, g0 + lane);
        rb.load(b, g0 + lane);
    }
    for (; g0 < groups; g0 += stride) {
        const uint64_t g = g0 + lane;
        Raw4<IdT> na, nb;
        if (g + stride < groups) {
            na.load(a, g + stride);
            nb.load(b, g + stride);
        }
        uint32_t u[4] = {0, 0, 0, 0}, v[4] = {0, 0, 0, 0};
        bool ok[4] = {false, false, false, false};
        if (g < groups) {
            bool oka[4] = {true, true, true, true}, okb[4] = {true, true, true, true};
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
        ra = na;
        rb = nb;
        bool hu[4] = {false, false, false, false}, hv[4] = {false, false, false, false};
        if (filt && !(r.exp & 4u)) {
            uint2 bu[4], bv[4];
            uint32_t ru[4], rv[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                bu[k] = tab[hot_bucket(u[k], hot.bits, ru[k])];
                bv[k] = tab[hot_bucket(v[k], hot.bits, rv[k])];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                hu[k] = (r.exp & 16u) ? hot_match_fields(bu[k], ru[k], five) : hot_match(bu[k], ru[k], five);
                hv[k] = (r.exp & 16u) ? hot_match_fields(bv[k], rv[k], five) : hot_match(bv[k], rv[k], five);
            }
        }
        // singles: one endpoint known (key = part); doubles: none (key = 64 + part of u); no giant
        // yet: every edge survives as it is
        uint32_t key[4], xs[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool single = filt && ok[k] && (hu[k] != hv[k]);
            const bool dbl = filt && ok[k] && !hu[k] && !hv[k];
            xs[k] = hu[k] ? v[k] : u[k];
            key[k] = single ? (xs[k] >> kPartBits) : dbl ? 64u + (u[k] >> kPartBits) : kInvalid;
        }
        bool spl[4] = {false, false, false, false};
        if (r.exp & 2u) {                            // timing lab: no sort, no stores
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) x += key[k];
            if (x == 0x12345678u) st[lane].x = x;
        } else {
            wave_route2(st, lcur_s, lcur_d, lists_s, lists_d, r.cap, r.parts, key, xs, v, spl, !(r.exp & 1u));
        }
        // no giant: survivors as they are; spilled entries: decided from global gbits (rare)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            bool keep = !filt && ok[k];
            uint2 e = make_uint2(u[k], v[k]);
            const bool sps = spl[k] && key[k] < 64, spd = spl[k] && key[k] >= 64;
            if (sps && !gbit(f.gbits, xs[k])) { keep = true; e = make_uint2(gR | kSurvFlag, xs[k]); }
            if (spd) {
                const bool gu = gbit(f.gbits, u[k]), gv = gbit(f.gbits, v[k]);
                if (!(gu && gv)) {
                    keep = true;
                    e = make_uint2(gu ? (gR | kSurvFlag) : u[k], gv ? (gR | kSurvFlag) : v[k]);
                }
            }
            surv_push(r, 0, &lsurv, keep, e, f.rc.err);
        }
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < r.parts; p += blockDim.x) {
        r.cnt[(uint64_t)blockIdx.x * r.parts + p] = (uint32_t)min((uint64_t)lcur_s[p], r.cap);
        r.cnt[((uint64_t)r.grid + blockIdx.x) * r.parts + p] = (uint32_t)min((uint64_t)lcur_d[p], r.cap);
    }
    if (threadIdx.x == 0) r.scnt[blockIdx.x] = (uint32_t)min((uint64_t)lsurv, r.scap);
}

// B (FIRST) / C: the part's gbits slice in LDS. Workgroup b owns part b % parts (b and b + parts
// share an XCD when parts is a multiple of 8: the slice is fetched into that XCD's L2 once) and
// reads the lists of producers j == b / parts (mod wpp). The lists are cut into chunks of 256
// entries (a 16-B load per lane for singles, two for doubles) numbered through an LDS prefix over
// the workgroup's lists; a wave takes kProbeBatch chunks at a time and issues every load of the
// batch before deciding the first entry (one chunk at a time left the kernel latency-bound: a
// list read is a few hundred entries).
constexpr int kProbeBatch = 4;
constexpr uint32_t kProbeMaxLists = 256;             // lists per workgroup and kind (grid / parts <= 256)

template <bool FIRST>
__global__ __launch_bounds__(kProbeThreads) void k_probe(FoldArgs f, HotArgs hot, RouteArgs r) {
    __shared__ __attribute__((aligned(16))) uint32_t slice[kPartWords];
    __shared__ __attribute__((aligned(16))) uint32_t stage[kProbeWaves][256];
    __shared__ uint32_t lcur[kRouteMaxParts];
    __shared__ uint32_t pre_s[kProbeMaxLists + 1], pre_d[kProbeMaxLists + 1];
    __shared__ uint32_t len_s[kProbeMaxLists], len_d[kProbeMaxLists];
    __shared__ uint32_t lsurv;
    const uint32_t p = blockIdx.x % r.parts, sub = blockIdx.x / r.parts, wpp = gridDim.x / r.parts;
    const uint32_t nl = (r.grid - sub + wpp - 1) / wpp;       // producer lists j = sub + i * wpp
    const uint64_t sw = (uint64_t)p * kPartWords;
    lds_fill<kPartWords, kProbeThreads>(slice, f.gbits + sw, r.gwords > sw ? r.gwords - sw : 0);
    for (uint32_t q = threadIdx.x; q < kRouteMaxParts; q += blockDim.x) lcur[q] = 0u;
    if (threadIdx.x == 0) lsurv = 0u;
    const uint32_t* const cs = FIRST ? r.cnt : r.cnt + 2ull * r.grid * r.parts;
    const uint32_t* const cd = r.cnt + (uint64_t)r.grid * r.parts;
    for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x) {
        const uint64_t j = sub + (uint64_t)i * wpp;
        len_s[i] = cs[j * r.parts + p];
        if (FIRST) len_d[i] = cd[j * r.parts + p];
    }
    __syncthreads();
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    if (wave == 0) {                                 // chunk prefixes over the lists
        uint32_t carry_s = 0, carry_d = 0;
        for (uint32_t i0 = 0; i0 < nl; i0 += 64) {
            const uint32_t i = i0 + lane;
            const uint32_t ns = i < nl ? (len_s[i] + 255) / 256 : 0u;
            const uint32_t nd = (FIRST && i < nl) ? (len_d[i] + 255) / 256 : 0u;
            uint32_t ts, td;
            const uint32_t es = wave_excl_scan(ns, ts), ed = wave_excl_scan(nd, td);
            if (i < nl) { pre_s[i] = carry_s + es; pre_d[i] = carry_d + ed; }
            carry_s += ts;
            carry_d += td;
        }
        if (lane == 0) { pre_s[nl] = carry_s; pre_d[nl] = carry_d; }
    }
    __syncthreads();
    const uint32_t gR = f.giant[1];
    const bool admit = hot.table && *r.admit != 0;
    const uint32_t sample = admit ? (uint32_t)min<uint64_t>(2 * hot.sample_edges / ((uint64_t)r.grid * r.parts), 4096) : 0u;
    uint32_t* const st = stage[wave];
    uint32_t* const out = r.qc + (uint64_t)blockIdx.x * r.parts * r.cap;
    const uint32_t base_v = p << kPartBits;
    auto in_giant = [&](uint32_t x) -> bool {
        const uint32_t lx = x - base_v;
        return (slice[(lx >> 5) & (kPartWords - 1)] >> (lx & 31)) & 1u;
    };
    const int kind = FIRST ? 1 : 2;
    // singles: A's (FIRST) or B's (C): x in the giant -> dropped, else a survivor joining the giant
    const uint32_t* const qs = FIRST ? r.qs : r.qc;
    const uint32_t ncs = pre_s[nl];
    uint32_t li = 0;                                 // list of the wave's current chunk (chunks ascend)
    for (uint32_t c0 = wave; c0 < ncs; c0 += kProbeWaves * kProbeBatch) {
        u32x4 raw[kProbeBatch];
        uint32_t len[kProbeBatch], e0[kProbeBatch];
#pragma unroll
        for (int b = 0; b < kProbeBatch; ++b) {
            const uint32_t c = c0 + b * kProbeWaves;
            len[b] = 0;
            e0[b] = 0;
            raw[b] = u32x4{base_v, base_v, base_v, base_v};
            if (c < ncs) {                           // uniform
                while (pre_s[li + 1] <= c) ++li;
                const uint32_t i = __builtin_amdgcn_readfirstlane(li);
                len[b] = len_s[i];
                e0[b] = (c - pre_s[i]) * 256 + 4 * lane;
                const uint32_t* lp = qs + ((uint64_t)(sub + i * wpp) * r.parts + p) * r.cap;
                if (e0[b] < len[b]) raw[b] = *reinterpret_cast<const u32x4*>(lp + e0[b]);
            }
        }
#pragma unroll
        for (int b = 0; b < kProbeBatch; ++b) {
            const uint32_t x[4] = {raw[b].x, raw[b].y, raw[b].z, raw[b].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool live = e0[b] + k < len[b];
                const bool g = live && in_giant(x[k]);
                if (g && e0[b] + k < sample) hot_admit(hot, x[k]);
                surv_push(r, kind, &lsurv, live && !g, make_uint2(gR | kSurvFlag, x[k]), f.rc.err);
            }
        }
    }
    if (FIRST) {                                     // A's doubles: u here, v routed to C
        const uint2* const qd = r.qd;
        const uint32_t ncd = pre_d[nl];
        uint32_t li = 0;
        for (uint32_t c0 = wave; c0 < ncd; c0 += kProbeWaves * kProbeBatch) {
            u32x4 raw[kProbeBatch][2];
            uint32_t len[kProbeBatch], e0[kProbeBatch];
#pragma unroll
            for (int b = 0; b < kProbeBatch; ++b) {
                const uint32_t c = c0 + b * kProbeWaves;
                len[b] = 0;
                e0[b] = 0;
                raw[b][0] = raw[b][1] = u32x4{base_v, base_v, base_v, base_v};
                if (c < ncd) {
                    while (pre_d[li + 1] <= c) ++li;
                    const uint32_t i = __builtin_amdgcn_readfirstlane(li);
                    len[b] = len_d[i];
                    e0[b] = (c - pre_d[i]) * 256 + 2 * lane;       // entries e0, e0+1 and e0+128, e0+129
                    const uint2* lp = qd + ((uint64_t)(sub + i * wpp) * r.parts + p) * r.cap;
                    if (e0[b] < len[b]) raw[b][0] = *reinterpret_cast<const u32x4*>(lp + e0[b]);
                    if (e0[b] + 128 < len[b]) raw[b][1] = *reinterpret_cast<const u32x4*>(lp + e0[b] + 128);
                }
            }
#pragma unroll
            for (int b = 0; b < kProbeBatch; ++b) {
                const uint32_t u[4] = {raw[b][0].x, raw[b][0].z, raw[b][1].x, raw[b][1].z};
                const uint32_t v[4] = {raw[b][0].y, raw[b][0].w, raw[b][1].y, raw[b][1].w};
                const uint32_t ei[4] = {e0[b], e0[b] + 1, e0[b] + 128, e0[b] + 129};
                uint32_t pv[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const bool live = ei[k] < len[b];
                    const bool gu = live && in_giant(u[k]);
                    if (gu && ei[k] < sample) hot_admit(hot, u[k]);
                    // v in this same part: decided here
                    const bool here = gu && (v[k] >> kPartBits) == p;
                    const bool gv = here && in_giant(v[k]);
                    pv[k] = (gu && !here) ? (v[k] >> kPartBits) : kInvalid;
                    const bool keep = (live && !gu) || (here && !gv);
                    const uint2 e = !gu ? make_uint2(u[k], v[k]) : make_uint2(gR | kSurvFlag, v[k]);
                    surv_push(r, kind, &lsurv, keep, e, f.rc.err);
                }
                bool sp[4];
                wave_route<4, 1>(st, lcur, out, r.cap, r.parts, pv, v, v, sp);
#pragma unroll
                for (int k = 0; k < 4; ++k) {    // spilled: v from global gbits
                    const bool keep = sp[k] && !gbit(f.gbits, v[k]);
                    surv_push(r, kind, &lsurv, keep, make_uint2(gR | kSurvFlag, v[k]), f.rc.err);
                }
            }
        }
    }
    __syncthreads();
    if (FIRST)
        for (uint32_t q = threadIdx.x; q < r.parts; q += blockDim.x)
            r.cnt[(2ull * r.grid + blockIdx.x) * r.parts + q] = (uint32_t)min((uint64_t)lcur[q], r.cap);
    if (threadIdx.x == 0) r.scnt[(uint64_t)kind * r.grid + blockIdx.x] = (uint32_t)min((uint64_t)lsurv, r.scap);
}

// U: the survivors of A, B and C (3 x grid regions) and the overflow list, unioned kUnionEpt per
// lane with their parent gathers issued together (union_group_g). kUnionSplit blocks share a
// region (a young window's regions hold thousands of survivors each); the blocks past the
// regions stride over the overflow list. (One index space over all regions through an LDS prefix
// put a binary search in front of every survivor: late windows 14 -> 23 us.)
constexpr int kUnionEpt = 2;
constexpr uint32_t kUnionSplit = 4;
constexpr uint32_t kUnionMaxRegions = 3 * 256 + 1;

template <bool MARK>
__global__ __launch_bounds__(256) void k_union_surv(FoldArgs f, RouteArgs r, uint32_t overflow_blocks) {
    const uint32_t gR = f.giant[1];
    FoldStats st;
    const uint32_t regions = 3 * r.grid;
    const uint2* src;
    uint64_t n, i0, step;
    if (blockIdx.x < regions * kUnionSplit) {
        const uint32_t reg = blockIdx.x / kUnionSplit, part = blockIdx.x % kUnionSplit;
        src = r.surv + (uint64_t)reg * r.scap;
        n = r.scnt[reg];
        i0 = ((uint64_t)part * blockDim.x + threadIdx.x) * kUnionEpt;
        step = (uint64_t)kUnionSplit * blockDim.x * kUnionEpt;
    } else {
        src = r.over;
        const unsigned long long o = *r.ocount;
        n = o < r.ocap ? o : r.ocap;
        i0 = ((uint64_t)(blockIdx.x - regions * kUnionSplit) * blockDim.x + threadIdx.x) * kUnionEpt;
        step = (uint64_t)overflow_blocks * blockDim.x * kUnionEpt;
    }
    for (uint64_t i = i0; i < n; i += step) {
        uint32_t u[kUnionEpt], v[kUnionEpt], gf[kUnionEpt];
        bool ok[kUnionEpt];
#pragma unroll
        for (int k = 0; k < kUnionEpt; ++k) {
            ok[k] = i + k < n;
            const uint2 e = ok[k] ? src[i + k] : make_uint2(0u, 0u);
            const uint32_t fu = e.x >> 31, fv = e.y >> 31;
            u[k] = fu ? gR : e.x;
            v[k] = fv ? gR : e.y;
            gf[k] = fu | (fv << 1);
        }
        union_group_g<MARK, false, kUnionEpt>(f, u, v, ok, gf, gR, st);
    }
}

}  // namespace gsgpu
