// route_fold.hpp — EXPERIMENT (make exp EXP=ROUTE; not in the product library): the steady fold
// with the giant filter read from LDS slices of gbits instead of L2 lookups. Parity-green on the
// headline stream and the variant streams; measured 239 us per steady RMAT-26 window (A 98, B 100,
// C 41 us) against k_fold_ring's 209 us (profiles/r02_ab_experiments.txt r02_aj..r02_an, DESIGN.md
// section 8). Included by cc_api.hip only under GS_EXP_ROUTE.
#pragma once

#include "cc_kernels.hpp"

namespace gsgpu {

// ---- routed steady fold: the giant filter out of LDS slices of gbits ----
// The ring fold's filter is bound by L2 requests: ~10 M gbits lookups per RMAT-26 window miss an
// XCD's 4 MiB L2 half the time (8 MiB bitmap) and random misses run at ~59 G/s chip-wide
// (tools/request_lab.hip), the warm set's L2 hits at ~260 G/s. Here no filter lookup leaves the CU:
//   A (k_route_a): streams the edges, drops those whose endpoints both hit the LDS hot set, and
//      appends the rest to per-part lists by their first endpoint the hot set did not answer
//      (part = id >> 20: 2^20 vertices, 128 KiB of gbits);
//   B (k_route_bc<true>): a workgroup loads its part's gbits slice into LDS and decides each listed
//      edge from it: the looked-up endpoint outside the giant -> survivor; inside and the other
//      endpoint known -> dropped; inside and the other unknown -> listed for the other's part;
//   C (k_route_bc<false>): as B for those (the second endpoint).
// Survivors go through the wave-private LDS rings and union_group_g as in k_fold_ring.
// Lists: every workgroup of a launch owns one region of cap entries per part (append cursor in
// LDS: no global atomic, no barrier), written (u | hu << 31, v | hv << 31) with bit 31 = that
// endpoint is a known giant member (ids < 2^31 on this path); its counts go to cnt[] at the end.
// An entry past its region's capacity is decided in place from global gbits (a skewed stream
// degrades to the ring fold's filter).
constexpr uint32_t kSliceBits = 20;                  // vertices per part: 2^20 bits = 128 KiB of LDS
constexpr uint32_t kSliceWords = 1u << (kSliceBits - 5);
constexpr uint32_t kMaxParts = 512;                  // ids < 2^29
constexpr uint32_t kMaxRouteGrid = 1024;
constexpr int kRouteThreads = 1024;
constexpr uint32_t kRouteChunk = 128;                // entries per wave work item in B / C (2 per lane)
constexpr int kBcItems = 2;                          // work items a wave loads before deciding the first

struct RouteArgs {
    uint2* qa;                     // A's lists: [grid][parts][cap]
    uint2* qb;                     // B's lists: [grid][parts][cap]
    uint32_t* cnt;                 // [2][grid][parts] list lengths (A's, then B's)
    unsigned long long* flags;     // [0]: this launch admits into the hot set (written by A)
    uint64_t cap;                  // entries per list
    uint32_t parts;                // 2^(B - kSliceBits), at least 1
    uint32_t gwords;               // gbits words (capacity / 32, rounded up)
};

__device__ __forceinline__ bool gbit(const uint32_t* __restrict__ gbits, uint32_t v) {
    return (gbits[v >> 5] >> (v & 31)) & 1u;
}

// Survivors into the wave's ring (one call per wave step, uniform), as k_fold_ring does
template <bool MARK, bool STATS, int N>
__device__ __forceinline__ void ring_push(const FoldArgs& f, uint2* ring, uint32_t& cnt, const uint32_t (&u)[N],
                                          const uint32_t (&v)[N], const bool (&ok)[N], const uint32_t (&gf)[N],
                                          uint32_t gR, FoldStats& st) {
    const int lane = threadIdx.x & 63;
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) c += ok[k];
    uint32_t incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    const uint32_t wtot = __shfl(incl, 63, 64);
    if (wtot == 0) return;                           // uniform
    if (wtot > kRingCap / 2) {                       // young window: union in place
        union_group_g<MARK, STATS, N>(f, u, v, ok, gf, gR, st);
        return;
    }
    if (cnt + wtot > kRingCap) ring_flush<MARK, STATS>(f, ring, cnt, kRingCap - wtot, st, gR);
    uint32_t pos = cnt + incl - c;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        if (!ok[k]) continue;
        ring[pos] = make_uint2(u[k] | ((gf[k] & 1u) << 31), v[k] | ((gf[k] >> 1) << 31));
        ++pos;
    }
    cnt += wtot;
    if (cnt >= 64) ring_flush<MARK, STATS>(f, ring, cnt, cnt - 64, st, gR);
}

// A: stream + LDS hot set + append to the part lists. One 1024-thread workgroup per CU; waves run
// free (no barrier until the end).
template <typename IdT, bool MARK, bool STATS>
__global__ __launch_bounds__(kRouteThreads) void k_route_a(const IdT* __restrict__ a, const IdT* __restrict__ b,
                                                           FoldArgs f, HotArgs hot, RouteArgs r) {
    __shared__ __attribute__((aligned(16))) uint2 tab[kHotBuckets];
    __shared__ uint32_t lcur[kMaxParts];
    __shared__ uint2 rings[kRouteThreads / 64][kRingCap];          // survivors of overfull lists (rare)
    const uint64_t n = f.n;
    const bool filt = *f.giant != kInvalid;          // uniform (the host routes only past the young forest)
    if (filt) lds_fill<2 * kHotBuckets>(reinterpret_cast<uint32_t*>(tab), reinterpret_cast<const uint32_t*>(hot.table), 2 * kHotBuckets);
    else for (uint32_t i = threadIdx.x; i < kHotBuckets; i += blockDim.x) tab[i] = make_uint2(0u, 0u);
    for (uint32_t p = threadIdx.x; p < r.parts; p += blockDim.x) lcur[p] = 0u;
    const uint32_t gR = f.giant[1];
    const uint32_t budget = hot.budget ? *hot.budget : 1u;
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (hot.budget && budget) *hot.budget = budget - 1;
        r.flags[0] = (hot.periodic || budget) ? 1ull : 0ull;            // B and C admit this launch
    }
    const int lane = threadIdx.x & 63;
    uint2* const ring = rings[threadIdx.x >> 6];
    uint2* const mine = r.qa + (uint64_t)blockIdx.x * r.parts * r.cap;
    uint32_t cnt = 0;
    FoldStats st;
    // a wave step takes 2 x 64 groups of 4 edges (8 edges per lane, four 16-B loads in flight)
    const uint64_t groups = n / 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 2;
    for (uint64_t g0 = ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) * 2; g0 < groups; g0 += stride) {
        uint32_t u[8], v[8];
        bool ok[8];
        Raw4<IdT> ra[2], rb[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint64_t g = g0 + h * 64 + lane;
            if (g < groups) {
                ra[h].load(a, g);
                rb[h].load(b, g);
            }
        }
        bool bad = false;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint64_t g = g0 + h * 64 + lane;
            uint32_t uu[4] = {0, 0, 0, 0}, vv[4] = {0, 0, 0, 0};
            bool oka[4] = {true, true, true, true}, okb[4] = {true, true, true, true};
            if (g < groups) {
                ra[h].unpack(uu, oka, f.rc.cap);
                rb[h].unpack(vv, okb, f.rc.cap);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool good = g < groups && oka[k] && okb[k];
                bad |= g < groups && !good;
                ok[4 * h + k] = good;
                u[4 * h + k] = good ? uu[k] : 0u;
                v[4 * h + k] = good ? vv[k] : 0u;
            }
        }
        if (bad) atomicOr(f.rc.err, 1u);
        uint2 bu[8], bv[8];
        uint32_t ru[8], rv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            bu[k] = tab[hot_bucket(u[k], hot.bits, ru[k])];
            bv[k] = tab[hot_bucket(v[k], hot.bits, rv[k])];
        }
        bool spill[8], hu[8], hv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            hu[k] = hot_match(bu[k], ru[k], hot.five != 0);
            hv[k] = hot_match(bv[k], rv[k], hot.five != 0);
            spill[k] = false;
            if (!ok[k] || (hu[k] && hv[k])) continue;                   // dropped: both in the giant
            const uint32_t part = (hu[k] ? v[k] : u[k]) >> kSliceBits;
            const uint32_t pos = atomicAdd(&lcur[part], 1u);
            if (pos < r.cap) mine[(uint64_t)part * r.cap + pos] = make_uint2(u[k] | ((uint32_t)hu[k] << 31), v[k] | ((uint32_t)hv[k] << 31));
            else spill[k] = true;
        }
        uint32_t gf[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {                                  // overfull list: decide in place
            const bool gu = spill[k] && (hu[k] || gbit(f.gbits, u[k]));
            const bool gv = spill[k] && (hv[k] || gbit(f.gbits, v[k]));
            gf[k] = gR == kInvalid ? 0u : ((uint32_t)gu | ((uint32_t)gv << 1));
            spill[k] = spill[k] && !(gu && gv);
        }
        ring_push<MARK, STATS, 8>(f, ring, cnt, u, v, spill, gf, gR, st);
    }
    ring_flush<MARK, STATS>(f, ring, cnt, 0, st, gR);
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < r.parts; p += blockDim.x)
        r.cnt[(uint64_t)blockIdx.x * r.parts + p] = (uint32_t)min((uint64_t)lcur[p], r.cap);
    if (STATS) {
        atomicAdd(&f.stats[3], (unsigned long long)st.hooks);
        atomicAdd(&f.stats[5], (unsigned long long)st.inits);
    }
}

// B / C: the part's gbits slice in LDS. gridDim / parts workgroups share a part (with more parts
// than workgroups, a workgroup takes parts in rounds); a workgroup reads the part's lists of every
// other wpp-th producer workgroup, cut into work items of kRouteChunk entries that its waves take
// in turn. FWD (B) looks up an entry's first unknown endpoint: outside the giant -> survivor;
// inside with the other endpoint known -> dropped; inside with the other unknown -> listed for the
// other's part. !FWD (C) looks up the listed entry's v (u confirmed in B).
template <bool FWD, bool MARK, bool STATS>
__global__ __launch_bounds__(kRouteThreads) void k_route_bc(FoldArgs f, HotArgs hot, RouteArgs r) {
    __shared__ __attribute__((aligned(16))) uint32_t slice[kSliceWords];
    __shared__ uint32_t lcur[kMaxParts];
    __shared__ uint32_t ipre[kMaxRouteGrid + 1];     // work items before list j
    __shared__ uint32_t llen[kMaxRouteGrid];         // list j's length
    __shared__ uint2 rings[kRouteThreads / 64][kRingCap];
    const uint32_t gR = f.giant[1];
    const uint2* const q = FWD ? r.qa : r.qb;
    const uint32_t* const qn = FWD ? r.cnt : r.cnt + (uint64_t)gridDim.x * r.parts;
    const bool admit = hot.table && r.flags[0] != 0;
    // admission: the first entries of every list, about 2 x sample_edges endpoint offers in all
    const uint64_t sample = 2 * hot.sample_edges / ((uint64_t)gridDim.x * r.parts);
    if (FWD)
        for (uint32_t p = threadIdx.x; p < r.parts; p += blockDim.x) lcur[p] = 0u;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint2* const ring = rings[wave];
    uint2* const mine = r.qb + (uint64_t)blockIdx.x * r.parts * r.cap;
    uint32_t cnt = 0;
    FoldStats st;
    const uint32_t wpp = max(1u, gridDim.x / r.parts);             // workgroups per part
    const uint32_t pstride = gridDim.x / wpp;
    const uint32_t sub = blockIdx.x % wpp;
    const uint32_t nlist = (gridDim.x - sub + wpp - 1) / wpp;       // producer lists this workgroup reads
    const uint32_t rounds = (r.parts + pstride - 1) / pstride;
    for (uint32_t rd = 0; rd < rounds; ++rd) {
        const uint32_t p = blockIdx.x / wpp + rd * pstride;
        const bool live = p < r.parts && blockIdx.x / wpp < pstride;      // uniform
        __syncthreads();                             // the previous round's readers are done
        if (live) {
            lds_fill<kSliceWords>(slice, f.gbits + (uint64_t)p * kSliceWords,
                                  r.gwords > p * kSliceWords ? r.gwords - (uint64_t)p * kSliceWords : 0);
            // work items per list, then an exclusive scan by wave 0
            for (uint32_t j = threadIdx.x; j < nlist; j += blockDim.x) {
                const uint32_t len = qn[(uint64_t)(sub + j * wpp) * r.parts + p];
                llen[j] = len;
                ipre[j + 1] = (len + kRouteChunk - 1) / kRouteChunk;
            }
        } else {
            for (uint32_t j = threadIdx.x; j < nlist; j += blockDim.x) {
                llen[j] = 0u;
                ipre[j + 1] = 0u;
            }
        }
        __syncthreads();
        if (wave == 0) {
            uint32_t carry = 0;
            for (uint32_t j0 = 0; j0 < nlist; j0 += 64) {
                uint32_t x = (j0 + lane < nlist) ? ipre[j0 + lane + 1] : 0u;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t y = __shfl_up(x, off, 64);
                    if (lane >= off) x += y;
                }
                if (j0 + lane < nlist) ipre[j0 + lane + 1] = x + carry;
                carry += __shfl(x, 63, 64);
            }
            if (lane == 0) ipre[0] = 0u;
        }
        __syncthreads();
        const uint32_t items = ipre[nlist];
        const uint32_t base_v = p << kSliceBits;
        // a wave takes kBcItems work items per pass, every item's entries loaded (16 B per lane:
        // entries 2 lane, 2 lane + 1) before the first is decided
        constexpr uint32_t kWaves = kRouteThreads / 64;
        for (uint32_t it0 = wave; it0 < items; it0 += kWaves * kBcItems) {
            u32x4 raw[kBcItems];
            uint32_t len2[kBcItems];                 // entries of the item this lane holds: 0, 1 or 2
            uint32_t e0s[kBcItems];
#pragma unroll
            for (int j = 0; j < kBcItems; ++j) {
                const uint32_t it = it0 + j * kWaves;
                uint32_t lo = 0, hi = nlist;         // list: ipre[lo] <= it < ipre[lo + 1]
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (ipre[mid] <= it) lo = mid; else hi = mid;
                }
                lo = __builtin_amdgcn_readfirstlane(lo);         // wave-uniform: list addressing in SGPRs
                const bool live_it = it < items;
                const uint32_t prod = sub + lo * wpp;
                const uint32_t len = live_it ? llen[lo] : 0u;
                const uint32_t e0 = live_it ? (it - ipre[lo]) * kRouteChunk : 0u;
                const uint32_t i = e0 + 2 * lane;
                len2[j] = i < len ? min(len - i, 2u) : 0u;
                e0s[j] = i;
                const uint2* const lp = q + ((uint64_t)prod * r.parts + p) * r.cap;
                // lists start 16-B aligned (cap even), so entries (i, i + 1) are one 16-B load
                raw[j] = len2[j] == 2 ? *reinterpret_cast<const u32x4*>(lp + i)
                       : len2[j] == 1 ? u32x4{lp[i].x, lp[i].y, 0u, 0u} : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int j = 0; j < kBcItems; ++j) {
                const uint2 ent[2] = {make_uint2(raw[j].x, raw[j].y), make_uint2(raw[j].z, raw[j].w)};
                uint32_t u[2], v[2], gf[2];
                bool ok[2], spill[2];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const bool in = (uint32_t)k < len2[j];
                    const bool hu = in && (ent[k].x >> 31), hv = in && (ent[k].y >> 31);
                    u[k] = in ? ent[k].x & 0x7FFFFFFFu : 0u;
                    v[k] = in ? ent[k].y & 0x7FFFFFFFu : 0u;
                    const uint32_t x = (FWD && !hu) ? u[k] : v[k];     // the endpoint this part answers
                    const uint32_t lx = x - base_v;
                    const bool gx = in && ((slice[(lx >> 5) & (kSliceWords - 1)] >> (lx & 31)) & 1u);
                    if (admit && gx && e0s[j] + k < sample) hot_admit(hot, x);
                    ok[k] = in && !gx;                               // survivor: x outside the giant
                    gf[k] = gR == kInvalid ? 0u : FWD ? ((uint32_t)hu | ((uint32_t)hv << 1)) : 1u;
                    spill[k] = false;
                    if (FWD && gx && !hu && !hv) {                   // u inside, v unknown: v's part
                        const uint32_t part = v[k] >> kSliceBits;
                        const uint32_t pos = atomicAdd(&lcur[part], 1u);
                        if (pos < r.cap) mine[(uint64_t)part * r.cap + pos] = make_uint2(u[k] | (1u << 31), v[k]);
                        else spill[k] = true;
                    }
                }
                if (FWD) {
#pragma unroll
                    for (int k = 0; k < 2; ++k) {    // overfull list: v from global gbits
                        if (spill[k]) {
                            ok[k] = !gbit(f.gbits, v[k]);
                            gf[k] = gR == kInvalid ? 0u : 1u;
                        }
                    }
                }
                ring_push<MARK, STATS, 2>(f, ring, cnt, u, v, ok, gf, gR, st);
            }
        }
    }
    ring_flush<MARK, STATS>(f, ring, cnt, 0, st, gR);
    if (FWD) {
        __syncthreads();
        for (uint32_t p = threadIdx.x; p < r.parts; p += blockDim.x)
            r.cnt[(uint64_t)gridDim.x * r.parts + (uint64_t)blockIdx.x * r.parts + p] = (uint32_t)min((uint64_t)lcur[p], r.cap);
    }
    if (STATS) {
        atomicAdd(&f.stats[3], (unsigned long long)st.hooks);
        atomicAdd(&f.stats[5], (unsigned long long)st.inits);
    }
}

}  // namespace gsgpu
