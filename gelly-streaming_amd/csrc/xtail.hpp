// xtail.hpp — the steady fold with an XCD-sliced giant-filter tail (UpdateCC past the young
// forest, DisjointSet.java:92-118 via ConnectedComponents.java:83-85).
//
// Why: k_fold_ring answers an endpoint from the LDS hot set, then the warm set (1 MiB, L2 hits),
// then gbits (8 MiB). gbits does not fit an XCD's 4 MiB L2 next to the warm set, so its ~10 M
// lookups per RMAT-26 2^24-edge window run at the 8 MiB-table random rate (~120 G/s, half of them
// Infinity-Cache fills) instead of the L2-hit rate (~260 G/s, tools/request_lab.hip). Here gbits is
// cut into 8 slices (slice(x) = x >> (B - 3): 1 MiB each at B = 26) and every workgroup reads only
// the slice numbered blockIdx % 8. Blocks b and b + 8 share an XCD (MI355X_MICROARCH.md §Workgroup
// dispatch), so each XCD's L2 holds one slice; which XCD gets which slice does not matter, and a
// different placement changes only speed, never results.
//
//   A  k_fold_xr: the ring fold's stream, LDS hot set and warm set; a warm-missing endpoint in the
//      workgroup's own slice is looked up there (L2 hit). An edge still undecided becomes a SINGLE
//      x (4 B: the other endpoint is a known giant member) listed for slice(x), or a DOUBLE (u, v)
//      (8 B: neither known) listed for slice(u). Lists are per (slice, producer workgroup) regions
//      at LDS cursors; a wave writes each slice's entries of a step as one contiguous run
//      (ballot multisplit: no LDS sort). Known survivors are unioned in the wave's LDS ring.
//   B  k_xr_tail<true>: workgroup b reads the singles and doubles of slice b % 8 from producers
//      j = b / 8 (mod grid / 8). A single outside the giant joins it; a double's u is looked up, and
//      its v too when v is in the same slice; a double whose u is in the giant and whose v is in
//      another slice lists v as a single for C.
//   C  k_xr_tail<false>: B's singles, as B's.
// Survivors of B and C are unioned in per-wave LDS rings (union_group_g: a giant member's parent
// read is replaced by the giant root gR). A list entry past its region's capacity is decided in
// place from global gbits (a skewed stream degrades to the plain filter, never to a wrong answer).
// Correctness rests on the same facts as k_fold_ring: gbits bit v = label(v) == gR at the last
// close, hot- and warm-set entries are members of that component, and components only merge until
// reset, so a "both in the giant" edge is already one component and x's union with any giant
// member is its union with gR.
#pragma once

#include "cc_kernels.hpp"

namespace gsgpu {

constexpr uint32_t kXSlices = 8;                 // gbits slices: one per XCD group (blockIdx % 8)
constexpr int kXThreads = 1024;
constexpr uint32_t kXNone = 0xFFu;               // no list entry
constexpr uint32_t kXChunk = 256;                // entries per wave chunk in the tails

struct XrArgs {
    uint32_t* qs;        // singles    [kXSlices][grid][cap]
    uint2* qd;           // doubles    [kXSlices][grid][cap]
    uint32_t* qc;        // B -> C singles [kXSlices][grid][cap]
    uint32_t* cnt;       // list lengths [3][kXSlices][grid] (qs, qd, qc)
    uint64_t cap;        // entries per region (a multiple of 4)
    uint32_t grid;       // workgroups of every xr kernel (a multiple of kXSlices)
    uint32_t shift;      // slice(x) = x >> shift
};

__device__ __forceinline__ bool gbit_of(uint32_t w, uint32_t x) { return (w >> (x & 31)) & 1u; }

// Survivor pairs (ok[k]) into the wave's LDS ring, flushed (unioned, one per lane) whenever it
// holds 64; a step with more survivors than half a ring is unioned in place (k_fold_ring's scheme).
template <bool MARK>
__device__ __forceinline__ void ring_push4(const FoldArgs& f, uint2* ring, uint32_t& cnt, const uint32_t (&u)[4],
                                           const uint32_t (&v)[4], const bool (&ok)[4], const uint32_t (&gf)[4],
                                           uint32_t gR, FoldStats& st) {
    const int lane = threadIdx.x & 63;
    const uint32_t c = (uint32_t)ok[0] + ok[1] + ok[2] + ok[3];
    uint32_t incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    const uint32_t wtot = __shfl(incl, 63, 64);
    if (wtot == 0) return;                           // uniform
    if (wtot > kRingCap / 2) {
        union_group_g<MARK, false, 4>(f, u, v, ok, gf, gR, st);
        return;
    }
    if (cnt + wtot > kRingCap) ring_flush<MARK, false>(f, ring, cnt, kRingCap - wtot, st, gR);
    uint32_t pos = cnt + incl - c;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (!ok[k]) continue;
        ring[pos] = make_uint2(u[k] | ((gf[k] & 1u) << 31), v[k] | ((gf[k] >> 1) << 31));
        ++pos;
    }
    cnt += wtot;
    if (cnt >= 64) ring_flush<MARK, false>(f, ring, cnt, cnt - 64, st, gR);
}

// Wave multisplit of one entry per lane by key (< NKEYS, or kXNone): each key's entries get
// consecutive positions at that key's LDS cursor (one LDS atomic per key present in the wave).
// Returns the lane's position (undefined for kXNone).
template <int KBITS>
__device__ __forceinline__ uint32_t wave_reserve(uint32_t key, uint32_t* __restrict__ lcur) {
    const bool live = key != kXNone;
    uint64_t m = __ballot(live);
#pragma unroll
    for (int bi = 0; bi < KBITS; ++bi) {
        const uint64_t bb = __ballot(live && ((key >> bi) & 1u));
        m &= ((key >> bi) & 1u) ? bb : ~bb;
    }
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane) - 1));
    uint32_t base = 0;
    if (live && rank == 0) base = atomicAdd(&lcur[key], (uint32_t)__popcll(m));
    const int leader = live ? (__ffsll((long long)m) - 1) : (int)lane;
    base = __shfl(base, leader, 64);
    return base + rank;
}

// A: stream + LDS hot set + warm set + own gbits slice; the rest listed per slice.
template <typename IdT, bool MARK>
__global__ __launch_bounds__(kXThreads) void k_fold_xr(const IdT* __restrict__ a, const IdT* __restrict__ b,
                                                       FoldArgs f, HotArgs hot, XrArgs x) {
    __shared__ __attribute__((aligned(16))) uint2 tab[kHotBuckets];
    __shared__ uint2 rings[kXThreads / 64][kRingCap];
    __shared__ uint32_t lcur[2 * kXSlices];
    const uint64_t n = f.n;
    lds_fill<2 * kHotBuckets>(reinterpret_cast<uint32_t*>(tab), reinterpret_cast<const uint32_t*>(hot.table), 2 * kHotBuckets);
    if (threadIdx.x < 2 * kXSlices) lcur[threadIdx.x] = 0u;
    const bool filt = *f.giant != kInvalid;          // uniform
    const uint32_t gR = filt ? f.giant[1] : kInvalid;
    const uint32_t budget = hot.budget ? *hot.budget : 1u;
    const uint64_t sample_edges = (hot.periodic || budget) ? hot.sample_edges : 0;
    const bool warm_ok = hot.warm && *hot.warm_valid != 0;                    // uniform
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0 && hot.budget && budget) *hot.budget = budget - 1;
    const int lane = threadIdx.x & 63;
    uint2* const ring = rings[threadIdx.x >> 6];
    uint32_t cnt = 0;
    FoldStats st;
    const uint32_t my = blockIdx.x & (kXSlices - 1);
    const uint32_t sh = x.shift;
    const bool five = hot.five != 0;
    const __amdgpu_buffer_rsrc_t wr = buffer_rsrc(hot.warm, warm_ok ? (4ull << hot.warm_bits) : 0ull);
    const __amdgpu_buffer_rsrc_t gr = buffer_rsrc(f.gbits, (((uint64_t)f.rc.cap + 31) >> 5) << 2);
    uint32_t* const qs = x.qs;
    uint2* const qd = x.qd;
    const uint64_t groups = n / 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); g0 < groups; g0 += stride) {
        const uint64_t g = g0 + lane;
        uint32_t u[4] = {0, 0, 0, 0}, v[4] = {0, 0, 0, 0};
        bool ok[4] = {false, false, false, false};
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
        // LDS hot set: every bucket read, then the compares
        bool ku[4], kv[4], gu[4], gv[4];
        {
            uint2 bu[4], bv[4];
            uint32_t ru[4], rv[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                bu[k] = tab[hot_bucket(u[k], hot.bits, ru[k])];
                bv[k] = tab[hot_bucket(v[k], hot.bits, rv[k])];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                gu[k] = hot_match(bu[k], ru[k], five);
                gv[k] = hot_match(bv[k], rv[k], five);
            }
        }
        bool hu[4], hv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) { hu[k] = gu[k]; hv[k] = gv[k]; }
        // warm set for the LDS misses (masked lanes: no request, 0 read), all in flight together
        {
            uint32_t xu[4], xv[4], ru[4], rv[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t iu = warm_word(u[k], hot.bits, hot.warm_bits, ru[k]);
                const uint32_t iv = warm_word(v[k], hot.bits, hot.warm_bits, rv[k]);
                xu[k] = __builtin_amdgcn_raw_buffer_load_b32(wr, (gu[k] || !warm_ok) ? kNoLoad : iu << 2, 0, 0);
                xv[k] = __builtin_amdgcn_raw_buffer_load_b32(wr, (gv[k] || !warm_ok) ? kNoLoad : iv << 2, 0, 0);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                gu[k] = gu[k] | warm_match(xu[k], ru[k]);
                gv[k] = gv[k] | warm_match(xv[k], rv[k]);
            }
        }
        // the workgroup's own gbits slice (L2-resident on this XCD) for the rest in it
        {
            uint32_t wu[4], wv[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool lu = !gu[k] && (u[k] >> sh) == my;
                const bool lv = !gv[k] && (v[k] >> sh) == my;
                wu[k] = __builtin_amdgcn_raw_buffer_load_b32(gr, lu ? (u[k] >> 5) << 2 : kNoLoad, 0, 0);
                wv[k] = __builtin_amdgcn_raw_buffer_load_b32(gr, lv ? (v[k] >> 5) << 2 : kNoLoad, 0, 0);
                ku[k] = gu[k] || lu;
                kv[k] = gv[k] || lv;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                gu[k] = gu[k] || (ku[k] && gbit_of(wu[k], u[k]));
                gv[k] = gv[k] || (kv[k] && gbit_of(wv[k], v[k]));
            }
        }
        if (filt && g * 4 < sample_edges) {                  // admission: endpoints found in the giant off LDS
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (ok[k] && !hu[k] && gu[k]) hot_admit(hot, u[k]);
                if (ok[k] && !hv[k] && gv[k]) hot_admit(hot, v[k]);
            }
        }
        // classify: drop, survivor (ring), single for slice(x), double for slice(u)
        bool surv[4];
        uint32_t gf[4];
        uint32_t ks[4], kd[4], xs[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            surv[k] = false;
            gf[k] = 0u;
            ks[k] = kXNone;
            kd[k] = kXNone;
            xs[k] = 0u;
            if (!ok[k]) continue;
            if (!filt) {                                             // no giant yet: every edge unions
                surv[k] = true;
                continue;
            }
            const bool both = ku[k] && kv[k];
            if (both) {
                surv[k] = !(gu[k] && gv[k]);
                gf[k] = (uint32_t)gu[k] | ((uint32_t)gv[k] << 1);
            } else if (ku[k] || kv[k]) {
                const bool gk = ku[k] ? gu[k] : gv[k];                   // the known side
                if (gk) {
                    xs[k] = ku[k] ? v[k] : u[k];
                    ks[k] = xs[k] >> sh;
                } else {
                    surv[k] = true;                                      // known outside the giant
                }
            } else {
                kd[k] = u[k] >> sh;
            }
        }
        // list writes: one multisplit per entry slot over 16 keys (8 slices x single/double)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t key = ks[k] != kXNone ? ks[k] : (kd[k] != kXNone ? kXSlices + kd[k] : kXNone);
            const uint32_t pos = wave_reserve<4>(key, lcur);
            if (key == kXNone) continue;
            const uint64_t region = (uint64_t)(key & (kXSlices - 1)) * x.grid + blockIdx.x;
            if (pos < x.cap) {
#ifndef GS_EXP_XRNOSTORE
                if (key < kXSlices) qs[region * x.cap + pos] = xs[k];
                else qd[region * x.cap + pos] = make_uint2(u[k], v[k]);
#else
                // timing lab (wrong results on purpose): the list entries are not stored
                asm volatile("" ::"v"(pos), "v"((uint32_t)region));
#endif
                continue;
            }
            // region full: decided here from global gbits (rare)
            if (key < kXSlices) {
                const bool gx = gbit_of(f.gbits[xs[k] >> 5], xs[k]);
                surv[k] = !gx;
                gf[k] = ku[k] ? 1u : 2u;                             // the known side is in the giant
            } else {
                const bool g1 = gbit_of(f.gbits[u[k] >> 5], u[k]), g2 = gbit_of(f.gbits[v[k] >> 5], v[k]);
                surv[k] = !(g1 && g2);
                gf[k] = (uint32_t)g1 | ((uint32_t)g2 << 1);
            }
        }
        ring_push4<MARK>(f, ring, cnt, u, v, surv, gf, gR, st);
    }
    ring_flush<MARK, false>(f, ring, cnt, 0, st, gR);
    __syncthreads();
    if (threadIdx.x < 2 * kXSlices) {
        const uint32_t kind = threadIdx.x / kXSlices, s = threadIdx.x % kXSlices;
        x.cnt[((uint64_t)kind * kXSlices + s) * x.grid + blockIdx.x] = (uint32_t)min((uint64_t)lcur[threadIdx.x], x.cap);
    }
}

// B (FIRST) / C: the lists of slice b % 8 from producers j = b / 8 (mod grid / 8), in chunks of
// kXChunk entries per wave (4 singles or 4 doubles per lane, 16-B loads); every gbits lookup of a
// chunk is issued before the first compare.
template <bool MARK, bool FIRST>
__global__ __launch_bounds__(kXThreads) void k_xr_tail(FoldArgs f, XrArgs x) {
    __shared__ uint2 rings[kXThreads / 64][kRingCap];
    __shared__ uint32_t lcur[kXSlices];
    __shared__ uint32_t pre[2][kXThreads / kXSlices + 1];
    const uint32_t my = blockIdx.x & (kXSlices - 1), sub = blockIdx.x / kXSlices, wpp = x.grid / kXSlices;
    const uint32_t nl = (x.grid - sub + wpp - 1) / wpp;          // producer regions j = sub + i * wpp
    if (threadIdx.x < kXSlices) lcur[threadIdx.x] = 0u;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t* const cs = x.cnt + ((FIRST ? 0ull : 2ull) * kXSlices + my) * x.grid;
    const uint32_t* const cd = x.cnt + (1ull * kXSlices + my) * x.grid;
    if (wave == 0) {                                 // chunk prefixes over the regions (nl <= 64 here)
        const uint32_t j = sub + lane * wpp;
        const uint32_t ns = lane < nl ? (cs[j] + kXChunk - 1) / kXChunk : 0u;
        const uint32_t nd = (FIRST && lane < nl) ? (cd[j] + kXChunk - 1) / kXChunk : 0u;
        uint32_t is = ns, id = nd;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t ys = __shfl_up(is, off, 64), yd = __shfl_up(id, off, 64);
            if ((int)lane >= off) { is += ys; id += yd; }
        }
        if (lane < nl) { pre[0][lane + 1] = is; pre[1][lane + 1] = id; }
        if (lane == 0) { pre[0][0] = 0u; pre[1][0] = 0u; }
    }
    __syncthreads();
    const uint32_t gR = f.giant[1];
    const uint32_t sh = x.shift;
    const __amdgpu_buffer_rsrc_t gr = buffer_rsrc(f.gbits, (((uint64_t)f.rc.cap + 31) >> 5) << 2);
    uint2* const ring = rings[wave];
    uint32_t cnt = 0;
    FoldStats st;
    const uint32_t* const qs = FIRST ? x.qs : x.qc;
    // singles: x in the giant -> dropped, else x joins the giant
    {
        const uint32_t nc = pre[0][nl];
        uint32_t li = 0;
        for (uint32_t c = wave; c < nc; c += kXThreads / 64) {
            while (pre[0][li + 1] <= c) ++li;                        // uniform
            const uint32_t j = sub + li * wpp;
            const uint32_t len = cs[j];
            const uint32_t e0 = (c - pre[0][li]) * kXChunk + 4 * lane;
            const uint32_t* lp = qs + ((uint64_t)my * x.grid + j) * x.cap;
            u32x4 q = u32x4{0u, 0u, 0u, 0u};
            if (e0 < len) q = *reinterpret_cast<const u32x4*>(lp + e0);
            const uint32_t xv[4] = {q.x, q.y, q.z, q.w};
            uint32_t w[4];
            bool live[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                live[k] = e0 + k < len;
                w[k] = __builtin_amdgcn_raw_buffer_load_b32(gr, live[k] ? (xv[k] >> 5) << 2 : kNoLoad, 0, 0);
            }
            uint32_t su[4], sv[4], gf[4];
            bool sk[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                sk[k] = live[k] && !gbit_of(w[k], xv[k]);
                su[k] = gR;
                sv[k] = xv[k];
                gf[k] = 1u;                                          // u side = the giant root
            }
            ring_push4<MARK>(f, ring, cnt, su, sv, sk, gf, gR, st);
        }
    }
    if (FIRST) {                                     // doubles: u here; v here too, or listed for C
        const uint32_t nc = pre[1][nl];
        uint32_t li = 0;
        for (uint32_t c = wave; c < nc; c += kXThreads / 64) {
            while (pre[1][li + 1] <= c) ++li;
            const uint32_t j = sub + li * wpp;
            const uint32_t len = cd[j];
            const uint32_t e0 = (c - pre[1][li]) * kXChunk + 2 * lane;   // entries e0, e0+1, e0+128, e0+129
            const uint2* lp = x.qd + ((uint64_t)my * x.grid + j) * x.cap;
            u32x4 q0 = u32x4{0u, 0u, 0u, 0u}, q1 = u32x4{0u, 0u, 0u, 0u};
            if (e0 < len) q0 = *reinterpret_cast<const u32x4*>(lp + e0);
            if (e0 + 128 < len) q1 = *reinterpret_cast<const u32x4*>(lp + e0 + 128);
            const uint32_t uu[4] = {q0.x, q0.z, q1.x, q1.z};
            const uint32_t vv[4] = {q0.y, q0.w, q1.y, q1.w};
            const uint32_t ei[4] = {e0, e0 + 1, e0 + 128, e0 + 129};
            bool live[4], lv[4];
            uint32_t wu[4], wv[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                live[k] = ei[k] < len;
                lv[k] = live[k] && (vv[k] >> sh) == my;
                wu[k] = __builtin_amdgcn_raw_buffer_load_b32(gr, live[k] ? (uu[k] >> 5) << 2 : kNoLoad, 0, 0);
                wv[k] = __builtin_amdgcn_raw_buffer_load_b32(gr, lv[k] ? (vv[k] >> 5) << 2 : kNoLoad, 0, 0);
            }
            bool sk[4];
            uint32_t gf[4], su[4], sv[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool g1 = live[k] && gbit_of(wu[k], uu[k]);
                const bool g2 = lv[k] && gbit_of(wv[k], vv[k]);
                const bool toc = g1 && live[k] && !lv[k];                 // v in another slice
                uint32_t key = toc ? (vv[k] >> sh) : kXNone;
                const uint32_t pos = wave_reserve<3>(key, lcur);
                bool spill = false;
                if (toc) {
                    if (pos < x.cap) x.qc[((uint64_t)key * x.grid + blockIdx.x) * x.cap + pos] = vv[k];
                    else spill = true;
                }
                // survivors: u outside the giant; or both here and not both in it; or a spilled v
                // decided from global gbits
                const bool gs = spill && gbit_of(f.gbits[vv[k] >> 5], vv[k]);
                sk[k] = live[k] && ((!g1) || (lv[k] && !g2) || (spill && !gs));
                su[k] = uu[k];
                sv[k] = vv[k];
                gf[k] = (uint32_t)g1 | ((uint32_t)(g2 || gs) << 1);
            }
            ring_push4<MARK>(f, ring, cnt, su, sv, sk, gf, gR, st);
        }
    }
    ring_flush<MARK, false>(f, ring, cnt, 0, st, gR);
    if (FIRST) {
        __syncthreads();
        if (threadIdx.x < kXSlices)
            x.cnt[(2ull * kXSlices + threadIdx.x) * x.grid + blockIdx.x] = (uint32_t)min((uint64_t)lcur[threadIdx.x], x.cap);
    }
}

}  // namespace gsgpu
