// parse.hip — edge-file ingestion on the device.
//
// Reference: ConnectedComponentsExample.getGraphStream (example/ConnectedComponentsExample.java:
// 108-119) reads a text file line by line and for each line does
//     String[] fields = s.split("\\s");  src = Long.parseLong(fields[0]);  trg = Long.parseLong(fields[1]);
// so: fields are separated by exactly one whitespace character (two in a row make an empty field,
// which parseLong rejects), trailing whitespace is dropped by split(), fields past the second are
// ignored, a field is an optional '+'/'-' and decimal digits within the int64 range, and any other
// line fails the job. This file restates those rules for every line in parallel:
//   k_nl_count      per 4 KiB chunk: number of '\n' (16-B loads)
//   k_nl_scan_*     exclusive scan of the chunk counts (two levels) = the first line of each chunk
//   k_parse_chunk   per 4 KiB chunk again: each thread's 16 bytes, a workgroup scan of their '\n'
//                   counts, and every line that STARTS in those bytes parsed by that thread: its index
//                   is the chunk's first line + the '\n's before it, so no line-offset array is
//                   written or read (the round-3 version wrote and re-read 8 B per line: 0.54 ms of
//                   its 1.77 ms per 2^24 lines); a bad line records its index (atomicMin) and the
//                   host reports the first one.
// Scratch (chunk counts and offsets, the bad-line word, a device copy of host text) is kept per
// thread and device and grown, not allocated per call.
#include <algorithm>
#include <cerrno>
#include <cstring>
#include <mutex>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "cc_internal.hpp"

namespace gsgpu {

constexpr int kChunk = 4096;                 // bytes per workgroup (256 threads x 16 B)

// the '\n' bytes of a thread's 16 bytes at base (one 16-B load when the whole block is in the text)
__device__ __forceinline__ uint32_t nl_mask16(const char* __restrict__ t, uint64_t n, uint64_t base) {
    uint32_t m = 0;
    if (base + 16 <= n) {
        const uint4 q = *reinterpret_cast<const uint4*>(t + base);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k) m |= (((w[j] >> (8 * k)) & 0xFFu) == '\n' ? 1u : 0u) << (4 * j + k);
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) m |= (base + k < n && t[base + k] == '\n' ? 1u : 0u) << k;
    }
    return m;
}

__global__ __launch_bounds__(256) void k_nl_count(const char* __restrict__ t, uint64_t n, uint32_t* __restrict__ cnt) {
    const uint64_t base = (uint64_t)blockIdx.x * kChunk + threadIdx.x * 16;
    uint32_t c = (uint32_t)__popc(nl_mask16(t, n, base));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
    __shared__ uint32_t ws[4];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// exclusive scan of the chunk counts in two levels: k_nl_scan_local scans 1024 chunks per
// workgroup (one chunk per thread) into off[] and writes each group's total; k_nl_scan_top scans
// the group totals (one workgroup) into gpre[] and writes the line count off[nb]; k_parse_chunk
// adds its group's gpre. (One 1024-thread workgroup scanning every count cost 45 us per 2^24 lines.)
constexpr int kScanGroup = 1024;
__device__ __forceinline__ unsigned long long block_excl_scan(unsigned long long x, unsigned long long* wsum,
                                                              unsigned long long* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    unsigned long long wbase = 0, all = 0;
    const int nw = (int)(blockDim.x >> 6);
    for (int w = 0; w < nw; ++w) {
        if (w < wid) wbase += wsum[w];
        all += wsum[w];
    }
    *total = all;
    return wbase + incl - x;
}

__global__ __launch_bounds__(kScanGroup) void k_nl_scan_local(const uint32_t* __restrict__ cnt, uint64_t* __restrict__ off,
                                                               unsigned long long* __restrict__ gsum, uint32_t nb) {
    __shared__ unsigned long long wsum[kScanGroup / 64];
    const uint32_t c = blockIdx.x * kScanGroup + threadIdx.x;
    unsigned long long total = 0;
    const unsigned long long ex = block_excl_scan(c < nb ? cnt[c] : 0u, wsum, &total);
    if (c < nb) off[c] = ex;
    if (threadIdx.x == 0) gsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanGroup) void k_nl_scan_top(const unsigned long long* __restrict__ gsum,
                                                             unsigned long long* __restrict__ gpre, uint32_t ng,
                                                             uint64_t* __restrict__ off, uint32_t nb) {
    __shared__ unsigned long long wsum[kScanGroup / 64];
    unsigned long long run = 0;
    for (uint32_t b0 = 0; b0 < ng; b0 += kScanGroup) {          // uniform
        const uint32_t g = b0 + threadIdx.x;
        unsigned long long total = 0;
        const unsigned long long ex = block_excl_scan(g < ng ? gsum[g] : 0ull, wsum, &total);
        if (g < ng) gpre[g] = run + ex;
        run += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) off[nb] = run;
}

__device__ __forceinline__ bool is_ws(char ch) {          // Java \s: [ \t\n\x0B\f\r]
    return ch == ' ' || ch == '\t' || ch == '\n' || ch == '\x0B' || ch == '\f' || ch == '\r';
}

// Long.parseLong of t[a, b): optional sign, >= 1 digit, no overflow
__device__ bool parse_long(const char* __restrict__ t, uint64_t a, uint64_t b, int64_t* out) {
    if (a >= b) return false;
    bool neg = false;
    if (t[a] == '-' || t[a] == '+') { neg = t[a] == '-'; ++a; }
    if (a >= b) return false;
    uint64_t v = 0;
    const uint64_t lim = neg ? (uint64_t)INT64_MAX + 1 : (uint64_t)INT64_MAX;
    for (uint64_t i = a; i < b; ++i) {
        const char ch = t[i];
        if (ch < '0' || ch > '9') return false;
        const uint64_t d = (uint64_t)(ch - '0');
        if (v > (lim - d) / 10) return false;
        v = v * 10 + d;
    }
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return true;
}

// the line [a, e) (e = its '\n' or the end of the text) -> (x, y); false if the reference rejects it
__device__ __forceinline__ bool parse_line(const char* __restrict__ t, uint64_t a, uint64_t e, int64_t* x, int64_t* y) {
    uint64_t b = e;
    while (b > a && is_ws(t[b - 1])) --b;                       // split() drops trailing empty fields
    uint64_t s1 = a;
    while (s1 < b && !is_ws(t[s1])) ++s1;                       // field 0 = [a, s1)
    uint64_t e2 = s1 + 1;                                       // field 1 starts right after ONE separator
    while (e2 < b && !is_ws(t[e2])) ++e2;
    return s1 < b && parse_long(t, a, s1, x) && parse_long(t, s1 + 1, e2, y);
}

// line i (its text at a) -> src[pos], dst[pos]
template <typename IdT>
__device__ __forceinline__ void parse_store(const char* __restrict__ t, uint64_t n, uint64_t a, uint64_t i, uint64_t pos,
                                            IdT* __restrict__ src, IdT* __restrict__ dst,
                                            unsigned long long* __restrict__ bad_line) {
    uint64_t e = a;
    while (e < n && t[e] != '\n') ++e;
    int64_t x = 0, y = 0;
    const bool ok = parse_line(t, a, e, &x, &y) &&
                    (sizeof(IdT) == 8 || ((uint64_t)x <= 0xFFFFFFFEull && (uint64_t)y <= 0xFFFFFFFEull));
    if (!ok) { atomicMin(bad_line, (unsigned long long)i); return; }
    src[pos] = static_cast<IdT>(x);
    dst[pos] = static_cast<IdT>(y);
}

__device__ __forceinline__ uint4 load16(const char* __restrict__ t, uint64_t n, uint64_t base) {
    if (base + 16 <= n) return *reinterpret_cast<const uint4*>(t + base);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (base + k < n) w[k >> 2] |= (uint32_t)(uint8_t)t[base + k] << (8 * (k & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Field scanner of one line from a 48-byte window of the LDS copy (the line starts at window byte r,
// which is text byte base + r; bytes at or past text byte n end the line). Java's rules (file header):
// field 0 = optional sign + digits up to ONE whitespace, field 1 = optional sign + digits up to
// whitespace / end of line, anything after field 1 ignored; every other shape is rejected, as are
// values outside int64. Phase by phase (a loop per digit run, one LDS byte per step: a byte-wise
// state machine over all six states cost ~1,200 instructions per wave-line). Returns 1 = parsed,
// 0 = rejected, 2 = the line runs past the window (the caller parses it from memory).
// overflow without a division: v * 10 + d > limit (INT64_MAX, or 2^63 for a '-' field) exactly when
// v > limit / 10 (the same for both) or v == limit / 10 and d > limit % 10 (7, or 8)
constexpr uint64_t kLim10 = 922337203685477580ull;
__device__ __forceinline__ bool acc_digit(uint64_t& v, uint64_t d, bool neg) {
    if (v > kLim10 || (v == kLim10 && d > (neg ? 8u : 7u))) return false;
    v = v * 10 + d;
    return true;
}
constexpr uint32_t kPastWindow = 0x100u;
// the window byte q (an LDS byte read; a one-word cache, an LDS read per 4 bytes, measured slower:
// 0.47 vs 0.43 ms per 2^24 lines)
// (kIn: the whole window lies inside the text, so no byte needs the end-of-text test)
template <bool kIn>
struct WinReader {
    const uint8_t* w;
    uint64_t base, n;
    __device__ __forceinline__ uint32_t at(int q) const {
        if (q >= 48) return kPastWindow;
        if (kIn) return (uint32_t)w[q];
        return base + (uint64_t)q < n ? (uint32_t)w[q] : (uint32_t)'\n';
    }
};
// one field: optional sign and >= 1 digits from window byte *p; on return *p is the byte after the
// digits and *c that byte. 1 = ok, 0 = rejected, 2 = past the window. The first 9 digits accumulate
// in 32 bits and digits 10-18 in 64 bits without a test (< 10^18 cannot overflow); the limit test
// runs from the 19th digit on
template <bool kIn>
__device__ __forceinline__ int scan_field(WinReader<kIn>& rd, int* p, uint32_t* c, int64_t* out) {
    uint32_t ch = rd.at(*p);
    bool neg = false;
    if (ch == '+' || ch == '-') { neg = ch == '-'; ch = rd.at(++*p); }
    if (ch >= kPastWindow) return 2;
    if (ch - '0' > 9u) return 0;
    uint32_t v32 = 0;
    int nd = 0;
    while (ch - '0' <= 9u && nd < 9) {
        v32 = v32 * 10u + (ch - '0');
        ++nd;
        ch = rd.at(++*p);
    }
    uint64_t v = v32;
    while (ch - '0' <= 9u) {
        if (nd < 18) v = v * 10 + (ch - '0');
        else if (!acc_digit(v, ch - '0', neg)) return 0;
        ++nd;
        ch = rd.at(++*p);
    }
    if (ch >= kPastWindow) return 2;
    *c = ch;
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return 1;
}
template <bool kIn>
__device__ __forceinline__ int scan_window(const uint8_t* w, int r, uint64_t base, uint64_t n, int64_t* x, int64_t* y) {
    WinReader<kIn> rd{w, base, n};
    int p = r;
    uint32_t c = 0;
    int k = scan_field(rd, &p, &c, x);
    if (k != 1) return k;
    if (!(c == ' ' || c == '\t' || c == 0x0B || c == '\f' || c == '\r')) return 0;   // ONE separator, not '\n'
    ++p;
    k = scan_field(rd, &p, &c, y);
    if (k != 1) return k;
    return (c == ' ' || c == '\t' || c == '\n' || c == 0x0B || c == '\f' || c == '\r') ? 1 : 0;  // field 1 ends at whitespace
}

// One 4 KiB chunk per workgroup, 16 bytes per thread, staged in LDS with the 32 bytes after the
// chunk: a thread parses every line that STARTS in its 16 bytes (after each '\n' there, and line 0
// at byte 0) from a 48-byte window of that LDS copy (a line longer than the window is parsed from
// memory); line index = the chunk's first line (off, the scan of k_nl_count) + the '\n's before it.
// Outputs: line i at position (gbase + i) mod ring of src / dst (the streaming ingestion's edge ring;
// gs_parse_edges: gbase 0, ring ~0); lines i >= lcap are not written (the caller's capacity).
struct LineOut {
    uint64_t gbase = 0, ring = ~0ull, lcap = ~0ull;
    __device__ __forceinline__ uint64_t pos(uint64_t i) const {
        const uint64_t p = gbase + i;
        return p >= ring ? p - ring : p;
    }
};
template <typename IdT>
__global__ __launch_bounds__(256) void k_parse_chunk(const char* __restrict__ t, uint64_t n, const uint64_t* __restrict__ off,
                                                     const unsigned long long* __restrict__ gpre,
                                                     IdT* __restrict__ src, IdT* __restrict__ dst,
                                                     unsigned long long* __restrict__ bad_line, LineOut lo) {
    __shared__ uint4 s_text[kChunk / 16 + 2];
    const uint64_t cbase = (uint64_t)blockIdx.x * kChunk;
    const uint64_t base = cbase + threadIdx.x * 16;
    const uint4 q = load16(t, n, base);
    s_text[threadIdx.x] = q;
    if (threadIdx.x < 2) s_text[kChunk / 16 + threadIdx.x] = load16(t, n, cbase + kChunk + threadIdx.x * 16);
    uint32_t m = 0;
    {
        const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                m |= ((((qw[j] >> (8 * k)) & 0xFFu) == '\n' && base + 4 * j + k < n) ? 1u : 0u) << (4 * j + k);
    }
    const uint32_t c = (uint32_t)__popc(m);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    __shared__ uint32_t ws[4];
    if (lane == 63) ws[wid] = incl;
    __syncthreads();
    uint32_t wbase = 0;
    for (int w = 0; w < wid; ++w) wbase += ws[w];
    uint64_t i = off[blockIdx.x] + gpre[blockIdx.x / kScanGroup] + wbase + incl - c;   // '\n's before this thread's bytes
    const uint8_t* win = reinterpret_cast<const uint8_t*>(s_text) + threadIdx.x * 16;
    const bool in = base + 48 <= n;
    auto one = [&](int r, uint64_t li) {
        if (li >= lo.lcap) return;
        int64_t x = 0, y = 0;
        const int k = in ? scan_window<true>(win, r, base, n, &x, &y) : scan_window<false>(win, r, base, n, &x, &y);
        const uint64_t p = lo.pos(li);
        if (k == 2) { parse_store<IdT>(t, n, base + r, li, p, src, dst, bad_line); return; }
        const bool ok = k == 1 && (sizeof(IdT) == 8 || ((uint64_t)x <= 0xFFFFFFFEull && (uint64_t)y <= 0xFFFFFFFEull));
        if (!ok) { atomicMin(bad_line, (unsigned long long)li); return; }
        src[p] = static_cast<IdT>(x);
        dst[p] = static_cast<IdT>(y);
    };
    if (base == 0) one(0, 0);                                  // line 0
    while (m) {
        const int k = __ffs(m) - 1;
        m &= m - 1;
        ++i;                                                    // the line after this '\n'
        if (base + (uint64_t)k + 1 < n) one(k + 1, i);
    }
}

}  // namespace gsgpu

using namespace gsgpu;


namespace {

// Device scratch of one parse: chunk '\n' counts, their offsets, per-1024-chunk group sums and
// prefixes, the bad-line word, and a pinned mirror [bad line, '\n' count, last byte]. Every buffer
// records its own capacity and a failed allocation leaves it empty (capacity 0), so a later call
// allocates again instead of launching on a null pointer.
template <typename T>
int grow_elems(T** p, size_t* cap, size_t want, const char* what) {
    if (*p && *cap >= want) return GS_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(p), want * sizeof(T)) != hipSuccess) {
        (void)hipGetLastError();
        return fail(GS_ERR_NOMEM, "%s: %zu bytes of scratch", what, want * sizeof(T));
    }
    *cap = want;
    return GS_OK;
}

struct ParseScratch {
    uint32_t* cnt = nullptr;
    size_t cnt_cap = 0;
    uint64_t* off = nullptr;
    size_t off_cap = 0;
    unsigned long long* gsum = nullptr;
    size_t gsum_cap = 0;
    unsigned long long* gpre = nullptr;
    size_t gpre_cap = 0;
    unsigned long long* bad = nullptr;
    size_t bad_cap = 0;
    unsigned long long* hbuf = nullptr;   // pinned: [bad line, '\n' count, last byte of the text]

    int ensure(uint32_t nb, const char* what) {
        const uint32_t ng = (nb + kScanGroup - 1) / kScanGroup;
        GS_TRY(grow_elems(&cnt, &cnt_cap, (size_t)nb + 1, what));
        GS_TRY(grow_elems(&off, &off_cap, (size_t)nb + 2, what));
        GS_TRY(grow_elems(&gsum, &gsum_cap, (size_t)std::max<uint32_t>(ng, 1), what));
        GS_TRY(grow_elems(&gpre, &gpre_cap, (size_t)std::max<uint32_t>(ng, 1), what));
        GS_TRY(grow_elems(&bad, &bad_cap, 1, what));
        if (!hbuf) {
            if (hipHostMalloc(reinterpret_cast<void**>(&hbuf), 3 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess) {
                (void)hipGetLastError();
                hbuf = nullptr;
                return fail(GS_ERR_NOMEM, "%s: pinned scratch", what);
            }
        }
        return GS_OK;
    }
    void release() {
        if (cnt) (void)hipFree(cnt);
        if (off) (void)hipFree(off);
        if (gsum) (void)hipFree(gsum);
        if (gpre) (void)hipFree(gpre);
        if (bad) (void)hipFree(bad);
        if (hbuf) (void)hipHostFree(hbuf);
        *this = ParseScratch{};
    }
};

// The '\n' count of aligned device text (k_nl_count + the two-level scan), its total and the text's
// last byte copied to sc.hbuf[1], [2] behind it on stream s. ensure() must have run for the text.
int enqueue_count(ParseScratch& sc, const char* dtext, uint64_t n_bytes, hipStream_t s) {
    const uint32_t nb = (uint32_t)((n_bytes + kChunk - 1) / kChunk);
    const uint32_t ng = (nb + kScanGroup - 1) / kScanGroup;
    hipLaunchKernelGGL(k_nl_count, dim3(nb), dim3(256), 0, s, dtext, n_bytes, sc.cnt);
    hipLaunchKernelGGL(k_nl_scan_local, dim3(ng), dim3(kScanGroup), 0, s, sc.cnt, sc.off, sc.gsum, nb);
    hipLaunchKernelGGL(k_nl_scan_top, dim3(1), dim3(kScanGroup), 0, s, (const unsigned long long*)sc.gsum, sc.gpre, ng,
                       sc.off, nb);
    GS_HIP(hipGetLastError());
    sc.hbuf[2] = 0;
    GS_HIP(hipMemcpyAsync(&sc.hbuf[1], sc.off + nb, 8, hipMemcpyDeviceToHost, s));
    GS_HIP(hipMemcpyAsync(&sc.hbuf[2], dtext + n_bytes - 1, 1, hipMemcpyDeviceToHost, s));
    return GS_OK;
}

// k_parse_chunk over the counted text into src / dst (device, positions per lo), the first bad line
// copied to sc.hbuf[0] (~0: none) behind it on stream s.
int enqueue_parse(ParseScratch& sc, const char* dtext, uint64_t n_bytes, uint32_t id_bits, void* src, void* dst,
                  LineOut lo, hipStream_t s) {
    const uint32_t nb = (uint32_t)((n_bytes + kChunk - 1) / kChunk);
    GS_HIP(hipMemsetAsync(sc.bad, 0xFF, 8, s));
    if (id_bits == 32)
        hipLaunchKernelGGL(k_parse_chunk<uint32_t>, dim3(nb), dim3(256), 0, s, dtext, n_bytes, (const uint64_t*)sc.off,
                           (const unsigned long long*)sc.gpre, (uint32_t*)src, (uint32_t*)dst, sc.bad, lo);
    else
        hipLaunchKernelGGL(k_parse_chunk<int64_t>, dim3(nb), dim3(256), 0, s, dtext, n_bytes, (const uint64_t*)sc.off,
                           (const unsigned long long*)sc.gpre, (int64_t*)src, (int64_t*)dst, sc.bad, lo);
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(&sc.hbuf[0], sc.bad, 8, hipMemcpyDeviceToHost, s));
    return GS_OK;
}

// gs_parse_edges' scratch: one per device, shared by every thread under a mutex (a call holds it
// from its first launch to its last sync), freed with the library. A host (or misaligned) text's
// device copy larger than kKeepText is freed after the call.
constexpr int kMaxParseDevices = 64;
constexpr size_t kKeepText = 256ull << 20;
struct ParseDevice {
    std::mutex mu;
    ParseScratch sc;
    char* text = nullptr;
    size_t text_cap = 0;
    ~ParseDevice() {                       // (process exit: the runtime may already be gone; best effort)
        if (text) (void)hipFree(text);
        sc.release();
    }
};
ParseDevice g_parse[kMaxParseDevices];

int parse_edges_locked(ParseDevice& pd, const char* text, uint64_t n_bytes, uint32_t id_bits, void* src, void* dst,
                       uint64_t cap, uint64_t* n_edges, hipStream_t s) {
    ParseScratch& sc = pd.sc;
    const size_t esz = id_bits / 8;
    const uint32_t nb = (uint32_t)((n_bytes + kChunk - 1) / kChunk);
    GS_TRY(sc.ensure(nb, "gs_parse_edges"));
    // the kernels read the text in 16-B loads: host or misaligned device text goes through a copy
    const char* dtext = text;
    if (!is_device_pointer(text) || (reinterpret_cast<uintptr_t>(text) & 15)) {
        GS_TRY(grow_elems(&pd.text, &pd.text_cap, n_bytes, "gs_parse_edges"));
        GS_HIP(hipMemcpyAsync(pd.text, text, n_bytes, hipMemcpyDefault, s));
        dtext = pd.text;
    }
    GS_TRY(enqueue_count(sc, dtext, n_bytes, s));
    GS_HIP(hipStreamSynchronize(s));
    const uint64_t nl = sc.hbuf[1];
    const uint64_t lines = nl + ((char)sc.hbuf[2] != '\n');     // a last line without '\n' still counts
    if (lines > cap) {
        *n_edges = lines;
        return fail(GS_ERR_CAPACITY, "gs_parse_edges: %llu lines, capacity %llu", (unsigned long long)lines,
                    (unsigned long long)cap);
    }
    const bool dev_out = is_device_pointer(src) && is_device_pointer(dst);
    void* dsrc = src;
    void* ddst = dst;
    if (!dev_out) {                                          // host outputs: staged per call
        dsrc = ddst = nullptr;
        if (hipMalloc(&dsrc, (size_t)std::max<uint64_t>(lines, 1) * esz) != hipSuccess ||
            hipMalloc(&ddst, (size_t)std::max<uint64_t>(lines, 1) * esz) != hipSuccess) {
            (void)hipGetLastError();
            if (dsrc) (void)hipFree(dsrc);
            return fail(GS_ERR_NOMEM, "gs_parse_edges: output staging");
        }
    }
    LineOut lo;
    lo.lcap = lines;
    int rc = enqueue_parse(sc, dtext, n_bytes, id_bits, dsrc, ddst, lo, s);
    if (rc == GS_OK && !dev_out && lines &&
        (hipMemcpyAsync(src, dsrc, lines * esz, hipMemcpyDeviceToHost, s) != hipSuccess ||
         hipMemcpyAsync(dst, ddst, lines * esz, hipMemcpyDeviceToHost, s) != hipSuccess))
        rc = fail(GS_ERR_HIP, "gs_parse_edges: copy of the outputs failed");
    if (hipStreamSynchronize(s) != hipSuccess && rc == GS_OK) rc = fail(GS_ERR_HIP, "gs_parse_edges: stream sync failed");
    if (!dev_out) {
        (void)hipFree(dsrc);
        (void)hipFree(ddst);
    }
    if (rc != GS_OK) return rc;
    const unsigned long long first_bad = sc.hbuf[0];
    if (first_bad != ~0ull) {
        *n_edges = first_bad;
        return fail(GS_ERR_INVALID, "gs_parse_edges: line %llu is not \"<long><whitespace><long>\" "
                    "(Long.parseLong of split(\"\\\\s\") fields 0 and 1)", first_bad + 1);
    }
    *n_edges = lines;
    return GS_OK;
}

}  // namespace

extern "C" int gs_parse_edges(const char* text, uint64_t n_bytes, uint32_t id_bits, void* src, void* dst,
                              uint64_t cap, uint64_t* n_edges, int device, void* stream) {
    if (!n_edges) return fail(GS_ERR_INVALID, "gs_parse_edges: null n_edges");
    *n_edges = 0;
    if (id_bits != 32 && id_bits != 64) return fail(GS_ERR_INVALID, "gs_parse_edges: id_bits must be 32 or 64");
    if (n_bytes == 0) return GS_OK;
    if (!text) return fail(GS_ERR_INVALID, "gs_parse_edges: null text");
    if (device < 0 || device >= kMaxParseDevices) return fail(GS_ERR_INVALID, "gs_parse_edges: device %d", device);
    DeviceGuard g(device);
    if (!g.ok) return fail(GS_ERR_HIP, "gs_parse_edges: hipSetDevice(%d) failed", device);
    ParseDevice& pd = g_parse[device];
    std::lock_guard<std::mutex> lock(pd.mu);
    const int rc = parse_edges_locked(pd, text, n_bytes, id_bits, src, dst, cap, n_edges, static_cast<hipStream_t>(stream));
    if (pd.text && pd.text_cap > kKeepText) {
        (void)hipStreamSynchronize(static_cast<hipStream_t>(stream));
        (void)hipFree(pd.text);
        pd.text = nullptr;
        pd.text_cap = 0;
    }
    return rc;
}

// ---- streaming edge-file ingestion: gs_cc_fold_text / gs_cc_fold_file ----
// ConnectedComponentsExample reads its edge file with readTextFile and streams the parsed edges into
// the operator (example/ConnectedComponentsExample.java:108-119 -> :61). Here the text moves in
// chunks of at most chunk_bytes, each cut after its last '\n' (the partial line is carried to the
// next chunk), through two pinned staging buffers and two device text buffers, so that the host's
// read of chunk i+1 and its copy overlap the parse of chunk i and the folds of chunk i-1:
//   copy stream   H2D chunk i -> dtext[i & 1], k_nl_count + scans (its line count to the host)
//   parse stream  k_parse_chunk: line j of chunk i -> the edge ring at (G_i + j) mod R
//   h->stream     the chunk's edges folded straight from the ring in count windows of W edges, each
//                 window closed (gs_cc_fold / gs_cc_fold_windows / gs_cc_close_window): the ids never
//                 leave the device.
// The ring holds R = a multiple of W >= W + 2 x Lmax edges (Lmax: the most lines a chunk can hold,
// chunk_bytes / 4 + 1, a valid line being >= 4 bytes), so a window is contiguous in it, the open
// window's edges stay in place across chunks, and chunk i's lines overwrite only edges of windows
// that ended before chunk i-1 began (folded by chunk i-2's folds, which the parse of chunk i waits for).
namespace {

constexpr uint64_t kDefaultChunk = 64ull << 20;

struct Ingest {
    int device = 0;
    uint32_t esz = 0;
    uint64_t chunk = 0, lmax = 0, ring = 0;
    char* pin[2] = {nullptr, nullptr};    // pinned staging (file and pageable sources)
    char* dtext[2] = {nullptr, nullptr};  // device text of chunks i & 1
    void* rs = nullptr;                   // edge ring: src ids, dst ids (ring entries each)
    void* rd = nullptr;
    ParseScratch sc[2];
    hipStream_t cs = nullptr, ps = nullptr;
    hipEvent_t copied[2] = {}, counted[2] = {}, parsed[2] = {}, folded[2] = {}, start = nullptr;

    void release() {
        if (cs) (void)hipStreamSynchronize(cs);
        if (ps) (void)hipStreamSynchronize(ps);
        for (int k = 0; k < 2; ++k) {
            if (pin[k]) (void)hipHostFree(pin[k]);
            if (dtext[k]) (void)hipFree(dtext[k]);
            pin[k] = dtext[k] = nullptr;
            sc[k].release();
        }
        if (rs) (void)hipFree(rs);
        if (rd) (void)hipFree(rd);
        rs = rd = nullptr;
        chunk = ring = lmax = 0;
    }
    void destroy() {
        release();
        for (int k = 0; k < 2; ++k)
            for (hipEvent_t* e : {&copied[k], &counted[k], &parsed[k], &folded[k]})
                if (*e) (void)hipEventDestroy(*e);
        if (start) (void)hipEventDestroy(start);
        if (cs) (void)hipStreamDestroy(cs);
        if (ps) (void)hipStreamDestroy(ps);
    }
};

void ingest_free(void* p) {
    Ingest* g = static_cast<Ingest*>(p);
    DeviceGuard dg(g->device);
    g->destroy();
    delete g;
}

// the handle's ingestion state, sized for chunks of `chunk` bytes and windows of W edges
int ingest_get(gs_cc_t* h, const CcInfo& in, uint32_t id_bits, uint64_t chunk, uint64_t W, Ingest** out) {
    Ingest* g = static_cast<Ingest*>(cc_ingest_get(h));
    if (!g) {
        g = new Ingest();
        g->device = in.device;
        cc_ingest_set(h, g, ingest_free);
        GS_HIP(hipStreamCreateWithFlags(&g->cs, hipStreamNonBlocking));
        GS_HIP(hipStreamCreateWithFlags(&g->ps, hipStreamNonBlocking));
        for (int k = 0; k < 2; ++k)
            for (hipEvent_t* e : {&g->copied[k], &g->counted[k], &g->parsed[k], &g->folded[k]})
                GS_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
        GS_HIP(hipEventCreateWithFlags(&g->start, hipEventDisableTiming));
    }
    const uint32_t esz = id_bits / 8;
    const uint64_t lmax = chunk / 4 + 1;
    uint64_t ring = W + 2 * lmax;
    ring = (ring + W - 1) / W * W;
    if (g->chunk < chunk || g->ring < ring || g->esz != esz || g->ring % W) {
        g->release();
        g->esz = esz;
        for (int k = 0; k < 2; ++k) {
            if (hipHostMalloc(reinterpret_cast<void**>(&g->pin[k]), chunk, hipHostMallocDefault) != hipSuccess ||
                hipMalloc(&g->dtext[k], chunk) != hipSuccess) {
                (void)hipGetLastError();
                g->release();
                return fail(GS_ERR_NOMEM, "gs_cc_fold_text: staging buffers of %llu bytes", (unsigned long long)chunk);
            }
            GS_TRY(g->sc[k].ensure((uint32_t)((chunk + kChunk - 1) / kChunk), "gs_cc_fold_text"));
        }
        if (hipMalloc(&g->rs, ring * esz) != hipSuccess || hipMalloc(&g->rd, ring * esz) != hipSuccess) {
            (void)hipGetLastError();
            g->release();
            return fail(GS_ERR_NOMEM, "gs_cc_fold_text: edge ring of %llu edges", (unsigned long long)ring);
        }
        g->chunk = chunk;
        g->ring = ring;
        g->lmax = lmax;
    }
    *out = g;
    return GS_OK;
}

// Where a chunk's bytes come from. Memory sources hand out [pos, last '\n' of the next chunk_bytes];
// a file is read(2) into the pinned buffer behind the carried tail of the previous chunk.
struct TextSource {
    enum Kind { kPageable, kPinned, kDevice, kFile } kind = kPageable;
    const char* p = nullptr;          // memory sources
    uint64_t n = 0, pos = 0;
    int fd = -1;                      // file source
    bool eof = false;
    std::vector<char> carry;          // file: the partial last line of the previous chunk
    bool done() const { return kind == kFile ? (eof && carry.empty()) : pos >= n; }
};

struct Chunk {
    const char* src = nullptr;        // bytes to copy to the device (host, pinned or device memory)
    uint64_t len = 0;
    bool final = false;
};

// the next chunk of s into slot k of g (the slot's pinned buffer is free: its last copy completed)
int next_chunk(Ingest* g, TextSource& s, int k, Chunk* c) {
    const uint64_t cap = g->chunk;
    if (s.kind == TextSource::kFile) {
        char* b = g->pin[k];
        uint64_t have = s.carry.size();
        if (have) std::memcpy(b, s.carry.data(), have);
        s.carry.clear();
        while (!s.eof && have < cap) {
            const ssize_t r = ::read(s.fd, b + have, (size_t)(cap - have));
            if (r < 0) {
                if (errno == EINTR) continue;
                return fail(GS_ERR_INVALID, "gs_cc_fold_file: read failed: %s", std::strerror(errno));
            }
            if (r == 0) s.eof = true;
            have += (uint64_t)r;
        }
        c->src = b;
        c->final = s.eof;
        c->len = have;
        if (!s.eof) {
            const void* nl = memrchr(b, '\n', (size_t)have);
            if (!nl) return fail(GS_ERR_CAPACITY, "gs_cc_fold_file: a line longer than the %llu-byte chunk",
                                 (unsigned long long)cap);
            c->len = (uint64_t)(static_cast<const char*>(nl) - b) + 1;
            s.carry.assign(b + c->len, b + have);
        }
        return GS_OK;
    }
    const uint64_t rem = s.n - s.pos;
    uint64_t len = std::min(rem, cap);
    c->final = len == rem;
    if (!c->final) {
        if (s.kind == TextSource::kDevice)              // (device text is handed over in one chunk)
            return fail(GS_ERR_INVALID, "gs_cc_fold_text: device text is handed over in one chunk");
        const void* nl = memrchr(s.p + s.pos, '\n', (size_t)len);
        if (!nl) return fail(GS_ERR_CAPACITY, "gs_cc_fold_text: a line longer than the %llu-byte chunk",
                             (unsigned long long)cap);
        len = (uint64_t)(static_cast<const char*>(nl) - (s.p + s.pos)) + 1;
    }
    if (s.kind == TextSource::kPageable) {            // into the pinned buffer (host copy), then DMA
        std::memcpy(g->pin[k], s.p + s.pos, (size_t)len);
        c->src = g->pin[k];
    } else {
        c->src = s.p + s.pos;
    }
    c->len = len;
    s.pos += len;
    return GS_OK;
}

// Folds ring edges [G, G + L) (global edge numbers) into h in count windows of W edges on h's
// stream: the open window's piece, then whole windows (gs_cc_fold_windows: the run-ahead steady
// fold), then the start of the next window; a window closes when its last edge is folded.
struct WindowHook {
    gs_window_fn fn = nullptr;
    void* ctx = nullptr;
};
int fold_ring(gs_cc_t* h, Ingest* g, uint64_t G, uint64_t L, uint64_t W, uint64_t* windows, const WindowHook& hook) {
    const char* rs = static_cast<const char*>(g->rs);
    const char* rd = static_cast<const char*>(g->rd);
    const size_t esz = g->esz;
    while (L) {
        const uint64_t r = G % g->ring;                 // ring position (windows never wrap: R % W == 0)
        const uint64_t in_win = G % W;
        if (in_win == 0 && L >= W && !hook.fn) {
            const uint64_t k = std::min(L / W, (g->ring - r) / W);
            uint64_t nw = 0;
            GS_TRY(gs_cc_fold_windows(h, nullptr, GS_MERGE_ALLGATHER, rs + r * esz, rd + r * esz, k * W, W, &nw));
            *windows += nw;
            G += k * W;
            L -= k * W;
            continue;
        }
        const uint64_t m = std::min(L, W - in_win);
        GS_TRY(gs_cc_fold(h, rs + r * esz, rd + r * esz, m));
        G += m;
        L -= m;
        if (G % W == 0) {
            GS_TRY(gs_cc_close_window(h));
            if (hook.fn) hook.fn(hook.ctx, *windows);
            ++*windows;
        }
    }
    return GS_OK;
}

int fold_text_impl(gs_cc_t* h, TextSource& s, uint64_t W, uint64_t chunk, const WindowHook& hook, uint64_t* edges_out,
                   uint64_t* windows_out) {
    CcInfo in;
    GS_TRY(cc_info(h, &in));
    DeviceGuard dg(in.device);
    // the handle's id width: the ring holds ids of that width (gs_cc_fold reads them)
    const uint32_t id_bits = in.id_bits;
    if (s.kind == TextSource::kDevice) chunk = std::max<uint64_t>(s.n, 16);   // one chunk (see next_chunk)
    chunk = (chunk + 15) & ~(uint64_t)15;
    Ingest* g = nullptr;
    GS_TRY(ingest_get(h, in, id_bits, chunk, W, &g));
    hipStream_t hs = in.stream;
    // everything already on the handle's stream (earlier folds still reading the ring, the caller's
    // text if it is device memory) comes first
    GS_HIP(hipEventRecord(g->start, hs));
    GS_HIP(hipStreamWaitEvent(g->cs, g->start, 0));
    GS_HIP(hipStreamWaitEvent(g->ps, g->start, 0));
    for (int k = 0; k < 2; ++k) {
        GS_HIP(hipEventRecord(g->parsed[k], g->ps));
        GS_HIP(hipEventRecord(g->folded[k], hs));
        GS_HIP(hipEventRecord(g->copied[k], g->cs));
    }
    Chunk ch[2];
    // chunk i: host side into slot k (its pinned buffer free once copy i-2 is done), then its copy
    // (after parse i-2 read the slot's device text and scratch) and count on the copy stream
    auto stage = [&](uint64_t i) -> int {
        const int k = (int)(i & 1);
        if (s.kind == TextSource::kFile || s.kind == TextSource::kPageable) GS_HIP(hipEventSynchronize(g->copied[k]));
        GS_TRY(next_chunk(g, s, k, &ch[k]));
        GS_HIP(hipStreamWaitEvent(g->cs, g->parsed[k], 0));
        if (ch[k].len) {
            GS_HIP(hipMemcpyAsync(g->dtext[k], ch[k].src, ch[k].len,
                                  s.kind == TextSource::kDevice ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, g->cs));
            GS_HIP(hipEventRecord(g->copied[k], g->cs));
            GS_TRY(enqueue_count(g->sc[k], g->dtext[k], ch[k].len, g->cs));
        } else {
            GS_HIP(hipEventRecord(g->copied[k], g->cs));
        }
        GS_HIP(hipEventRecord(g->counted[k], g->cs));
        return GS_OK;
    };
    uint64_t G = 0, windows = 0, line0 = 0;
    int rc = GS_OK;
    int stage_rc = GS_OK;                               // the next chunk could not be staged (a line
    bool more = !s.done();                              // longer than a chunk, a read error): chunk i
    if (more) GS_TRY(stage(0));                         // is still parsed and folded, then the call fails
    for (uint64_t i = 0; more; ++i) {
        const int k = (int)(i & 1);
        const bool last = ch[k].final || s.done();
        if (!last) stage_rc = stage(i + 1);             // read + copy + count of the next chunk meanwhile
        more = !last && stage_rc == GS_OK;
        if (!ch[k].len) continue;
        GS_HIP(hipEventSynchronize(g->counted[k]));
        const uint64_t lines = g->sc[k].hbuf[1] + ((char)g->sc[k].hbuf[2] != '\n');
        // parse into the ring once the folds of chunk i-2 are done with the edges it overwrites
        GS_HIP(hipStreamWaitEvent(g->ps, g->counted[k], 0));
        GS_HIP(hipStreamWaitEvent(g->ps, g->folded[k], 0));
        LineOut lo;
        lo.gbase = G % g->ring;
        lo.ring = g->ring;
        lo.lcap = std::min(lines, g->lmax);
        GS_TRY(enqueue_parse(g->sc[k], g->dtext[k], ch[k].len, id_bits, g->rs, g->rd, lo, g->ps));
        GS_HIP(hipEventRecord(g->parsed[k], g->ps));
        GS_HIP(hipEventSynchronize(g->parsed[k]));      // its bad-line word (the folds of chunk i-1 still run)
        const unsigned long long bad = g->sc[k].hbuf[0];
        uint64_t ok_lines = std::min(lines, g->lmax);
        if (bad != ~0ull) {
            ok_lines = bad;
            rc = fail(GS_ERR_INVALID, "gs_cc_fold_text: line %llu is not \"<long><whitespace><long>\" (Long.parseLong of "
                      "split(\"\\\\s\") fields 0 and 1)", (unsigned long long)(line0 + bad + 1));
        } else if (lines > g->lmax) {                   // (cannot happen without a bad line: see Lmax)
            rc = fail(GS_ERR_INVALID, "gs_cc_fold_text: %llu lines in a %llu-byte chunk", (unsigned long long)lines,
                      (unsigned long long)ch[k].len);
        }
        GS_HIP(hipStreamWaitEvent(hs, g->parsed[k], 0));
        const int frc = fold_ring(h, g, G, ok_lines, W, &windows, hook);
        GS_HIP(hipEventRecord(g->folded[k], hs));
        G += ok_lines;
        line0 += lines;
        if (frc != GS_OK) { rc = frc; break; }
        if (rc != GS_OK) break;
    }
    if (rc == GS_OK && stage_rc != GS_OK) rc = stage_rc;   // every line before the failed chunk folded
    if (rc == GS_OK && G % W) {                         // the last, partial window
        GS_TRY(gs_cc_close_window(h));
        if (hook.fn) hook.fn(hook.ctx, windows);
        ++windows;
    }
    // the ring and staging stay in use by the enqueued folds: the next call waits for them (start)
    GS_HIP(hipStreamSynchronize(g->cs));
    GS_HIP(hipStreamSynchronize(g->ps));
    if (edges_out) *edges_out = G;
    if (windows_out) *windows_out = windows;
    return rc;
}

}  // namespace

extern "C" int gs_cc_fold_text(gs_cc_t* h, const char* text, uint64_t n_bytes, uint64_t window_edges, uint64_t chunk_bytes,
                               gs_window_fn on_window, void* ctx, uint64_t* edges_out, uint64_t* windows_out) {
    if (edges_out) *edges_out = 0;
    if (windows_out) *windows_out = 0;
    if (!h) return fail(GS_ERR_INVALID, "null handle");
    if (window_edges == 0) return fail(GS_ERR_INVALID, "gs_cc_fold_text: window_edges must be > 0");
    if (n_bytes == 0) return GS_OK;
    if (!text) return fail(GS_ERR_INVALID, "gs_cc_fold_text: null text");
    TextSource s;
    s.p = text;
    s.n = n_bytes;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, text) == hipSuccess) {
        if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged || a.isManaged) s.kind = TextSource::kDevice;
        else if (a.type == hipMemoryTypeHost) s.kind = TextSource::kPinned;
    } else {
        (void)hipGetLastError();                       // pageable host memory
    }
    return fold_text_impl(h, s, window_edges, chunk_bytes ? chunk_bytes : kDefaultChunk, WindowHook{on_window, ctx},
                          edges_out, windows_out);
}

extern "C" int gs_cc_fold_file(gs_cc_t* h, const char* path, uint64_t window_edges, uint64_t chunk_bytes,
                               gs_window_fn on_window, void* ctx, uint64_t* edges_out, uint64_t* windows_out) {
    if (edges_out) *edges_out = 0;
    if (windows_out) *windows_out = 0;
    if (!h) return fail(GS_ERR_INVALID, "null handle");
    if (!path) return fail(GS_ERR_INVALID, "gs_cc_fold_file: null path");
    if (window_edges == 0) return fail(GS_ERR_INVALID, "gs_cc_fold_file: window_edges must be > 0");
    TextSource s;
    s.kind = TextSource::kFile;
    s.fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (s.fd < 0) return fail(GS_ERR_INVALID, "gs_cc_fold_file: cannot open %s: %s", path, std::strerror(errno));
    const int rc = fold_text_impl(h, s, window_edges, chunk_bytes ? chunk_bytes : kDefaultChunk, WindowHook{on_window, ctx},
                                  edges_out, windows_out);
    ::close(s.fd);
    return rc;
}
