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
#include <vector>

#include "common.hpp"

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

template <typename IdT>
__device__ __forceinline__ void parse_store(const char* __restrict__ t, uint64_t n, uint64_t a, uint64_t i,
                                            IdT* __restrict__ src, IdT* __restrict__ dst,
                                            unsigned long long* __restrict__ bad_line) {
    uint64_t e = a;
    while (e < n && t[e] != '\n') ++e;
    int64_t x = 0, y = 0;
    const bool ok = parse_line(t, a, e, &x, &y) &&
                    (sizeof(IdT) == 8 || ((uint64_t)x <= 0xFFFFFFFEull && (uint64_t)y <= 0xFFFFFFFEull));
    if (!ok) { atomicMin(bad_line, (unsigned long long)i); return; }
    src[i] = static_cast<IdT>(x);
    dst[i] = static_cast<IdT>(y);
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
template <typename IdT>
__global__ __launch_bounds__(256) void k_parse_chunk(const char* __restrict__ t, uint64_t n, const uint64_t* __restrict__ off,
                                                     const unsigned long long* __restrict__ gpre,
                                                     IdT* __restrict__ src, IdT* __restrict__ dst,
                                                     unsigned long long* __restrict__ bad_line) {
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
        int64_t x = 0, y = 0;
        const int k = in ? scan_window<true>(win, r, base, n, &x, &y) : scan_window<false>(win, r, base, n, &x, &y);
        if (k == 2) { parse_store<IdT>(t, n, base + r, li, src, dst, bad_line); return; }
        const bool ok = k == 1 && (sizeof(IdT) == 8 || ((uint64_t)x <= 0xFFFFFFFEull && (uint64_t)y <= 0xFFFFFFFEull));
        if (!ok) { atomicMin(bad_line, (unsigned long long)li); return; }
        src[li] = static_cast<IdT>(x);
        dst[li] = static_cast<IdT>(y);
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
// per thread and device scratch, grown and kept (a parse call allocates nothing in steady use)
struct ParseScratch {
    char* text = nullptr;                // device copy of host (or misaligned) text
    size_t text_cap = 0;
    uint32_t* cnt = nullptr;
    uint64_t* off = nullptr;
    size_t chunks_cap = 0;
    unsigned long long* bad = nullptr;
    unsigned long long* hbad = nullptr;  // pinned: [bad line, '\n' count]
    unsigned long long* gsum = nullptr;  // per 1024-chunk group: '\n' total, then its prefix (gpre)
    unsigned long long* gpre = nullptr;
    size_t groups_cap = 0;
};
constexpr int kMaxParseDevices = 64;
thread_local ParseScratch t_scratch[kMaxParseDevices];

int grow(void** p, size_t* cap, size_t want) {
    if (*cap >= want) return GS_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, want) != hipSuccess) { (void)hipGetLastError(); return fail(GS_ERR_NOMEM, "gs_parse_edges: scratch of %zu bytes", want); }
    *cap = want;
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
    hipStream_t s = static_cast<hipStream_t>(stream);
    ParseScratch& sc = t_scratch[device];
    const size_t esz = id_bits / 8;
    const uint32_t nb = (uint32_t)((n_bytes + kChunk - 1) / kChunk);
    // the kernels read the text in 16-B loads: host or misaligned device text goes through the
    // scratch copy
    const char* dtext = text;
    if (!is_device_pointer(text) || (reinterpret_cast<uintptr_t>(text) & 15)) {
        size_t c = sc.text_cap;
        GS_TRY(grow(reinterpret_cast<void**>(&sc.text), &c, n_bytes));
        sc.text_cap = c;
        GS_HIP(hipMemcpyAsync(sc.text, text, n_bytes, hipMemcpyDefault, s));
        dtext = sc.text;
    }
    if (sc.chunks_cap < (size_t)nb + 1) {
        size_t c1 = sc.chunks_cap ? sc.chunks_cap * 4 : 0, c2 = sc.chunks_cap ? (sc.chunks_cap + 1) * 8 : 0;
        GS_TRY(grow(reinterpret_cast<void**>(&sc.cnt), &c1, ((size_t)nb + 1) * 4));
        GS_TRY(grow(reinterpret_cast<void**>(&sc.off), &c2, ((size_t)nb + 2) * 8));
        sc.chunks_cap = (size_t)nb + 1;
    }
    const uint32_t ng = (nb + kScanGroup - 1) / kScanGroup;
    if (sc.groups_cap < ng) {
        size_t c1 = sc.groups_cap * 8, c2 = sc.groups_cap * 8;
        GS_TRY(grow(reinterpret_cast<void**>(&sc.gsum), &c1, (size_t)ng * 8));
        GS_TRY(grow(reinterpret_cast<void**>(&sc.gpre), &c2, (size_t)ng * 8));
        sc.groups_cap = ng;
    }
    if (!sc.bad) {
        size_t c = 0;
        GS_TRY(grow(reinterpret_cast<void**>(&sc.bad), &c, 8));
        if (hipHostMalloc(&sc.hbad, 2 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            return fail(GS_ERR_NOMEM, "gs_parse_edges: pinned scratch");
        }
    }
    GS_HIP(hipMemsetAsync(sc.bad, 0xFF, 8, s));
    hipLaunchKernelGGL(k_nl_count, dim3(nb), dim3(256), 0, s, dtext, n_bytes, sc.cnt);
    hipLaunchKernelGGL(k_nl_scan_local, dim3(ng), dim3(kScanGroup), 0, s, sc.cnt, sc.off, sc.gsum, nb);
    hipLaunchKernelGGL(k_nl_scan_top, dim3(1), dim3(kScanGroup), 0, s, (const unsigned long long*)sc.gsum, sc.gpre, ng,
                       sc.off, nb);
    GS_HIP(hipGetLastError());
    char last = '\n';
    GS_HIP(hipMemcpyAsync(&sc.hbad[1], sc.off + nb, 8, hipMemcpyDeviceToHost, s));
    GS_HIP(hipMemcpyAsync(&last, dtext + n_bytes - 1, 1, hipMemcpyDeviceToHost, s));
    GS_HIP(hipStreamSynchronize(s));
    const uint64_t nl = sc.hbad[1];
    const uint64_t lines = nl + (last != '\n');             // a last line without '\n' still counts
    if (lines > cap) {
        *n_edges = lines;
        return fail(GS_ERR_CAPACITY, "gs_parse_edges: %llu lines, capacity %llu", (unsigned long long)lines,
                    (unsigned long long)cap);
    }
    const bool dev_out = is_device_pointer(src) && is_device_pointer(dst);
    void* dsrc = src;
    void* ddst = dst;
    if (!dev_out) {                                          // host outputs: staged per call
        if (hipMalloc(&dsrc, (size_t)std::max<uint64_t>(lines, 1) * esz) != hipSuccess ||
            hipMalloc(&ddst, (size_t)std::max<uint64_t>(lines, 1) * esz) != hipSuccess) {
            (void)hipGetLastError();
            if (dsrc != src) (void)hipFree(dsrc);
            return fail(GS_ERR_NOMEM, "gs_parse_edges: output staging");
        }
    }
    if (id_bits == 32)
        hipLaunchKernelGGL(k_parse_chunk<uint32_t>, dim3(nb), dim3(256), 0, s, dtext, n_bytes, sc.off,
                           (const unsigned long long*)sc.gpre, (uint32_t*)dsrc, (uint32_t*)ddst, sc.bad);
    else
        hipLaunchKernelGGL(k_parse_chunk<int64_t>, dim3(nb), dim3(256), 0, s, dtext, n_bytes, sc.off,
                           (const unsigned long long*)sc.gpre, (int64_t*)dsrc, (int64_t*)ddst, sc.bad);
    int rc = GS_OK;
    if (hipGetLastError() != hipSuccess) rc = fail(GS_ERR_HIP, "gs_parse_edges: k_parse_chunk launch failed");
    if (rc == GS_OK && hipMemcpyAsync(&sc.hbad[0], sc.bad, 8, hipMemcpyDeviceToHost, s) != hipSuccess)
        rc = fail(GS_ERR_HIP, "gs_parse_edges: copy of the bad-line word failed");
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
    const unsigned long long first_bad = sc.hbad[0];
    if (first_bad != ~0ull) {
        *n_edges = first_bad;
        return fail(GS_ERR_INVALID, "gs_parse_edges: line %llu is not \"<long><whitespace><long>\" "
                    "(Long.parseLong of split(\"\\\\s\") fields 0 and 1)", first_bad + 1);
    }
    *n_edges = lines;
    return GS_OK;
}
