// parse.hip — edge-file ingestion on the device.
//
// Reference: ConnectedComponentsExample.getGraphStream (example/ConnectedComponentsExample.java:
// 108-119) reads a text file line by line and for each line does
//     String[] fields = s.split("\\s");  src = Long.parseLong(fields[0]);  trg = Long.parseLong(fields[1]);
// so: fields are separated by exactly one whitespace character (two in a row make an empty field,
// which parseLong rejects), trailing whitespace is dropped by split(), fields past the second are
// ignored, a field is an optional '+'/'-' and decimal digits within the int64 range, and any other
// line fails the job. This file restates those rules for every line in parallel:
//   k_nl_count   per 4 KiB chunk: number of '\n'
//   k_nl_scan    exclusive scan of the chunk counts (one workgroup)
//   k_nl_place   line end offsets
//   k_parse      one thread per line: two fields -> src[i], dst[i]; a bad line records its index
//                (atomicMin) and the host reports the first one.
#include <algorithm>
#include <vector>

#include "common.hpp"

namespace gsgpu {

constexpr int kChunk = 4096;                 // bytes per workgroup (256 threads x 16 B)

__global__ __launch_bounds__(256) void k_nl_count(const char* __restrict__ t, uint64_t n, uint32_t* __restrict__ cnt) {
    const uint64_t base = (uint64_t)blockIdx.x * kChunk + threadIdx.x * 16;
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) c += (base + k < n && t[base + k] == '\n');
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
    __shared__ uint32_t ws[4];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(1024) void k_nl_scan(const uint32_t* __restrict__ cnt, uint64_t* __restrict__ off, uint32_t nb) {
    __shared__ unsigned long long part[1024];
    const uint32_t per = (nb + blockDim.x - 1) / blockDim.x;
    const uint32_t lo = threadIdx.x * per, hi = min(lo + per, nb);
    unsigned long long s = 0;
    for (uint32_t i = lo; i < hi; ++i) s += cnt[i];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long run = 0;
        for (uint32_t t = 0; t < blockDim.x; ++t) { const unsigned long long x = part[t]; part[t] = run; run += x; }
        off[nb] = run;
    }
    __syncthreads();
    unsigned long long run = part[threadIdx.x];
    for (uint32_t i = lo; i < hi; ++i) { off[i] = run; run += cnt[i]; }
}

// line ends: ends[k] = byte offset of the k-th '\n'
__global__ __launch_bounds__(256) void k_nl_place(const char* __restrict__ t, uint64_t n, const uint64_t* __restrict__ off,
                                                  uint64_t* __restrict__ ends) {
    const uint64_t base = (uint64_t)blockIdx.x * kChunk + threadIdx.x * 16;
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) c += (base + k < n && t[base + k] == '\n');
    // exclusive scan of c over the workgroup
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
    uint64_t pos = off[blockIdx.x] + wbase + incl - c;
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (base + k < n && t[base + k] == '\n') ends[pos++] = base + k;
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

template <typename IdT>
__global__ __launch_bounds__(256) void k_parse(const char* __restrict__ t, const uint64_t* __restrict__ ends, uint64_t lines,
                                               IdT* __restrict__ src, IdT* __restrict__ dst,
                                               unsigned long long* __restrict__ bad_line) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += stride) {
        const uint64_t a = i ? ends[i - 1] + 1 : 0;
        uint64_t b = ends[i];                                   // exclusive ('\n' or end of text)
        while (b > a && is_ws(t[b - 1])) --b;                   // split() drops trailing empty fields
        uint64_t s1 = a;
        while (s1 < b && !is_ws(t[s1])) ++s1;                   // field 0 = [a, s1)
        uint64_t e2 = s1 + 1;                                   // field 1 starts right after ONE separator
        while (e2 < b && !is_ws(t[e2])) ++e2;
        int64_t x = 0, y = 0;
        const bool ok = s1 < b && parse_long(t, a, s1, &x) && parse_long(t, s1 + 1, e2, &y) &&
                        (sizeof(IdT) == 8 || ((uint64_t)x <= 0xFFFFFFFEull && (uint64_t)y <= 0xFFFFFFFEull));
        if (!ok) { atomicMin(bad_line, (unsigned long long)i); continue; }
        src[i] = static_cast<IdT>(x);
        dst[i] = static_cast<IdT>(y);
    }
}

}  // namespace gsgpu

using namespace gsgpu;

extern "C" int gs_parse_edges(const char* text, uint64_t n_bytes, uint32_t id_bits, void* src, void* dst,
                              uint64_t cap, uint64_t* n_edges, int device, void* stream) {
    if (!n_edges) return fail(GS_ERR_INVALID, "gs_parse_edges: null n_edges");
    *n_edges = 0;
    if (id_bits != 32 && id_bits != 64) return fail(GS_ERR_INVALID, "gs_parse_edges: id_bits must be 32 or 64");
    if (n_bytes == 0) return GS_OK;
    if (!text) return fail(GS_ERR_INVALID, "gs_parse_edges: null text");
    DeviceGuard g(device);
    if (!g.ok) return fail(GS_ERR_HIP, "gs_parse_edges: hipSetDevice(%d) failed", device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t esz = id_bits / 8;
    const uint32_t nb = (uint32_t)((n_bytes + kChunk - 1) / kChunk);
    // scratch: text copy (if host), chunk counts, offsets, bad-line word, line ends (sized after the count)
    char* dtext = nullptr;
    uint32_t* cnt = nullptr;
    uint64_t* off = nullptr;
    unsigned long long* bad = nullptr;
    uint64_t* ends = nullptr;
    void* dsrc = nullptr;
    void* ddst = nullptr;
    int rc = GS_OK;
    auto cleanup = [&]() {
        if (dtext && dtext != text) (void)hipFree(dtext);
        if (cnt) (void)hipFree(cnt);
        if (off) (void)hipFree(off);
        if (bad) (void)hipFree(bad);
        if (ends) (void)hipFree(ends);
        if (dsrc && dsrc != src) (void)hipFree(dsrc);
        if (ddst && ddst != dst) (void)hipFree(ddst);
    };
#define GS_PARSE_HIP(expr)                                                                            \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) { rc = fail(GS_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); cleanup(); return rc; } \
    } while (0)
    if (is_device_pointer(text)) {
        dtext = const_cast<char*>(text);
    } else {
        GS_PARSE_HIP(hipMalloc(&dtext, n_bytes));
        GS_PARSE_HIP(hipMemcpyAsync(dtext, text, n_bytes, hipMemcpyHostToDevice, s));
    }
    GS_PARSE_HIP(hipMalloc(&cnt, (size_t)nb * 4));
    GS_PARSE_HIP(hipMalloc(&off, ((size_t)nb + 1) * 8));
    GS_PARSE_HIP(hipMalloc(&bad, 8));
    GS_PARSE_HIP(hipMemsetAsync(bad, 0xFF, 8, s));
    hipLaunchKernelGGL(k_nl_count, dim3(nb), dim3(256), 0, s, dtext, n_bytes, cnt);
    hipLaunchKernelGGL(k_nl_scan, dim3(1), dim3(1024), 0, s, cnt, off, nb);
    GS_PARSE_HIP(hipGetLastError());
    uint64_t nl = 0;
    GS_PARSE_HIP(hipMemcpyAsync(&nl, off + nb, 8, hipMemcpyDeviceToHost, s));
    char last = '\n';
    GS_PARSE_HIP(hipMemcpyAsync(&last, dtext + n_bytes - 1, 1, hipMemcpyDeviceToHost, s));
    GS_PARSE_HIP(hipStreamSynchronize(s));
    const uint64_t lines = nl + (last != '\n');             // a last line without '\n' still counts
    GS_PARSE_HIP(hipMalloc(&ends, (size_t)std::max<uint64_t>(lines, 1) * 8));
    hipLaunchKernelGGL(k_nl_place, dim3(nb), dim3(256), 0, s, dtext, n_bytes, off, ends);
    if (last != '\n') GS_PARSE_HIP(hipMemcpyAsync(ends + nl, &n_bytes, 8, hipMemcpyHostToDevice, s));
    const bool dev_out = is_device_pointer(src) && is_device_pointer(dst);
    if (lines > cap) {
        *n_edges = lines;
        cleanup();
        return fail(GS_ERR_CAPACITY, "gs_parse_edges: %llu lines, capacity %llu", (unsigned long long)lines,
                    (unsigned long long)cap);
    }
    if (dev_out) {
        dsrc = src;
        ddst = dst;
    } else {
        GS_PARSE_HIP(hipMalloc(&dsrc, (size_t)std::max<uint64_t>(lines, 1) * esz));
        GS_PARSE_HIP(hipMalloc(&ddst, (size_t)std::max<uint64_t>(lines, 1) * esz));
    }
    const unsigned grid = (unsigned)std::min<uint64_t>((lines + 255) / 256 + 1, 16384);
    if (id_bits == 32)
        hipLaunchKernelGGL(k_parse<uint32_t>, dim3(grid), dim3(256), 0, s, dtext, ends, lines, (uint32_t*)dsrc, (uint32_t*)ddst, bad);
    else
        hipLaunchKernelGGL(k_parse<int64_t>, dim3(grid), dim3(256), 0, s, dtext, ends, lines, (int64_t*)dsrc, (int64_t*)ddst, bad);
    GS_PARSE_HIP(hipGetLastError());
    unsigned long long first_bad = 0;
    GS_PARSE_HIP(hipMemcpyAsync(&first_bad, bad, 8, hipMemcpyDeviceToHost, s));
    if (!dev_out && lines) {
        GS_PARSE_HIP(hipMemcpyAsync(src, dsrc, lines * esz, hipMemcpyDeviceToHost, s));
        GS_PARSE_HIP(hipMemcpyAsync(dst, ddst, lines * esz, hipMemcpyDeviceToHost, s));
    }
    GS_PARSE_HIP(hipStreamSynchronize(s));
#undef GS_PARSE_HIP
    cleanup();
    if (first_bad != ~0ull) {
        *n_edges = first_bad;
        return fail(GS_ERR_INVALID, "gs_parse_edges: line %llu is not \"<long><whitespace><long>\" "
                    "(Long.parseLong of split(\"\\\\s\") fields 0 and 1)", first_bad + 1);
    }
    *n_edges = lines;
    return GS_OK;
}
