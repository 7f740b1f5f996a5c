// cc_latency — BASELINE config 5's per-window emission latency at the C ABI, without Python: the
// cost a Java shim calling libgsgpu.so through FFM / JNI sees, beside bench.py's
// Python-driven `window_latency`.
//
// RMAT scale 24, edge factor 16, seed 3 (2^28 edges, ids scrambled), generated in HBM by gs_gen_rmat;
// 4,096 windows of 2^16 edges. Per window: ONE gs_cc_fold_windows call (fold + close = the Merger's
// emission, resident in HBM) on the handle's stream, then hipStreamSynchronize; the wall time of the
// two, host clock. After a warm-up pass over the stream, one timed pass from a reset. Prints one
// JSON line: p50 / p99 / max of the window latency, and the last window's emission checksum (the C
// oracle's fixture tests/golden/c5_rmat24.json holds it: window 4,096).
//
// usage: cc_latency [windows]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gsgpu.h"

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        int rc_ = (x);                                                                             \
        if (rc_ != GS_OK) {                                                                        \
            std::fprintf(stderr, "%s failed: %d %s\n", #x, rc_, gs_last_error());                 \
            return 2;                                                                              \
        }                                                                                          \
    } while (0)

int main(int argc, char** argv) {
    const int scale = 24;
    const uint64_t V = 1ull << scale, W = 1ull << 16;
    const uint64_t nwin = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 4096;
    const uint64_t E = nwin * W;
    uint32_t *src = nullptr, *dst = nullptr;
    if (hipMalloc(&src, E * 4) != hipSuccess || hipMalloc(&dst, E * 4) != hipSuccess) {
        std::fprintf(stderr, "hipMalloc failed\n");
        return 2;
    }
    // Graph500 (a, b, c) = (0.57, 0.19, 0.19) as 32-bit thresholds (gsgpu/gen.py rmat_thresholds)
    const uint32_t ta = (uint32_t)(0.57 * 4294967296.0), tb = (uint32_t)(0.19 * 4294967296.0),
                   tc = (uint32_t)(0.19 * 4294967296.0);
    CHECK(gs_gen_rmat(src, dst, 32, 0, E, scale, 3, ta, tb, tc, 1, nullptr));
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    gs_cc_config cfg{sizeof(gs_cc_config), 32, V, 0, 0, 0};
    gs_cc_t* h = nullptr;
    CHECK(gs_cc_create(&h, &cfg));
    void* sv = nullptr;
    CHECK(gs_cc_get_stream(h, &sv));
    hipStream_t s = static_cast<hipStream_t>(sv);
    std::vector<double> lat;
    lat.reserve(nwin);
    uint64_t nw = 0;
    for (int pass = 0; pass < 2; ++pass) {
        CHECK(gs_cc_reset(h));
        if (hipStreamSynchronize(s) != hipSuccess) return 2;
        for (uint64_t w = 0; w < nwin; ++w) {
            const auto t0 = std::chrono::steady_clock::now();
            CHECK(gs_cc_fold_windows(h, nullptr, GS_MERGE_ALLGATHER, src + w * W, dst + w * W, W, W, &nw));
            if (hipStreamSynchronize(s) != hipSuccess) return 2;
            const auto t1 = std::chrono::steady_clock::now();
            if (pass == 1) lat.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
    }
    uint64_t sum = 0, nv = 0, nc = 0;
    CHECK(gs_cc_checksum(h, &sum, &nv, &nc));
    std::vector<double> sorted = lat;
    std::sort(sorted.begin(), sorted.end());
    const size_t n = sorted.size();
    std::printf("{\"workload\": \"c5_rmat24_ef16_window64K\", \"windows\": %llu, \"p50_us\": %.2f, \"p99_us\": %.2f, "
                "\"max_us\": %.2f, \"mean_us\": %.2f, \"final_checksum\": \"%llu\", \"final_vertices\": %llu, "
                "\"final_components\": %llu, \"caller\": \"C ABI, one gs_cc_fold_windows + hipStreamSynchronize per window\"}\n",
                (unsigned long long)n, sorted[n / 2], sorted[std::min(n - 1, (size_t)(n * 0.99))], sorted[n - 1],
                [&] { double t = 0; for (double x : lat) t += x; return t / n; }(), (unsigned long long)sum,
                (unsigned long long)nv, (unsigned long long)nc);
    gs_cc_destroy(h);
    (void)hipFree(src);
    (void)hipFree(dst);
    return 0;
}
