// Microbenchmark: stream E edges (uint32 SoA, 16 B/lane nontemporal) + 2 random bit lookups per
// edge into a bitmap of S bytes. Modes: 0 = ids mod table (global), 1 = per-XCD slice (block b
// uses slice b%8 of the table, S/8 bytes), 2 = no lookups (stream only).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "gsgpu.h"
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k(const uint32_t* a, const uint32_t* b, uint64_t n, const uint32_t* bits,
                                         uint32_t words, int mode, uint32_t* out) {
    uint32_t acc = 0;
    const uint32_t slice = words / 8, sbase = (blockIdx.x % 8) * slice;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n / 4; g += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a) + g);
        const u32x4 y = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b) + g);
        uint32_t u[4] = {x.x, x.y, x.z, x.w}, v[4] = {y.x, y.y, y.z, y.w};
        if (mode == 2) { acc += u[0] ^ v[3]; continue; }
        uint32_t wu[4], wv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t iu = u[i] >> 5, iv = v[i] >> 5;
            if (mode == 1) { iu = sbase + iu % slice; iv = sbase + iv % slice; } else { iu %= words; iv %= words; }
            wu[i] = bits[iu]; wv[i] = bits[iv];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) acc += (wu[i] >> (u[i] & 31)) & (wv[i] >> (v[i] & 31)) & 1;
    }
    if (acc == 0xFFFFFFFF) out[0] = acc;
}
int main() {
    const uint64_t E = 1ull << 24; const int scale = 26;
    uint32_t *a, *b, *bits, *out; hipMalloc(&a, E * 4); hipMalloc(&b, E * 4); hipMalloc(&out, 4);
    hipMalloc(&bits, 64u << 20); hipMemset(bits, 0x5A, 64u << 20);
    gs_gen_rmat(a, b, 32, 5ull << 24, E, scale, 1, (uint32_t)(0.57 * 4294967296.0), (uint32_t)(0.19 * 4294967296.0), (uint32_t)(0.19 * 4294967296.0), 1, nullptr);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const uint32_t sizes_kb[] = {256, 1024, 2048, 4096, 8192, 16384, 32768};
    for (int mode = 0; mode < 3; ++mode) for (uint32_t kb : sizes_kb) {
        if (mode == 2 && kb != 8192) continue;
        const uint32_t words = kb * 256;
        float best = 1e9;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(e0); k<<<16384, 256>>>(a, b, E, bits, words, mode, out); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        printf("mode %d table %6u KiB: %.1f us per 16M edges (%.1f G lookups/s)\n", mode, kb, best * 1e3, mode == 2 ? 0.0 : 2.0 * E / (best * 1e-3) / 1e9);
    }
    return 0;
}
