// Microbenchmark: is the steady fold's filter (two random 4-B lookups per edge into the 8 MiB
// giant bitmap, RMAT-26 edges, 2^24 per pass) bound by memory-level parallelism or by a
// throughput limit? Measured (gpurun_out/lab/mlp.txt, first version): waves per CU 4..32 and
// 4..16 edges per lane change nothing (8 MiB: ~270 us, 125 G lookups/s; 4 MiB: ~168 us; 2 MiB:
// ~150 us): a throughput limit. This version: the cost when a fraction of the lookups is free.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "gsgpu.h"
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// the production hot-set probe (5 x 12-bit slots, cc_kernels.hpp hot_probe) on a 128 KiB LDS table
__device__ __forceinline__ bool probe5(const uint2* tab, uint32_t v) {
    const uint32_t h = (v * 0x9E3779B1u) & ((1u << 26) - 1);
    const uint2 w = tab[h >> 12];
    const uint32_t r = (h & 4095u) + 1;
    const uint64_t x = ((uint64_t)w.y << 32) | w.x;
    return ((x & 0xFFFu) == r) | (((x >> 12) & 0xFFFu) == r) | (((x >> 24) & 0xFFFu) == r) |
           (((x >> 36) & 0xFFFu) == r) | (((x >> 48) & 0xFFFu) == r);
}

template <int EPT, bool LDS>
__global__ __launch_bounds__(1024) void k(const uint32_t* a, const uint32_t* b, uint64_t n, const uint32_t* bits,
                                          uint32_t mask, uint32_t skip, uint32_t* out) {
    extern __shared__ uint2 tab[];
    if (LDS) {
        for (uint32_t i = threadIdx.x; i < (1u << 14); i += blockDim.x) tab[i] = make_uint2(i * 2654435761u, i * 40503u);
        __syncthreads();
    }
    uint32_t acc = 0;
    const uint64_t groups = n / EPT;
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < groups; g += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t u[EPT], v[EPT];
#pragma unroll
        for (int q = 0; q < EPT / 4; ++q) {
            const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a) + g * (EPT / 4) + q);
            const u32x4 y = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b) + g * (EPT / 4) + q);
            u[4 * q] = x.x; u[4 * q + 1] = x.y; u[4 * q + 2] = x.z; u[4 * q + 3] = x.w;
            v[4 * q] = y.x; v[4 * q + 1] = y.y; v[4 * q + 2] = y.z; v[4 * q + 3] = y.w;
        }
        uint32_t wu[EPT], wv[EPT];
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
            // skip: lookups of ids whose hash falls below `skip` (of 2^16) are answered for free
            // (what an LDS hot set with that hit rate and a zero-cost probe would do)
            const bool su = ((u[i] * 0x9E3779B1u) >> 16) < skip, sv = ((v[i] * 0x9E3779B1u) >> 16) < skip;
            if (LDS) acc += probe5(tab, u[i]) + probe5(tab, v[i]);   // pay for the probes
            wu[i] = su ? ~0u : bits[(u[i] >> 5) & mask];
            wv[i] = sv ? ~0u : bits[(v[i] >> 5) & mask];
        }
#pragma unroll
        for (int i = 0; i < EPT; ++i) acc += (wu[i] >> (u[i] & 31)) & (wv[i] >> (v[i] & 31)) & 1;
    }
    if (acc == 0xFFFFFFFF) out[0] = acc;
}

int main() {
    const uint64_t E = 1ull << 24; const int scale = 26;
    const uint32_t V = 1u << scale, words = V / 32;
    uint32_t *a, *b, *bits, *out, *junk;
    hipMalloc(&a, E * 4); hipMalloc(&b, E * 4); hipMalloc(&out, 4); hipMalloc(&junk, 512u << 20);
    hipMalloc(&bits, words * 4); hipMemset(bits, 0x5A, words * 4);
    gs_gen_rmat(a, b, 32, 5ull << 24, E, scale, 1, (uint32_t)(0.57 * 4294967296.0), (uint32_t)(0.19 * 4294967296.0),
                (uint32_t)(0.19 * 4294967296.0), 1, nullptr);
    int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int lds : {0, 1}) for (uint32_t skip_pct : {0u, 33u}) {
        const uint32_t mib = 8, mask = (mib << 20) / 4 - 1, skip = skip_pct * 65536 / 100;
        for (int ept : {4}) for (int bpc : {1}) {
            float best = 1e9;
            for (int r = 0; r < 4; ++r) {
                hipMemsetAsync(junk, r, 512u << 20);                     // edges cold
                hipMemcpyAsync(junk, bits, (mib << 20), hipMemcpyDeviceToDevice);   // bitmap warm
                hipEventRecord(e0);
                const dim3 grid(cus * bpc);
                if (lds) hipLaunchKernelGGL((k<4, true>), grid, dim3(1024), 128u << 10, 0, a, b, E, bits, mask, skip, out);
                else hipLaunchKernelGGL((k<4, false>), grid, dim3(1024), 0, 0, a, b, E, bits, mask, skip, out);
                hipEventRecord(e1); hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                if (r && ms < best) best = ms;
            }
            printf("bitmap %u MiB  skip %2u%%  LDS probes %d  (1024-thread blocks, 1 per CU): %6.1f us per 2^24 edges\n",
                   mib, skip_pct, lds, best * 1e3);
        }
    }
    return 0;
}
