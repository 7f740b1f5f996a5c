// Throughput of the memory operations the young-window fold is made of, on gfx950: random 4-B
// loads, device-scope atomics (no-return atomicOr, returning atomicCAS) and plain stores, at
// uniform random addresses and at RMAT-26 endpoint addresses (power-law: hub contention), over an
// 8 MiB bitmap and a 256 MiB parent array. 2^25 operations per pass (one per edge endpoint of a
// 2^24-edge window). Build: hipcc -O3 --offload-arch=gfx950 -I../include tools/atomic_lab.hip
// -Lgelly-streaming_amd/gsgpu/lib -lgsgpu -o tools/atomic_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "gsgpu.h"

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// MODE: 0 load, 1 atomicOr (no return), 2 atomicCAS (kInvalid -> v, returning), 3 plain store,
// 4 atomicOr to the word of the bit (bitmap addressing v >> 5)
template <int MODE, bool RMAT>
__global__ __launch_bounds__(256) void k(const uint32_t* __restrict__ ids, uint64_t n, uint32_t* __restrict__ mem,
                                         uint32_t mask, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = RMAT ? ids[i] : mix((uint32_t)i * 2654435761u + 12345u);
        const uint32_t a = (MODE == 4 ? (v >> 5) : v) & mask;
        if (MODE == 0) acc += mem[a];
        if (MODE == 1) __hip_atomic_fetch_or(&mem[a], 1u << (v & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (MODE == 4) __hip_atomic_fetch_or(&mem[a], 1u << (v & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (MODE == 2) acc += atomicCAS(&mem[a], 0xFFFFFFFFu, v);
        if (MODE == 3) mem[a] = v;
        if (MODE == 5) __hip_atomic_store(&mem[a], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int MODE, bool RMAT>
float run(const uint32_t* ids, uint64_t n, uint32_t* mem, uint32_t mask, uint32_t* out, size_t bytes) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        hipMemset(mem, 0xFF, bytes);
        hipEventRecord(a);
        hipLaunchKernelGGL((k<MODE, RMAT>), dim3(8192), dim3(256), 0, 0, ids, n, mem, mask, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best;
}

int main() {
    const uint64_t W = 1ull << 24, n = 2 * W;
    uint32_t *ids, *mem, *out;
    hipMalloc(&ids, n * 4);
    hipMalloc(&mem, 256u << 20);
    hipMalloc(&out, 64);
    // RMAT-26 endpoints of window 1 (src then dst)
    if (gs_gen_rmat(ids, ids + W, 32, 0, W, 26, 1, 2448131358u, 816043786u, 816043786u, 1, nullptr) != 0) {
        printf("gen failed: %s\n", gs_last_error());
        return 1;
    }
    hipDeviceSynchronize();
    const uint32_t m8 = (8u << 20) / 4 - 1, m256 = (256u << 20) / 4 - 1;
    const size_t b8 = 8u << 20, b256 = 256u << 20;
    printf("{\"ops\": %llu,\n", (unsigned long long)n);
    printf(" \"load_uniform_8MiB_us\": %.1f, \"load_uniform_256MiB_us\": %.1f,\n",
           1e3 * run<0, false>(ids, n, mem, m8, out, b8), 1e3 * run<0, false>(ids, n, mem, m256, out, b256));
    printf(" \"load_rmat_256MiB_us\": %.1f,\n", 1e3 * run<0, true>(ids, n, mem, m256, out, b256));
    printf(" \"atomic_or_uniform_8MiB_us\": %.1f, \"atomic_or_uniform_256MiB_us\": %.1f,\n",
           1e3 * run<1, false>(ids, n, mem, m8, out, b8), 1e3 * run<1, false>(ids, n, mem, m256, out, b256));
    printf(" \"atomic_or_bitmap_rmat_8MiB_us\": %.1f, \"atomic_or_bitmap_uniform_8MiB_us\": %.1f,\n",
           1e3 * run<4, true>(ids, n, mem, m8, out, b8), 1e3 * run<4, false>(ids, n, mem, m8, out, b8));
    printf(" \"cas_uniform_256MiB_us\": %.1f, \"cas_rmat_256MiB_us\": %.1f,\n",
           1e3 * run<2, false>(ids, n, mem, m256, out, b256), 1e3 * run<2, true>(ids, n, mem, m256, out, b256));
    printf(" \"store_uniform_256MiB_us\": %.1f, \"store_rmat_256MiB_us\": %.1f,\n",
           1e3 * run<3, false>(ids, n, mem, m256, out, b256), 1e3 * run<3, true>(ids, n, mem, m256, out, b256));
    // a relaxed agent-scope atomic STORE (non-returning, coherent): the claim of a never-touched vertex
    // when no union can race with it (round 5, k_filter CLAIM)
    printf(" \"atomic_store_uniform_256MiB_us\": %.1f, \"atomic_store_rmat_256MiB_us\": %.1f}\n",
           1e3 * run<5, false>(ids, n, mem, m256, out, b256), 1e3 * run<5, true>(ids, n, mem, m256, out, b256));
    return 0;
}
