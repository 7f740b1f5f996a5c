// Lab: rocPRIM radix sort of the warm-set count sample (uint32 keys, 27 significant bits) on
// gfx950, to price a sort-based warm build against the atomic counters. Not product code.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sort_lab.hip -o tools/sort_lab
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_fill(uint32_t* k, uint32_t n, uint32_t real, uint32_t bits, uint64_t seed) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (i >= real) { k[i] = 1u << bits; continue; }
        uint64_t z = seed + i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        // skewed: power-law-ish ids (min of two uniforms, squared)
        const uint32_t a = (uint32_t)z & ((1u << bits) - 1), b = (uint32_t)(z >> 32) & ((1u << bits) - 1);
        k[i] = (uint32_t)(((uint64_t)std::min(a, b) * std::min(a, b)) >> bits);
    }
}

int main() {
    const uint32_t bits = 26;
    for (uint32_t n : {1u << 22, 1u << 23, 1u << 24}) {
        uint32_t *in, *out;
        CK(hipMalloc(&in, (size_t)n * 4));
        CK(hipMalloc(&out, (size_t)n * 4));
        size_t tmp_bytes = 0;
        CK(rocprim::radix_sort_keys(nullptr, tmp_bytes, in, out, n, 0, bits + 1));
        void* tmp;
        CK(hipMalloc(&tmp, tmp_bytes));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (uint32_t real : {n / 2, n}) {
            float best = 1e9f;
            for (int rep = 0; rep < 6; ++rep) {
                hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, in, n, real, bits, 1234 + rep);
                CK(hipEventRecord(e0, 0));
                CK(rocprim::radix_sort_keys(tmp, tmp_bytes, in, out, n, 0, bits + 1));
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep) best = std::min(best, ms);
            }
            std::vector<uint32_t> h(n);
            CK(hipMemcpy(h.data(), out, (size_t)n * 4, hipMemcpyDeviceToHost));
            const bool sorted = std::is_sorted(h.begin(), h.end());
            printf("{\"keys\": %u, \"real\": %u, \"end_bit\": %u, \"tmp_bytes\": %zu, \"best_us\": %.1f, \"sorted\": %s}\n",
                   n, real, bits + 1, tmp_bytes, best * 1e3, sorted ? "true" : "false");
        }
        CK(hipFree(in));
        CK(hipFree(out));
        CK(hipFree(tmp));
    }
    return 0;
}
