// gen.hip — counter-based synthetic edge streams generated directly in HBM (bench inputs).
// Definition (shared bit for bit with the host restatement oracle/gen.c, checked by the tests):
//   s0 = splitmix64(seed); base(i) = splitmix64(s0 + i*0x9E3779B97F4A7C15);
//   r_k(i) = splitmix64(base(i) + k)
//   RMAT: level l uses the 32-bit draw (l even ? lo32 : hi32)(r_{l/2}) against cumulative
//         thresholds c1 = ta, c2 = ta+tb, c3 = ta+tb+tc; then a seeded bijection of [0, 2^scale)
//   ER  : src = mulhi64(r_0, nv), dst = mulhi64(r_1, nv)
#include "common.hpp"

namespace gsgpu {

__device__ __forceinline__ uint64_t scramble(uint64_t x, int scale, uint64_t k) {
    const uint64_t mask = (scale >= 64) ? ~0ULL : ((1ULL << scale) - 1);
    x = (x * 0x9E3779B97F4A7C15ULL + k) & mask;
    x ^= x >> ((scale + 1) / 2);
    x = (x * 0xBF58476D1CE4E5B9ULL) & mask;
    x ^= x >> ((scale + 2) / 3);
    return x;
}

template <typename IdT>
__global__ __launch_bounds__(256) void k_gen_rmat(IdT* __restrict__ src, IdT* __restrict__ dst, uint64_t first,
                                                  uint64_t n, int scale, uint64_t s0, uint64_t k, uint64_t c1,
                                                  uint64_t c2, uint64_t c3, int scr) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        const uint64_t i = first + j;
        const uint64_t base = splitmix64(s0 + i * 0x9E3779B97F4A7C15ULL);
        uint64_t u = 0, v = 0, r = 0;
        for (int l = 0; l < scale; ++l) {
            if ((l & 1) == 0) r = splitmix64(base + (uint64_t)(l >> 1));
            const uint64_t x = (l & 1) ? (r >> 32) : (r & 0xFFFFFFFFULL);
            const uint64_t bit = 1ULL << (scale - 1 - l);
            const bool sb = x >= c2;                       // quadrants c, d set the src bit
            const bool db = (x >= c1 && x < c2) || x >= c3; // quadrants b, d set the dst bit
            u |= sb ? bit : 0;
            v |= db ? bit : 0;
        }
        if (scr) { u = scramble(u, scale, k); v = scramble(v, scale, k); }
        src[j] = static_cast<IdT>(u);
        dst[j] = static_cast<IdT>(v);
    }
}

template <typename IdT>
__global__ __launch_bounds__(256) void k_gen_er(IdT* __restrict__ src, IdT* __restrict__ dst, uint64_t first,
                                                uint64_t n, uint64_t nv, uint64_t s0) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        const uint64_t i = first + j;
        const uint64_t base = splitmix64(s0 + i * 0x9E3779B97F4A7C15ULL);
        src[j] = static_cast<IdT>(__umul64hi(splitmix64(base + 0), nv));
        dst[j] = static_cast<IdT>(__umul64hi(splitmix64(base + 1), nv));
    }
}

static unsigned gen_blocks(uint64_t n) {
    const uint64_t b = (n + 255) / 256;
    return (unsigned)(b < 16384 ? (b ? b : 1) : 16384);
}

}  // namespace gsgpu

using namespace gsgpu;

extern "C" int gs_gen_rmat(void* src, void* dst, uint32_t id_bits, uint64_t first, uint64_t n, int scale,
                           uint64_t seed, uint32_t ta, uint32_t tb, uint32_t tc, int scr, void* stream) {
    if (!src || !dst) return fail(GS_ERR_INVALID, "gs_gen_rmat: null output");
    if (id_bits != 32 && id_bits != 64) return fail(GS_ERR_INVALID, "gs_gen_rmat: id_bits must be 32 or 64");
    if (scale < 1 || scale > (id_bits == 32 ? 32 : 62)) return fail(GS_ERR_INVALID, "gs_gen_rmat: bad scale %d", scale);
    if (!is_device_pointer(src) || !is_device_pointer(dst))
        return fail(GS_ERR_INVALID, "gs_gen_rmat: outputs must be device memory");
    if (n == 0) return GS_OK;
    const uint64_t s0 = splitmix64(seed), k = splitmix64(seed ^ 0xA0761D6478BD642FULL);
    const uint64_t c1 = ta, c2 = c1 + tb, c3 = c2 + tc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (id_bits == 32)
        hipLaunchKernelGGL(k_gen_rmat<uint32_t>, dim3(gen_blocks(n)), dim3(256), 0, s, (uint32_t*)src, (uint32_t*)dst,
                           first, n, scale, s0, k, c1, c2, c3, scr);
    else
        hipLaunchKernelGGL(k_gen_rmat<int64_t>, dim3(gen_blocks(n)), dim3(256), 0, s, (int64_t*)src, (int64_t*)dst,
                           first, n, scale, s0, k, c1, c2, c3, scr);
    GS_HIP(hipGetLastError());
    return GS_OK;
}

extern "C" int gs_gen_er(void* src, void* dst, uint32_t id_bits, uint64_t first, uint64_t n, uint64_t nv,
                         uint64_t seed, void* stream) {
    if (!src || !dst) return fail(GS_ERR_INVALID, "gs_gen_er: null output");
    if (id_bits != 32 && id_bits != 64) return fail(GS_ERR_INVALID, "gs_gen_er: id_bits must be 32 or 64");
    if (nv == 0 || (id_bits == 32 && nv > 0xFFFFFFFFull)) return fail(GS_ERR_INVALID, "gs_gen_er: bad nv");
    if (!is_device_pointer(src) || !is_device_pointer(dst))
        return fail(GS_ERR_INVALID, "gs_gen_er: outputs must be device memory");
    if (n == 0) return GS_OK;
    const uint64_t s0 = splitmix64(seed);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (id_bits == 32)
        hipLaunchKernelGGL(k_gen_er<uint32_t>, dim3(gen_blocks(n)), dim3(256), 0, s, (uint32_t*)src, (uint32_t*)dst,
                           first, n, nv, s0);
    else
        hipLaunchKernelGGL(k_gen_er<int64_t>, dim3(gen_blocks(n)), dim3(256), 0, s, (int64_t*)src, (int64_t*)dst,
                           first, n, nv, s0);
    GS_HIP(hipGetLastError());
    return GS_OK;
}
