// Request-rate roofline of gfx950 for the filter's access shape: independent random 4-B loads
// (one cache line each) over a table of T bytes, 8 loads in flight per lane, at 16 and 32 waves
// per CU, for T = 1 MiB (L2-resident), 8 MiB (the headline's gbits: half L2), 64 MiB (Infinity
// Cache) and 2 GiB (HBM). The random-load rate that stops rising with occupancy is the ceiling the
// steady k_fold_ring is measured against, next to the streaming read rate.
// Build: hipcc -O3 --offload-arch=gfx950 tools/request_lab.hip -o tools/request_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// n loads in total; each thread issues 8 independent loads per step
__global__ __launch_bounds__(256) void k_rand(const uint32_t* __restrict__ mem, uint64_t mask, uint64_t n,
                                              uint32_t seed, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 8;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; i < n; i += stride) {
        uint32_t x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint64_t h = ((uint64_t)mix((uint32_t)(i + k) ^ seed) << 16) ^ mix((uint32_t)(i + k) * 0x9E3779B1u + seed);
            x[k] = mem[(h & mask)];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += x[k];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// As k_rand over an 8 MiB table, but every workgroup only reads the 1 MiB slice numbered by its
// XCD (HW_REG_XCC_ID): each XCD's L2 then holds one slice instead of sharing the whole table —
// the access shape of an XCD-routed giant filter
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7u;
}
__global__ __launch_bounds__(256) void k_rand_xcd(const uint32_t* __restrict__ mem, uint64_t n, uint32_t seed,
                                                  uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    const uint32_t* slice = mem + (uint64_t)xcc_id() * (1u << 18);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 8;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; i < n; i += stride) {
        uint32_t x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = slice[mix((uint32_t)(i + k) * 0x9E3779B1u + seed) & ((1u << 18) - 1)];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += x[k];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_stream(const u32x4* __restrict__ mem, uint64_t n16, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 q = __builtin_nontemporal_load(mem + i);
        acc += q.x ^ q.y ^ q.z ^ q.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

static float time_ms(void (*f)(void*), void* arg) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(a);
        f(arg);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (rep && ms < best) best = ms;                  // rep 0 warms the caches
    }
    return best;
}

struct RandArg { const uint32_t* mem; uint64_t mask, n; unsigned blocks; uint32_t* out; };
static void run_rand(void* p) {
    RandArg* r = static_cast<RandArg*>(p);
    hipLaunchKernelGGL(k_rand, dim3(r->blocks), dim3(256), 0, 0, r->mem, r->mask, r->n, 0x1234u, r->out);
}
static void run_rand_xcd(void* p) {
    RandArg* r = static_cast<RandArg*>(p);
    hipLaunchKernelGGL(k_rand_xcd, dim3(r->blocks), dim3(256), 0, 0, r->mem, r->n, 0x1234u, r->out);
}
struct StreamArg { const u32x4* mem; uint64_t n16; uint32_t* out; };
static void run_stream(void* p) {
    StreamArg* s = static_cast<StreamArg*>(p);
    hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, s->mem, s->n16, s->out);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t big = 2ull << 30;
    uint32_t *mem, *out;
    if (hipMalloc(&mem, big) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(mem, 1, big);
    const uint64_t n = 1ull << 26;                       // loads per pass
    printf("{\"cus\": %d, \"loads\": %llu", cus, (unsigned long long)n);
    const size_t sizes[4] = {1u << 20, 8u << 20, 64u << 20, big};
    const char* names[4] = {"1MiB", "8MiB", "64MiB", "2GiB"};
    for (int s = 0; s < 4; ++s) {
        for (int wpc = 16; wpc <= 32; wpc *= 2) {          // waves per CU: 4 or 8 blocks of 4 waves
            RandArg r{mem, sizes[s] / 4 - 1, n, (unsigned)(cus * wpc / 4), out};
            const float ms = time_ms(run_rand, &r);
            printf(", \"rand4B_%s_%dw_Gps\": %.1f", names[s], wpc, n / (ms * 1e6));
        }
    }
    for (int wpc = 16; wpc <= 32; wpc *= 2) {
        RandArg r{mem, 0, n, (unsigned)(cus * wpc / 4), out};
        const float ms = time_ms(run_rand_xcd, &r);
        printf(", \"rand4B_8MiB_xcdslice_%dw_Gps\": %.1f", wpc, n / (ms * 1e6));
    }
    StreamArg st{reinterpret_cast<const u32x4*>(mem), big / 16, out};
    const float ms = time_ms(run_stream, &st);
    printf(", \"stream_read_TBps\": %.2f}\n", big / (ms * 1e9));
    return 0;
}
