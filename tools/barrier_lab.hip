// barrier_lab.hip — what a window boundary costs on gfx950: a kernel boundary (back-to-back
// dependent launches on one stream) against a grid barrier inside one co-resident (cooperative)
// launch. Measurement tool for DESIGN.md; not part of libgsgpu.
//   hipcc -O3 --offload-arch=gfx950 -o tools/barrier_lab tools/barrier_lab.hip
//   ./tools/barrier_lab            (prints one JSON line)
// Every spin loop is bounded in time (kSpinTicks of the 100 MHz s_memrealtime clock, 20 ms): a
// barrier that never completes sets an error word and falls through, so no wave can hang the GPU.
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr unsigned long long kSpinTicks = 2000000ull;      // 20 ms at 100 MHz

// one load + one store per thread: a launch that touches memory like a tiny fold window
__global__ void k_touch(unsigned* __restrict__ a, unsigned n, unsigned it) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = a[i] + it;
}

struct Bar {
    unsigned* count;   // arrivals of the current generation
    unsigned* gen;     // generation word (own 128-B line)
    unsigned* err;     // spin cap hit
};

// flat grid barrier: thread 0 of every workgroup releases its workgroup's stores (agent scope),
// arrives on one counter; the last arrival resets it and bumps the generation; the others poll it.
// g = the generation this workgroup waits to leave (read once at kernel start: no workgroup can
// bump it before every workgroup has arrived, so all start from the same value).
__device__ __forceinline__ void grid_barrier(const Bar& b, unsigned nblocks, unsigned& g) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned a = __hip_atomic_fetch_add(b.count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (a == nblocks - 1) {
            __hip_atomic_store(b.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(b.gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(b.gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (__hip_atomic_load(b.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;   // a peer timed out
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) { atomicOr(b.err, 1u); break; }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        g += 1;
    }
    __syncthreads();
}

// two-level grid barrier (round-5 verdict): workgroup b arrives on the counter of its XCD group
// (b % 8: the dispatcher places workgroups on the 8 XCDs round-robin), each on a 128-B line of its
// own; the last arrival of a group arrives on the top counter, whose last arrival bumps the
// generation. 8 + (blocks / 8) arrivals per counter instead of `blocks` on one. spin: poll without
// s_sleep.
struct Bar2 {
    unsigned* group;   // 8 counters, 32 words apart
    unsigned* top;     // own line
    unsigned* gen;     // own line
    unsigned* err;
};
template <bool kSpin>
__device__ __forceinline__ void grid_barrier2(const Bar2& b, unsigned nblocks, unsigned& g) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned x = blockIdx.x & 7u;
        const unsigned members = nblocks / 8 + ((nblocks & 7u) > x ? 1u : 0u);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        unsigned* gc = b.group + 32 * x;
        const unsigned a = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        bool released = false;
        if (a == members - 1) {
            __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned groups = nblocks < 8 ? nblocks : 8u;
            const unsigned t = __hip_atomic_fetch_add(b.top, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (t == groups - 1) {
                __hip_atomic_store(b.top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(b.gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                released = true;
            }
        }
        if (!released) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(b.gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (__hip_atomic_load(b.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;   // a peer timed out
                if (!kSpin) __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) { atomicOr(b.err, 1u); break; }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        g += 1;
    }
    __syncthreads();
}

// three-level cost split (round 5): the grid barrier above spends its time in the per-workgroup
// agent-scope fences (an L2 write-back on release, an invalidate on acquire, each serialised per
// XCD). Here only the LAST arrival of each XCD group fences at agent scope (after every workgroup
// of its group has arrived with a workgroup-scope release: its stores are in the XCD's L2), the
// top release bumps the generation, and each group's first leaver invalidates for its group while
// the others only wait for that on a group word. kFence = false: no agent-scope fence at all (the
// synchronisation alone; not a valid barrier for plain stores across XCDs, a lower bound).
struct Bar3 {
    unsigned* group;   // 8 arrival counters, 32 words apart
    unsigned* ggen;    // 8 per-group release words, 32 words apart
    unsigned* top;
    unsigned* gen;
    unsigned* err;
};
template <bool kFence>
__device__ __forceinline__ void grid_barrier3(const Bar3& b, unsigned nblocks, unsigned& g) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned x = blockIdx.x & 7u;
        const unsigned members = nblocks / 8 + ((nblocks & 7u) > x ? 1u : 0u);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        unsigned* gc = b.group + 32 * x;
        const unsigned a = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        if (a == members - 1) {                          // this XCD's last arrival: one write-back for all
            __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (kFence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            const unsigned groups = nblocks < 8 ? nblocks : 8u;
            const unsigned t = __hip_atomic_fetch_add(b.top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t == groups - 1) {
                __hip_atomic_store(b.top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(b.gen, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                while (__hip_atomic_load(b.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                    if (__hip_atomic_load(b.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) { atomicOr(b.err, 1u); break; }
                }
            }
            if (kFence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // one invalidate per XCD
            __hip_atomic_store(b.ggen + 32 * x, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            while (__hip_atomic_load(b.ggen + 32 * x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (__hip_atomic_load(b.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) { atomicOr(b.err, 1u); break; }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        g += 1;
    }
    __syncthreads();
}
template <bool kFence>
__global__ void k_barriers3(Bar3 b, unsigned iters, unsigned* __restrict__ a, unsigned n, int store) {
    unsigned g = 0;
    if (threadIdx.x == 0) g = __hip_atomic_load(b.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    for (unsigned it = 0; it < iters; ++it) {
        if (store && i < n) a[i] = a[i] + it;
        grid_barrier3<kFence>(b, gridDim.x, g);
    }
}

template <bool kSpin>
__global__ void k_barriers2(Bar2 b, unsigned iters, unsigned* __restrict__ a, unsigned n, int store) {
    unsigned g = 0;
    if (threadIdx.x == 0) g = __hip_atomic_load(b.gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    for (unsigned it = 0; it < iters; ++it) {
        if (store && i < n) a[i] = a[i] + it;
        grid_barrier2<kSpin>(b, gridDim.x, g);
    }
}

__global__ void k_barriers(Bar b, unsigned iters, unsigned* __restrict__ a, unsigned n, int store) {
    unsigned g = 0;
    if (threadIdx.x == 0) g = __hip_atomic_load(b.gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    for (unsigned it = 0; it < iters; ++it) {
        if (store && i < n) a[i] = a[i] + it;
        grid_barrier(b, gridDim.x, g);
    }
}

__global__ void k_cg_barriers(unsigned iters, unsigned* __restrict__ a, unsigned n, int store) {
    cooperative_groups::grid_group grid = cooperative_groups::this_grid();
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    for (unsigned it = 0; it < iters; ++it) {
        if (store && i < n) a[i] = a[i] + it;
        grid.sync();
    }
}

int main(int argc, char** argv) {
    const unsigned iters = argc > 1 ? (unsigned)atoi(argv[1]) : 2000;
    setvbuf(stdout, nullptr, _IONBF, 0);
    int dev = 0, cus = 0;
    CK(hipSetDevice(dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    unsigned* a = nullptr;
    const unsigned n = 1u << 20;
    CK(hipMalloc(&a, n * 4));
    CK(hipMemset(a, 0, n * 4));
    unsigned* ctl = nullptr;
    CK(hipMalloc(&ctl, 1024));
    CK(hipMemset(ctl, 0, 1024));
    Bar b{ctl, ctl + 32, ctl + 64};
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms = 0.f;
    printf("{\"cus\": %d, \"iters\": %u", cus, iters);
    unsigned* ctl2 = nullptr;
    CK(hipMalloc(&ctl2, 4096));
    CK(hipMemset(ctl2, 0, 4096));
    Bar2 b2{ctl2, ctl2 + 8 * 32, ctl2 + 9 * 32, ctl + 64};
    unsigned* ctl3 = nullptr;
    CK(hipMalloc(&ctl3, 8192));
    CK(hipMemset(ctl3, 0, 8192));
    Bar3 b3{ctl3, ctl3 + 8 * 32, ctl3 + 16 * 32, ctl3 + 17 * 32, ctl + 64};
    const unsigned blocks_list[] = {32u, 64u, (unsigned)cus, 2u * cus, 4u * cus};
    for (unsigned threads : {256u, 1024u}) {
        for (unsigned blocks : blocks_list) {
            if (threads == 1024 && blocks > (unsigned)cus) continue;
            // kernel boundaries: iters dependent launches of a one-load-one-store kernel
            hipLaunchKernelGGL(k_touch, dim3(blocks), dim3(threads), 0, s, a, n, 0u);
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(e0, s));
            for (unsigned it = 0; it < iters; ++it) hipLaunchKernelGGL(k_touch, dim3(blocks), dim3(threads), 0, s, a, n, it);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf(", \"launch_us_%ux%u\": %.3f", blocks, threads, ms * 1e3 / iters);
            // occupancy: the cooperative launch needs every workgroup resident
            int per_cu = 0;
            CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_barriers, threads, 0));
            if ((unsigned)per_cu * cus < blocks) { printf(", \"bar_%ux%u\": null", blocks, threads); continue; }
            for (int store = 0; store < 2; ++store) {
                void* args[] = {&b, (void*)&iters, &a, (void*)&n, &store};
                CK(hipLaunchCooperativeKernel((const void*)k_barriers, dim3(blocks), dim3(threads), args, 0, s));
                CK(hipStreamSynchronize(s));
                CK(hipEventRecord(e0, s));
                CK(hipLaunchCooperativeKernel((const void*)k_barriers, dim3(blocks), dim3(threads), args, 0, s));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                printf(", \"bar%s_us_%ux%u\": %.3f", store ? "_store" : "", blocks, threads, ms * 1e3 / iters);
                unsigned e = 0;
                CK(hipMemcpy(&e, ctl + 64, 4, hipMemcpyDeviceToHost));
                if (e) { printf(", \"spin_cap_hit\": 1}\n"); return 2; }
                void* cargs[] = {(void*)&iters, &a, (void*)&n, &store};
                CK(hipEventRecord(e0, s));
                CK(hipLaunchCooperativeKernel((const void*)k_cg_barriers, dim3(blocks), dim3(threads), cargs, 0, s));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                printf(", \"cg%s_us_%ux%u\": %.3f", store ? "_store" : "", blocks, threads, ms * 1e3 / iters);
                for (int spin = 0; spin < 2; ++spin) {            // the two-level barrier, s_sleep / spin
                    void* args2[] = {&b2, (void*)&iters, &a, (void*)&n, &store};
                    const void* k2 = spin ? (const void*)k_barriers2<true> : (const void*)k_barriers2<false>;
                    CK(hipLaunchCooperativeKernel(k2, dim3(blocks), dim3(threads), args2, 0, s));
                    CK(hipStreamSynchronize(s));
                    CK(hipEventRecord(e0, s));
                    CK(hipLaunchCooperativeKernel(k2, dim3(blocks), dim3(threads), args2, 0, s));
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    printf(", \"bar2%s%s_us_%ux%u\": %.3f", spin ? "_spin" : "", store ? "_store" : "", blocks, threads,
                           ms * 1e3 / iters);
                    CK(hipMemcpy(&e, ctl + 64, 4, hipMemcpyDeviceToHost));
                    if (e) { printf(", \"spin_cap_hit\": 1}\n"); return 2; }
                }
                for (int fence = 1; fence >= 0; --fence) {        // leaders-only fences / no fences
                    void* args3[] = {&b3, (void*)&iters, &a, (void*)&n, &store};
                    const void* k3 = fence ? (const void*)k_barriers3<true> : (const void*)k_barriers3<false>;
                    CK(hipLaunchCooperativeKernel(k3, dim3(blocks), dim3(threads), args3, 0, s));
                    CK(hipStreamSynchronize(s));
                    CK(hipEventRecord(e0, s));
                    CK(hipLaunchCooperativeKernel(k3, dim3(blocks), dim3(threads), args3, 0, s));
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    printf(", \"bar3%s%s_us_%ux%u\": %.3f", fence ? "_leaderfence" : "_nofence", store ? "_store" : "",
                           blocks, threads, ms * 1e3 / iters);
                    CK(hipMemcpy(&e, ctl + 64, 4, hipMemcpyDeviceToHost));
                    if (e) { printf(", \"spin_cap_hit\": 1}\n"); return 2; }
                }
            }
        }
    }
    unsigned err = 0;
    CK(hipMemcpy(&err, ctl + 64, 4, hipMemcpyDeviceToHost));
    printf(", \"spin_cap_hit\": %u}\n", err);
    return err ? 2 : 0;
}
