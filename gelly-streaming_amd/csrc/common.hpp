// common.hpp — shared helpers for libgsgpu (error reporting, device guard, splitmix64).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "gsgpu.h"

namespace gsgpu {

constexpr uint32_t kInvalid = 0xFFFFFFFFu;   // parent[v] of a vertex not in the summary
constexpr int kMaxSlotCaps = 16;              // slots of a fold with per-slot capacities (SlotCaps)

std::string& last_error();
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define GS_HIP(expr)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return ::gsgpu::fail(GS_ERR_HIP, "%s failed: %s (%s:%d)", #expr,                 \
                                 hipGetErrorString(e_), __FILE__, __LINE__);                 \
    } while (0)

#define GS_TRY(expr)                                                                         \
    do {                                                                                     \
        int rc_ = (expr);                                                                    \
        if (rc_ != GS_OK) return rc_;                                                        \
    } while (0)

// Makes `dev` current for the scope of an API call and restores the caller's device after.
struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = (hipSetDevice(dev) == hipSuccess);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// true if p is device (or managed) memory the kernels may dereference directly
bool is_device_pointer(const void* p);

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ uint64_t pair_mix(uint64_t v, uint64_t label) {
    return splitmix64(v ^ splitmix64(label ^ 0xD1B54A32D192ED03ULL));
}

}  // namespace gsgpu
