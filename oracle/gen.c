/*
 * gen.c — TEST INFRASTRUCTURE ONLY: host restatement of the counter-based synthetic stream
 * generators that libgsgpu.so runs on the device (gelly-streaming_amd/csrc/gen.hip). The tests
 * check the device output against this file bit for bit; the reference has no generator
 * (its sample stream is ConnectedComponentsExample.java:121-127), so the definition is ours:
 *
 *   s0        = splitmix64(seed)
 *   base(i)   = splitmix64(s0 + i * 0x9E3779B97F4A7C15)
 *   r_k(i)    = splitmix64(base(i) + k)
 *   RMAT      : level l in [0, scale) takes the 32-bit draw x = (l even ? lo32 : hi32)(r_{l/2});
 *               x < c1 -> quadrant a, < c2 -> b (dst bit), < c3 -> c (src bit), else d (both);
 *               bit = 1 << (scale-1-l); c1 = ta, c2 = ta+tb, c3 = ta+tb+tc (64-bit sums).
 *               Then both ids go through the seeded bijection scramble() of [0, 2^scale).
 *   ER        : src = mulhi64(r_0, nv), dst = mulhi64(r_1, nv).
 * Self-loops and duplicate edges are kept.
 */
#include "oracle.h"

static inline uint64_t mulhi64(uint64_t a, uint64_t b) {
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
}

static inline uint64_t scramble(uint64_t x, int scale, uint64_t k) {
    const uint64_t mask = (scale >= 64) ? ~0ULL : ((1ULL << scale) - 1);
    x = (x * 0x9E3779B97F4A7C15ULL + k) & mask;
    x ^= x >> ((scale + 1) / 2);
    x = (x * 0xBF58476D1CE4E5B9ULL) & mask;
    x ^= x >> ((scale + 2) / 3);
    return x;
}

void gso_gen_rmat(int64_t* src, int64_t* dst, uint64_t first, uint64_t n, int scale,
                  uint64_t seed, uint32_t ta, uint32_t tb, uint32_t tc, int scramble_ids) {
    const uint64_t s0 = gso_splitmix64(seed);
    const uint64_t k = gso_splitmix64(seed ^ 0xA0761D6478BD642FULL);
    const uint64_t c1 = ta, c2 = c1 + tb, c3 = c2 + tc;
    for (uint64_t j = 0; j < n; ++j) {
        const uint64_t i = first + j;
        const uint64_t base = gso_splitmix64(s0 + i * 0x9E3779B97F4A7C15ULL);
        uint64_t u = 0, v = 0, r = 0;
        for (int l = 0; l < scale; ++l) {
            if ((l & 1) == 0) r = gso_splitmix64(base + (uint64_t)(l >> 1));
            const uint64_t x = (l & 1) ? (r >> 32) : (r & 0xFFFFFFFFULL);
            const uint64_t bit = 1ULL << (scale - 1 - l);
            if (x < c1) {
            } else if (x < c2) {
                v |= bit;
            } else if (x < c3) {
                u |= bit;
            } else {
                u |= bit; v |= bit;
            }
        }
        if (scramble_ids) { u = scramble(u, scale, k); v = scramble(v, scale, k); }
        src[j] = (int64_t)u;
        dst[j] = (int64_t)v;
    }
}

void gso_gen_er(int64_t* src, int64_t* dst, uint64_t first, uint64_t n, uint64_t nv, uint64_t seed) {
    const uint64_t s0 = gso_splitmix64(seed);
    for (uint64_t j = 0; j < n; ++j) {
        const uint64_t i = first + j;
        const uint64_t base = gso_splitmix64(s0 + i * 0x9E3779B97F4A7C15ULL);
        src[j] = (int64_t)mulhi64(gso_splitmix64(base + 0), nv);
        dst[j] = (int64_t)mulhi64(gso_splitmix64(base + 1), nv);
    }
}
