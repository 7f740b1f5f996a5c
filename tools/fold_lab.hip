// Microbenchmark for the steady-state fold filter (2 random bit lookups per edge into a V/8-byte
// bitmap, V = 2^26): where can the lookups be served from, and what does it cost to get them
// there? Real RMAT-26 edges (gs_gen_rmat), 2^24 per pass.
//   mode 0  every block: its own edges, lookups anywhere in the 8 MiB table (today's k_fold)
//   mode 1  XCD-replicated read: every XCD (block b -> XCD b % 8) scans ALL edges and handles
//           only the two (quarter u, quarter v) classes assigned to it: lookups touch 4 MiB
//           (nontemporal edge loads)
//   mode 2  as 1 with default-policy edge loads (re-reads may hit the Infinity Cache)
//   mode 3  as 2 without lookups (cost of the 8x replicated stream alone)
//   mode 4  stream only, each edge read once
//   mode 5  every block its own edges, lookups remapped into its XCD's two quarters (4 MiB):
//           the lookup pattern of a quarter-pair binned fold
//   mode 6  as 5 with one quarter (2 MiB)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "gsgpu.h"
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__constant__ uint8_t kQuarters[8][2] = {{0, 1}, {0, 1}, {0, 2}, {2, 3}, {2, 3}, {0, 3}, {1, 2}, {1, 3}};
__constant__ uint8_t kGroupOf[16] = {0, 0, 2, 5, 1, 1, 6, 7, 2, 6, 3, 3, 5, 7, 4, 4};

template <int MODE>
__global__ __launch_bounds__(256) void k(const uint32_t* a, const uint32_t* b, uint64_t n, const uint32_t* bits,
                                         uint32_t q1, uint32_t q2, uint32_t q3, uint32_t* out) {
    uint32_t acc = 0;
    const uint32_t xcd = blockIdx.x & 7;
    const uint64_t nb = (MODE >= 1 && MODE <= 3) ? gridDim.x / 8 : gridDim.x;
    const uint64_t bi = (MODE >= 1 && MODE <= 3) ? blockIdx.x / 8 : blockIdx.x;
    for (uint64_t g = bi * blockDim.x + threadIdx.x; g < n / 4; g += nb * blockDim.x) {
        u32x4 x, y;
        if (MODE == 1 || MODE == 0 || MODE == 4) {
            x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a) + g);
            y = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b) + g);
        } else {
            x = reinterpret_cast<const u32x4*>(a)[g];
            y = reinterpret_cast<const u32x4*>(b)[g];
        }
        uint32_t u[4] = {x.x, x.y, x.z, x.w}, v[4] = {y.x, y.y, y.z, y.w};
        if (MODE == 3 || MODE == 4) { acc += u[0] ^ v[3]; continue; }
        if (MODE == 5 || MODE == 6) {
            const uint32_t qs = q1;                       // ids per quarter
            const uint32_t qa = kQuarters[xcd][0], qb = kQuarters[xcd][MODE == 5 ? 1 : 0];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                u[i] = (u[i] % qs) + ((u[i] & 1) ? qa : qb) * qs;
                v[i] = (v[i] % qs) + ((v[i] & 1) ? qb : qa) * qs;
            }
        }
        bool mine[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (MODE == 0 || MODE >= 5) { mine[i] = true; continue; }
            const uint32_t cu = (u[i] >= q1) + (u[i] >= q2) + (u[i] >= q3);
            const uint32_t cv = (v[i] >= q1) + (v[i] >= q2) + (v[i] >= q3);
            mine[i] = kGroupOf[4 * cu + cv] == xcd;
        }
        uint32_t wu[4], wv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            wu[i] = mine[i] ? bits[u[i] >> 5] : 0u;
            wv[i] = mine[i] ? bits[v[i] >> 5] : 0u;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) acc += (wu[i] >> (u[i] & 31)) & (wv[i] >> (v[i] & 31)) & 1;
    }
    if (acc == 0xFFFFFFFF) out[0] = acc;
}

int main() {
    const uint64_t E = 1ull << 24; const int scale = 26;
    const uint32_t V = 1u << scale, words = V / 32;
    uint32_t *a, *b, *bits, *out;
    hipMalloc(&a, E * 4); hipMalloc(&b, E * 4); hipMalloc(&out, 4);
    hipMalloc(&bits, words * 4); hipMemset(bits, 0x5A, words * 4);
    gs_gen_rmat(a, b, 32, 5ull << 24, E, scale, 1, (uint32_t)(0.57 * 4294967296.0), (uint32_t)(0.19 * 4294967296.0),
                (uint32_t)(0.19 * 4294967296.0), 1, nullptr);
    // a 512 MiB buffer swept before every pass evicts the edges from L2 / Infinity Cache
    uint32_t* junk; hipMalloc(&junk, 512u << 20);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const uint32_t q1 = words / 4 * 32, q2 = words / 2 * 32, q3 = words / 4 * 3 * 32;
    const int grids[] = {2048, 4096, 8192, 16384};
    for (int mode : {0, 4, 5, 6}) for (int grid : grids) {
        float best = 1e9, cold = 0;
        for (int r = 0; r < 6; ++r) {
            // edges cold (HBM), bitmap warm: what a steady window sees
            hipMemsetAsync(junk, r, 512u << 20);
            hipMemcpyAsync(junk, bits, words * 4, hipMemcpyDeviceToDevice);
            hipEventRecord(e0);
            switch (mode) {
                case 0: k<0><<<grid, 256>>>(a, b, E, bits, q1, q2, q3, out); break;
                case 1: k<1><<<grid, 256>>>(a, b, E, bits, q1, q2, q3, out); break;
                case 2: k<2><<<grid, 256>>>(a, b, E, bits, q1, q2, q3, out); break;
                case 3: k<3><<<grid, 256>>>(a, b, E, bits, q1, q2, q3, out); break;
                case 4: k<4><<<grid, 256>>>(a, b, E, bits, q1, q2, q3, out); break;
                case 5: k<5><<<grid, 256>>>(a, b, E, bits, q1, q2, q3, out); break;
                default: k<6><<<grid, 256>>>(a, b, E, bits, q1, q2, q3, out); break;
            }
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            if (r == 0) cold = ms; else if (ms < best) best = ms;
        }
        printf("mode %d grid %5d: first %.1f us, best %.1f us per 16M edges\n", mode, grid, cold * 1e3, best * 1e3);
    }
    return 0;
}
