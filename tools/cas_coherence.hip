// Diagnostic: are device-scope atomicCAS / atomicMin coherent across the 8 XCDs on hipMalloc memory?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k_claim(unsigned* words, unsigned nwords, unsigned* wins, int rounds) {
    const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
    for (int r = 0; r < rounds; ++r) {
        unsigned w = (tid * 2654435761u + r * 40503u) % nwords;       // every word claimed by many threads on many XCDs
        unsigned old = atomicCAS(&words[w], 0xFFFFFFFFu, tid);
        if (old == 0xFFFFFFFFu) atomicAdd(wins, 1u);
    }
}
__global__ void k_incr(unsigned* ctr, unsigned n, int iters) {
    for (int i = 0; i < iters; ++i) {
        unsigned* p = &ctr[(blockIdx.x + i) % n];
        unsigned old = *p, assumed;
        do { assumed = old; old = atomicCAS(p, assumed, assumed + 1); } while (old != assumed);
    }
}
int main() {
    const unsigned nwords = 1 << 20; unsigned *words, *wins, *ctr;
    hipMalloc(&words, nwords * 4); hipMalloc(&wins, 4); hipMalloc(&ctr, 64 * 4);
    hipMemset(words, 0xFF, nwords * 4); hipMemset(wins, 0, 4); hipMemset(ctr, 0, 256);
    k_claim<<<4096, 256>>>(words, nwords, wins, 8);
    unsigned h = 0; hipMemcpy(&h, wins, 4, hipMemcpyDeviceToHost);
    std::vector<unsigned> hw(nwords); hipMemcpy(hw.data(), words, nwords * 4, hipMemcpyDeviceToHost);
    unsigned claimed = 0; for (auto x : hw) claimed += (x != 0xFFFFFFFFu);
    printf("CAS claim: wins=%u claimed_words=%u (must be equal)\n", h, claimed);
    const int blocks = 2048, iters = 64;
    k_incr<<<blocks, 1>>>(ctr, 64, iters);
    std::vector<unsigned> hc(64); hipMemcpy(hc.data(), ctr, 256, hipMemcpyDeviceToHost);
    unsigned long long tot = 0; for (auto x : hc) tot += x;
    printf("CAS increments: total=%llu expected=%d\n", tot, blocks * iters);
    return 0;
}
