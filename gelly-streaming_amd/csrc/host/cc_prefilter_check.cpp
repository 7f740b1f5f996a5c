// cc_prefilter_check — the Merger-rank layout (GS_MERGE_PREFILTER) through the C++ mirror: P ranks
// of an in-process group on one GPU (one thread each), rank 0 taking `share0` of every window of
// `window` edges and the others splitting the rest, one foldWindows call per rank per window; rank
// 0 prints "w <emission checksum> <vertices> <components>" after every window (gs_cc_checksum).
// Edges: "src dst" lines on stdin (int32 ids below the capacity).
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <thread>
#include <vector>

#include "gsgpu.hpp"

using namespace gelly::streaming;

int main(int argc, char** argv) {
    const uint64_t window = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000;
    const int world = argc > 2 ? std::atoi(argv[2]) : 3;
    const double share0 = argc > 3 ? std::atof(argv[3]) : 0.2;
    const uint64_t cap = argc > 4 ? std::strtoull(argv[4], nullptr, 10) : (1u << 16);
    std::vector<int32_t> src, dst;
    long long a, b;
    while (std::cin >> a >> b) { src.push_back((int32_t)a); dst.push_back((int32_t)b); }
    const uint64_t n = src.size();
    // rank r's slice [lo, hi) of every window
    std::vector<std::vector<std::pair<uint64_t, uint64_t>>> sl((size_t)world);
    for (uint64_t lo = 0; lo < n; lo += window) {
        const uint64_t ln = std::min(window, n - lo);
        const uint64_t c0 = std::max<uint64_t>(1, (uint64_t)(ln * share0));
        uint64_t at = lo;
        for (int r = 0; r < world; ++r) {
            const uint64_t e = r == 0 ? lo + c0 : lo + c0 + ((ln - c0) * (uint64_t)r) / (uint64_t)(world - 1);
            sl[(size_t)r].push_back({at, e});
            at = e;
        }
    }
    std::vector<std::unique_ptr<Comm>> comms;
    try {
        comms = Comm::local(world, 0);
    } catch (const GsError& e) {
        std::cerr << e.what() << "\n";
        return 2;
    }
    std::vector<std::string> lines;
    std::vector<int> rc((size_t)world, 0);
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r) {
        th.emplace_back([&, r] {
            try {
                DisjointSet<int32_t> ds(cap);
                for (auto& s : sl[(size_t)r]) {
                    const uint64_t m = s.second - s.first;
                    ds.foldWindows(src.data() + s.first, dst.data() + s.first, m, m ? m : 1, comms[(size_t)r].get(),
                                   GS_MERGE_PREFILTER);
                    if (r == 0) {
                        uint64_t sum = 0, nv = 0, nc = 0;
                        check(gs_cc_checksum(ds.handle(), &sum, &nv, &nc), "gs_cc_checksum");
                        lines.push_back(std::to_string(sum) + " " + std::to_string(nv) + " " + std::to_string(nc));
                    }
                }
            } catch (const GsError& e) {
                std::cerr << "rank " << r << ": " << e.what() << "\n";
                rc[(size_t)r] = 2;
            }
        });
    }
    for (auto& t : th) t.join();
    for (int r = 0; r < world; ++r) if (rc[(size_t)r]) return rc[(size_t)r];
    for (size_t w = 0; w < lines.size(); ++w) std::printf("%zu %s\n", w, lines[w].c_str());
    return 0;
}
