// cc_example — ConnectedComponentsExample on the MI355X path
// (reference: src/main/java/org/apache/flink/graph/streaming/example/ConnectedComponentsExample.java).
//
//   cc_example                                   built-in sample stream (k, k+2), k = 1..100,
//                                                event time k*100 ms, merge window 1000 ms (:121-139)
//   cc_example <edges> <merge ms> <print ms> [capacity]
//                                                whitespace-separated "src trg" lines (:108-119),
//                                                streamed from the file through the device
//                                                (gs_cc_fold_file: chunked pinned H2D, parsed and
//                                                folded on the device); no timestamps in the file,
//                                                so the merge window is cut by edge count (<merge ms>
//                                                edges per window) and the print window by window
//                                                count (<print ms> windows: the emission of every
//                                                <print ms>-th window is printed); any Long ids (a
//                                                sparse-id summary of at most [capacity] distinct ids;
//                                                default: file size / 2 — a valid line has at least 4
//                                                bytes for its 2 ids — capped at 2^28)
//
// Output: like the reference's FlattenSet -> keyBy(vertex) -> timeWindow(print) -> fold(identity)
// -> print (:61-67): at the end of every print window, one "(vertex,root)" line per vertex with
// its latest emitted root. Roots are the canonical minimum vertex id of each component.
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <fstream>
#include <iterator>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <sys/stat.h>

#include "gsgpu.hpp"

using namespace gelly::streaming;

int main(int argc, char** argv) {
    SimpleEdgeStream<int64_t> s;
    long merge_ms = 1000, print_ms = 2000;
    uint64_t window_edges = 0;
    if (argc > 1) {
        if (argc != 4 && argc != 5) {
            std::cerr << "Usage: cc_example <input edges path> <merge window time (ms)> <print window time (ms)> [capacity]\n"
                         "  (file mode: <merge window time> edges per window; the emission of every <print window\n"
                         "   time>-th window is printed; [capacity] distinct ids, default file size / 2, at most 2^28)\n";
            return 1;
        }
        merge_ms = std::atol(argv[2]);
        print_ms = std::atol(argv[3]);
        window_edges = merge_ms > 0 ? (uint64_t)merge_ms : 1;
        uint64_t cap = 0;
        if (argc == 5) {
            cap = std::strtoull(argv[4], nullptr, 0);
        } else {                                     // distinct ids <= 2 per line <= bytes / 2
            struct stat st;
            if (::stat(argv[1], &st) != 0) {
                std::cerr << "cannot stat " << argv[1] << "\n";
                return 2;
            }
            cap = std::min<uint64_t>((uint64_t)st.st_size / 2 + 1, 1ull << 28);
            cap = std::max<uint64_t>(cap, 1024);
        }
        try {
            DisjointSet<int64_t> ds(cap, 0, GS_CC_SPARSE_IDS);
            ConnectedComponents<int64_t> cc(merge_ms, cap, 0, window_edges);
            std::vector<int64_t> v, l;
            // print window p = windows [p * print_ms, (p + 1) * print_ms): FlattenSet + IdentityFold
            // print the emission of its last window, i.e. the summary right after that window closes
            const uint64_t pw = print_ms > 0 ? (uint64_t)print_ms : 1;
            bool pending = false;
            auto flush = [&](DisjointSet<int64_t>& d) {
                d.pairs(v, l);
                for (size_t i = 0; i < v.size(); ++i) std::printf("(%lld,%lld)\n", (long long)v[i], (long long)l[i]);
            };
            cc.runFile(ds, argv[1], [&](DisjointSet<int64_t>& d, uint64_t w) {
                pending = true;
                if ((w + 1) % pw == 0) { flush(d); pending = false; }
            });
            if (pending) flush(ds);
        } catch (const GsError& e) {
            std::cerr << e.what() << "\n";
            return 2;
        }
        return 0;
    } else {
        std::cout << "Executing ConnectedComponentsExample example with default parameters and built-in default data.\n";
        for (long k = 1; k <= 100; ++k) {
            s.src.push_back(k);
            s.dst.push_back(k + 2);
            s.timestamps.push_back(k * 100);
        }
    }
    try {
        ConnectedComponents<int64_t> cc(merge_ms, 0, 0, window_edges);
        // the latest emission, kept current from each window's delta (the emissions are cumulative,
        // so at a print-window boundary it is exactly what FlattenSet + IdentityFold printed)
        std::map<int64_t, int64_t> latest;
        std::vector<int64_t> dv, dl;
        auto wins = s.windows(merge_ms, window_edges);
        size_t wi = 0;
        long current_print = -1;
        auto flush = [&]() {
            for (auto& kv : latest) std::printf("(%lld,%lld)\n", (long long)kv.first, (long long)kv.second);
        };
        cc.run(s, [&](DisjointSet<int64_t>& ds) {
            // event time of this emission = end of its window (count windows: index)
            const auto& w = wins[wi++];
            const long t = s.timestamps.empty() ? (long)wi : (long)s.timestamps[w.second - 1];
            const long pw = print_ms > 0 ? t / print_ms : 0;
            if (current_print >= 0 && pw != current_print) flush();
            current_print = pw;
            ds.delta(dv, dl);                        // FlattenSet + IdentityFold at O(changes)
            for (size_t i = 0; i < dv.size(); ++i) latest[dv[i]] = dl[i];
        });
        flush();
    } catch (const GsError& e) {
        std::cerr << e.what() << "\n";
        return 2;
    }
    return 0;
}
