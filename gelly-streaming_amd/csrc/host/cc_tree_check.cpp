// cc_tree_check — ConnectedComponents vs ConnectedComponentsTree(degree) on the same stream:
// prints one line per window "w <checksum-of-(vertex,label)> <vertices>" for each operator and
// exits non-zero if any window differs. Edges: whitespace-separated "src dst" lines on stdin.
#include <cstdio>
#include <iostream>
#include <vector>

#include "gsgpu.hpp"

using namespace gelly::streaming;

int main(int argc, char** argv) {
    const uint64_t window = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 4;
    const int degree = argc > 2 ? std::atoi(argv[2]) : 4;
    SimpleEdgeStream<int64_t> s;
    long long a, b;
    while (std::cin >> a >> b) { s.src.push_back(a); s.dst.push_back(b); }
    std::vector<std::map<int64_t, int64_t>> bulk, tree;
    try {
        ConnectedComponents<int64_t>(1000, 0, 0, window).run(s, [&](DisjointSet<int64_t>& ds) { bulk.push_back(ds.getMatches()); });
        ConnectedComponentsTree<int64_t>(1000, degree, 0, 0, window).run(s, [&](DisjointSet<int64_t>& ds) { tree.push_back(ds.getMatches()); });
    } catch (const GsError& e) {
        std::cerr << e.what() << "\n";
        return 2;
    }
    if (bulk.size() != tree.size()) return 1;
    for (size_t w = 0; w < bulk.size(); ++w) {
        std::printf("%zu %zu %s\n", w, bulk[w].size(), bulk[w] == tree[w] ? "same" : "DIFF");
        if (bulk[w] != tree[w]) return 1;
    }
    return 0;
}
