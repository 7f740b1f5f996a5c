// gsgpu.hpp — C++ host mirror of the reference's Connected Components operator surface, over the
// C ABI of libgsgpu.so (include/gsgpu.h). Header-only; no HIP types appear here.
//
// Reference types mirrored (paths relative to src/main/java/org/apache/flink/graph/streaming/):
//   DisjointSet<K>                 summaries/DisjointSet.java:25-150
//   UpdateCC / CombineCC           library/ConnectedComponents.java:70-126
//   SummaryBulkAggregation         SummaryBulkAggregation.java:46-131 (+ Merger, SummaryAggregation.java:94-136)
//   ConnectedComponents(long)      library/ConnectedComponents.java:44-55
//   SimpleEdgeStream::aggregate    SimpleEdgeStream.java:100-102
// Errors: the Java UDFs throw Exception; here a failing ABI call throws gelly::streaming::GsError
// carrying the GS_ERR_* code and gs_last_error() text.
#pragma once

#include <algorithm>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <sstream>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "gsgpu.h"

namespace gelly {
namespace streaming {

class GsError : public std::runtime_error {
public:
    GsError(int code, const std::string& where)
        : std::runtime_error(where + " failed (" + std::to_string(code) + "): " + gs_last_error()), code_(code) {}
    int code() const { return code_; }

private:
    int code_;
};

inline void check(int rc, const char* where) {
    if (rc != GS_OK) throw GsError(rc, where);
}

// One rank's communicator for the multi-GPU CombineCC (gs_comm_*, csrc/comm.hip): RCCL from a
// 128-byte unique id that rank 0 makes (uniqueId) and every rank passes, or an in-process group of
// `world` ranks on one device (local: one thread per rank, for tests).
class Comm {
public:
    using Id = std::vector<uint8_t>;
    static Id uniqueId() {
        Id id(128);
        check(gs_comm_unique_id(id.data(), id.size()), "gs_comm_unique_id");
        return id;
    }
    Comm(const Id& id, int rank, int world, int device = 0) {
        check(gs_comm_create(&c_, id.data(), rank, world, device), "gs_comm_create");
    }
    static std::vector<std::unique_ptr<Comm>> local(int world, int device = 0) {
        std::vector<gs_comm_t*> raw((size_t)world, nullptr);
        check(gs_comm_create_local(raw.data(), world, device), "gs_comm_create_local");
        std::vector<std::unique_ptr<Comm>> out;
        for (gs_comm_t* c : raw) out.emplace_back(new Comm(c));
        return out;
    }
    ~Comm() { gs_comm_destroy(c_); }
    Comm(const Comm&) = delete;
    Comm& operator=(const Comm&) = delete;
    gs_comm_t* handle() const { return c_; }

private:
    explicit Comm(gs_comm_t* c) : c_(c) {}
    gs_comm_t* c_ = nullptr;
};

// DisjointSet<K> on the device. K = int32_t or int64_t ids in [0, capacity); with
// flags = GS_CC_SPARSE_IDS (K = int64_t) any long id, at most `capacity` distinct ones.
template <typename K>
class DisjointSet {
    static_assert(std::is_same<K, int32_t>::value || std::is_same<K, int64_t>::value, "K must be int32_t or int64_t");

public:
    explicit DisjointSet(uint64_t capacity, int device = 0, uint32_t flags = 0) : cap_(capacity) {
        gs_cc_config cfg{};
        cfg.struct_size = sizeof(gs_cc_config);
        cfg.id_bits = sizeof(K) * 8;
        cfg.vertex_capacity = capacity;
        cfg.device = device;
        cfg.flags = flags;
        check(gs_cc_create(&h_, &cfg), "gs_cc_create");
    }
    ~DisjointSet() { gs_cc_destroy(h_); }
    DisjointSet(const DisjointSet&) = delete;
    DisjointSet& operator=(const DisjointSet&) = delete;
    DisjointSet(DisjointSet&& o) noexcept : h_(o.h_), cap_(o.cap_) { o.h_ = nullptr; }

    gs_cc_t* handle() const { return h_; }
    uint64_t capacity() const { return cap_; }

    void reset() { check(gs_cc_reset(h_), "gs_cc_reset"); }

    // makeSet (:53-56) for an id not yet present
    void makeSet(K e) { union_(e, e); }

    // union (:92-118); `union` is a C++ keyword
    void union_(K e1, K e2) { fold(&e1, &e2, 1); }

    // find (:66-80): root, or nullopt for an unknown id (Java null)
    std::optional<K> find(K e) {
        K r = -1;
        uint8_t found = 0;
        check(gs_cc_find_flags(h_, &e, &r, &found, 1), "gs_cc_find_flags");
        if (!found) return std::nullopt;
        return r;
    }

    // merge (:127-131)
    void merge(DisjointSet& other) { check(gs_cc_merge(h_, other.h_), "gs_cc_merge"); }

    // getMatches().size()
    uint64_t size() {
        uint64_t nv = 0, nc = 0;
        check(gs_cc_stats(h_, &nv, &nc), "gs_cc_stats");
        return nv;
    }
    uint64_t numComponents() {
        uint64_t nv = 0, nc = 0;
        check(gs_cc_stats(h_, &nv, &nc), "gs_cc_stats");
        return nc;
    }

    // getMatches() (:44-46) as the canonical vertex -> root map (roots are component minima)
    std::map<K, K> getMatches() {
        std::vector<K> v, l;
        pairs(v, l);
        std::map<K, K> m;
        for (size_t i = 0; i < v.size(); ++i) m.emplace(v[i], l[i]);
        return m;
    }

    // sorted (vertex, label) emission
    void pairs(std::vector<K>& v, std::vector<K>& l) {
        uint64_t n = size(), got = 0;
        v.resize(n);
        l.resize(n);
        check(gs_cc_emit_pairs(h_, v.data(), l.data(), n, &got), "gs_cc_emit_pairs");
        v.resize(got);
        l.resize(got);
    }

    // the per-window delta of the emission (gs_cc_emit_delta): the (vertex, label) pairs new or
    // changed since this summary's previous delta, sorted by vertex — a host-side mirror of the
    // Merger's output stays current at O(changes) per window (SummaryAggregation.java:110-111)
    void delta(std::vector<K>& v, std::vector<K>& l) {
        uint64_t cap = size(), got = 0;
        if (cap == 0) cap = 1;
        for (;;) {
            v.resize(cap);
            l.resize(cap);
            const int rc = gs_cc_emit_delta(h_, v.data(), l.data(), cap, &got);
            if (rc == GS_ERR_CAPACITY) { cap = got; continue; }
            check(rc, "gs_cc_emit_delta");
            break;
        }
        v.resize(got);
        l.resize(got);
    }

    // Merger checkpoint (ListCheckpointed, SummaryAggregation.java:127-135): the summary as its
    // canonical (vertex, label) pairs; restore = reset + union(v, label) for every pair
    void snapshot(std::vector<K>& v, std::vector<K>& l) { pairs(v, l); }
    void restore(const std::vector<K>& v, const std::vector<K>& l) {
        if (v.size() != l.size()) throw GsError(GS_ERR_INVALID, "restore: vertices / labels differ in length");
        reset();
        if (v.empty()) return;
        std::vector<K> inter(2 * v.size());
        for (size_t i = 0; i < v.size(); ++i) { inter[2 * i] = v[i]; inter[2 * i + 1] = l[i]; }
        check(gs_cc_fold_pairs(h_, inter.data(), v.size()), "gs_cc_fold_pairs");
        check(gs_cc_close_window(h_), "gs_cc_close_window");
    }

    // toString (:133-150): {root=[members...], ...}, roots and members ascending
    std::string toString() {
        std::vector<K> v, l;
        pairs(v, l);
        std::map<K, std::vector<K>> comps;
        for (size_t i = 0; i < v.size(); ++i) comps[l[i]].push_back(v[i]);
        std::ostringstream os;
        os << "{";
        bool first = true;
        for (auto& kv : comps) {
            if (!first) os << ", ";
            first = false;
            os << kv.first << "=[";
            for (size_t i = 0; i < kv.second.size(); ++i) os << (i ? ", " : "") << kv.second[i];
            os << "]";
        }
        os << "}";
        return os.str();
    }

    // batched UpdateCC: host or device buffers
    void fold(const K* src, const K* dst, uint64_t n) { check(gs_cc_fold(h_, src, dst, n), "gs_cc_fold"); }
    // after this rank's fold of a window: CombineCC across the ranks + the Merger's close
    // (GS_MERGE_ALLGATHER / GATHER / TREE; the handle needs GS_CC_TRACK_MARKS)
    void mergeWindow(Comm& comm, int mode) { check(gs_cc_merge_window(h_, comm.handle(), mode), "gs_cc_merge_window"); }
    // SummaryBulkAggregation over n edges in windows of windowEdges (this rank's slice of each
    // window): fold + close, or fold + merge over comm (any mode, GS_MERGE_PREFILTER included);
    // returns the windows folded
    uint64_t foldWindows(const K* src, const K* dst, uint64_t n, uint64_t windowEdges, Comm* comm = nullptr,
                         int mode = GS_MERGE_ALLGATHER) {
        uint64_t w = 0;
        check(gs_cc_fold_windows(h_, comm ? comm->handle() : nullptr, mode, src, dst, n, windowEdges, &w), "gs_cc_fold_windows");
        return w;
    }
    void closeWindow() { check(gs_cc_close_window(h_), "gs_cc_close_window"); }
    void sync() { check(gs_cc_sync(h_), "gs_cc_sync"); }

private:
    gs_cc_t* h_ = nullptr;
    uint64_t cap_ = 0;
};

// EdgesFold<K, NullValue, DisjointSet<K>> (ConnectedComponents.java:70-86)
template <typename K>
struct UpdateCC {
    DisjointSet<K>& foldEdges(DisjointSet<K>& ds, K vertex, K vertex2) {
        ds.union_(vertex, vertex2);
        return ds;
    }
    DisjointSet<K>& foldBatch(DisjointSet<K>& ds, const K* src, const K* dst, uint64_t n) {
        ds.fold(src, dst, n);
        return ds;
    }
};

// ReduceFunction<DisjointSet<K>> (ConnectedComponents.java:95-126)
template <typename K>
struct CombineCC {
    DisjointSet<K>* reduce(DisjointSet<K>* s1, DisjointSet<K>* s2) {
        gs_cc_t* out = nullptr;
        check(gs_cc_combine(s1->handle(), s2->handle(), &out), "gs_cc_combine");
        return out == s1->handle() ? s1 : s2;
    }
};

// An edge stream in arrival order with optional event timestamps (ms).
template <typename K>
struct SimpleEdgeStream {
    std::vector<K> src, dst;
    std::vector<int64_t> timestamps;   // empty => no event time

    // [begin, end) edge ranges of the windows: event-time tumbling windows of `millis`
    // (window = ts / millis) or, without timestamps, count windows of `window_edges`
    std::vector<std::pair<size_t, size_t>> windows(int64_t millis, uint64_t window_edges) const {
        std::vector<std::pair<size_t, size_t>> w;
        const size_t n = src.size();
        if (n == 0) return w;
        if (!timestamps.empty() && window_edges == 0) {
            size_t a = 0;
            for (size_t i = 1; i <= n; ++i)
                if (i == n || timestamps[i] / millis != timestamps[i - 1] / millis) { w.emplace_back(a, i); a = i; }
            return w;
        }
        const uint64_t W = window_edges ? window_edges : n;
        for (size_t a = 0; a < n; a += W) w.emplace_back(a, std::min<size_t>(a + W, n));
        return w;
    }
};

// SummaryBulkAggregation specialised to ConnectedComponents: every window's edges are folded into
// the cumulative device summary, the window is closed (compressed), and the Merger emits the
// summary (transientState == false keeps it across windows). Canonical labels equal the
// reference's whatever the partitioning (see gsgpu/aggregation.py, mode "fused").
template <typename K>
class ConnectedComponents {
public:
    explicit ConnectedComponents(long mergeWindowTime, uint64_t vertex_capacity = 0, int device = 0,
                                 uint64_t window_edges = 0)
        : millis_(mergeWindowTime), cap_(vertex_capacity), device_(device), window_edges_(window_edges) {}

    // SummaryAggregation.run -> one emission per window
    void run(const SimpleEdgeStream<K>& s, const std::function<void(DisjointSet<K>&)>& emit) {
        uint64_t cap = cap_;
        if (!cap) {
            K mx = 0;
            for (K x : s.src) mx = std::max(mx, x);
            for (K x : s.dst) mx = std::max(mx, x);
            cap = (uint64_t)mx + 1;
        }
        DisjointSet<K> summary(cap, device_);
        UpdateCC<K> update;
        for (auto& w : s.windows(millis_, window_edges_)) {
            update.foldBatch(summary, s.src.data() + w.first, s.dst.data() + w.first, w.second - w.first);
            summary.closeWindow();
            emit(summary);
        }
    }

    // the same operator over an edge FILE streamed through the device (gs_cc_fold_file: chunks of
    // text read into pinned staging, parsed on the device, folded from device memory; the reference's
    // readTextFile + split + parseLong, ConnectedComponentsExample.java:108-119): count windows of
    // window_edges edges (0: the constructor's), emit(summary, w) after window w's close. `summary`
    // must be a DisjointSet<K> made for the file's ids (GS_CC_SPARSE_IDS for arbitrary longs).
    void runFile(DisjointSet<K>& summary, const std::string& path,
                 const std::function<void(DisjointSet<K>&, uint64_t)>& emit, uint64_t window_edges = 0) {
        struct Ctx { DisjointSet<K>* ds; const std::function<void(DisjointSet<K>&, uint64_t)>* emit; };
        Ctx ctx{&summary, &emit};
        const uint64_t W = window_edges ? window_edges : (window_edges_ ? window_edges_ : (uint64_t)std::max(1L, millis_));
        uint64_t edges = 0, windows = 0;
        check(gs_cc_fold_file(summary.handle(), path.c_str(), W, 0,
                              [](void* c, uint64_t w) { Ctx* x = static_cast<Ctx*>(c); (*x->emit)(*x->ds, w); },
                              &ctx, &edges, &windows),
              "gs_cc_fold_file");
    }

private:
    long millis_;
    uint64_t cap_;
    int device_;
    uint64_t window_edges_;
};

// SummaryTreeReduce specialised to ConnectedComponents (library/ConnectedComponentsTree.java:28-34,
// SummaryTreeReduce.java:68-123): per window, `degree` fresh partial summaries (contiguous slices
// of the window), combined pairwise (key = partition / 2) while more than two remain, then the
// windowAll combine and the Merger's CombineCC(windowResult, summary). Emissions are canonical and
// equal ConnectedComponents' whatever the degree.
template <typename K>
class ConnectedComponentsTree {
public:
    explicit ConnectedComponentsTree(long mergeWindowTime, int degree = 2, uint64_t vertex_capacity = 0,
                                     int device = 0, uint64_t window_edges = 0)
        : millis_(mergeWindowTime), degree_(degree > 0 ? degree : 1), cap_(vertex_capacity), device_(device),
          window_edges_(window_edges) {}

    void run(const SimpleEdgeStream<K>& s, const std::function<void(DisjointSet<K>&)>& emit) {
        uint64_t cap = cap_;
        if (!cap) {
            K mx = 0;
            for (K x : s.src) mx = std::max(mx, x);
            for (K x : s.dst) mx = std::max(mx, x);
            cap = (uint64_t)mx + 1;
        }
        std::vector<std::unique_ptr<DisjointSet<K>>> pool;
        for (int i = 0; i <= degree_; ++i) pool.emplace_back(new DisjointSet<K>(cap, device_));
        DisjointSet<K>* summary = nullptr;
        UpdateCC<K> update;
        CombineCC<K> combine;
        for (auto& w : s.windows(millis_, window_edges_)) {
            std::vector<DisjointSet<K>*> free;
            for (auto& d : pool) if (d.get() != summary) free.push_back(d.get());
            const uint64_t len = w.second - w.first;
            std::vector<DisjointSet<K>*> level;
            for (int p = 0; p < degree_; ++p) {
                const uint64_t a = w.first + len * p / degree_, b = w.first + len * (p + 1) / degree_;
                if (a == b) { level.push_back(nullptr); continue; }
                DisjointSet<K>* part = free.back();
                free.pop_back();
                part->reset();
                update.foldBatch(*part, s.src.data() + a, s.dst.data() + a, b - a);
                level.push_back(part);
            }
            while (level.size() > 2) {                    // enhance(): key = partition / 2
                std::vector<DisjointSet<K>*> next;
                for (size_t i = 0; i < level.size(); i += 2) {
                    DisjointSet<K>* x = level[i];
                    DisjointSet<K>* y = i + 1 < level.size() ? level[i + 1] : nullptr;
                    next.push_back(!x ? y : (!y ? x : combine.reduce(x, y)));
                }
                level.swap(next);
            }
            DisjointSet<K>* acc = nullptr;               // windowAll reduce
            for (auto* x : level) if (x) acc = acc ? combine.reduce(acc, x) : x;
            summary = summary ? combine.reduce(acc, summary) : acc;
            summary->closeWindow();
            emit(*summary);
        }
    }

private:
    long millis_;
    int degree_;
    uint64_t cap_;
    int device_;
    uint64_t window_edges_;
};

}  // namespace streaming
}  // namespace gelly
