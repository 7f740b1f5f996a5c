// comm.hip — the multi-GPU CombineCC under the C ABI: gs_comm_* and gs_cc_merge_window.
//
// Replaces the reference's two exchanges of partial summaries (paths relative to the reference's
// src/main/java/org/apache/flink/graph/streaming/):
//   * the windowAll gather of every partition's window result to the parallelism-1 reduce and
//     Merger (SummaryBulkAggregation.java:81-83, SummaryAggregation.java:106-119), and
//   * ConnectedComponentsTree's pairwise tree, partials keyed by partition / 2 per round
//     (SummaryTreeReduce.java:95-123).
// One process per GPU; one RCCL communicator per rank (ncclCommInitRank from a unique id that
// rank 0 makes and the caller distributes, the way torch.distributed or a Flink job's
// configuration would). A partial summary crosses the wire as a DELTA: the (vertex, root) pairs
// of every root this rank hooked since its last export (gs_cc_export_marks), 8 B per pair;
// folding a delta (= DisjointSet.merge over its pairs, DisjointSet.java:127-131) carries every
// component join of that rank's window into another summary.
//
// Transports: RCCL over xGMI (production), or an in-process group of handles on one device driven
// by one thread per rank (gs_comm_create_local: the same exchange code, collectives done with
// device-to-device copies ordered by HIP events and host barriers) for tests on a one-GPU box,
// where RCCL refuses two ranks on one device.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "cc_internal.hpp"

namespace gsgpu {

namespace {

// pairs [n, m) of buf = copies of pair 0 (a repeated union is a no-op): fixed-size slots for the
// all-gather. P = uint2 (dense (vertex, root) uint32 pairs) or P16 (sparse (id, root id) int64
// pairs, 8-B aligned inside count-headed slots)
struct P16 { unsigned long long a, b; };
template <typename P>
__global__ void k_pad_pairs(P* __restrict__ buf, uint64_t n, uint64_t m) {
    const P p = buf[0];
    for (uint64_t i = n + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x)
        buf[i] = p;
}
void pad_pairs(bool sparse, uint32_t* buf, uint64_t n, uint64_t m, hipStream_t s) {
    const dim3 grid((unsigned)std::min<uint64_t>((m - n + 255) / 256, 4096));
    if (sparse) hipLaunchKernelGGL(k_pad_pairs<P16>, grid, dim3(256), 0, s, reinterpret_cast<P16*>(buf), n, m);
    else hipLaunchKernelGGL(k_pad_pairs<uint2>, grid, dim3(256), 0, s, reinterpret_cast<uint2*>(buf), n, m);
}
// bytes / 32-bit words per exported pair
inline uint64_t pbytes(const CcInfo& in) { return in.sparse ? 16 : 8; }
inline uint64_t pwords(const CcInfo& in) { return in.sparse ? 4 : 2; }

// ---- in-process group (tests): threads on one device ----
struct LocalGroup {
    explicit LocalGroup(int w) : world(w), send(w, nullptr), ev(w, nullptr), done(w, nullptr), box((size_t)w * w) {}
    int world;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<const void*> send;
    std::vector<hipEvent_t> ev, done;             // per rank: data ready / peers' reads done
    struct Box {                                   // point-to-point mailbox src -> dst
        const void* p = nullptr;
        size_t bytes = 0;
        hipEvent_t ready = nullptr, taken = nullptr;
        int state = 0;                             // 0 empty, 1 posted, 2 copied
    };
    std::vector<Box> box;
    bool failed = false;                           // a rank's exchange failed: every wait returns
    // false when the group has failed (the caller returns GS_ERR_COMM instead of hanging)
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (failed) return false;
        const uint64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g || failed; });
        }
        return !failed;
    }
    void fail_all() {
        std::lock_guard<std::mutex> lk(mu);
        failed = true;
        cv.notify_all();
    }
};

}  // namespace
}  // namespace gsgpu

using namespace gsgpu;

struct gs_comm {
    int rank = 0, world = 1, device = 0;
    ncclComm_t nccl = nullptr;                     // RCCL transport
    std::shared_ptr<LocalGroup> local;             // or the in-process group
    hipEvent_t ev_ready = nullptr, ev_done = nullptr;
    // exchange buffers (device), sized at the first merge for the handle's capacity
    uint64_t cap_pairs = 0;
    uint64_t pair_bytes = 0;                       // 8: dense (uint32 vertex, root); 16: sparse (int64 ids)
    uint32_t* sendbuf = nullptr;                   // cap_pairs pairs (2 x the handle's capacity)
    uint64_t send_pairs = 0;                       // pairs each send buffer holds (count word included):
                                                   // cap_pairs + 1, more for a prefilter sender's big slice
    uint32_t* sendbuf2 = nullptr;                  // allgather: exports alternate between the two, so a
                                                   // pending window's tail survives the next export
    uint32_t* recvbuf = nullptr;                   // exact rounds: grows to world * m pairs
    size_t recv_bytes = 0;
    uint32_t* slotbuf = nullptr;                   // speculative rounds: world count-headed slots
    size_t slot_bytes = 0;
    unsigned long long* dcnt = nullptr;            // [world + 1]: all-gathered counts, [world] own/received
    unsigned long long* hcnt = nullptr;            // pinned mirror
    bool root_marking_off = false;
    uint64_t spec_slot = 0;                        // allgather: slot size of the speculative round (0: exact)
    gs_cc_t* bound = nullptr;                      // the one handle and mode this communicator serves
    int mode = -1;
    uint64_t reset_gen = 0;                        // the handle's reset generation of the current stream
    bool broken = false;                           // an exchange failed: the communicator is unusable
    hipEvent_t ev_counts = nullptr;                // the speculative round's counts are on the host
    hipEvent_t ev_slots = nullptr;                 // the speculative round's slots have arrived
    hipStream_t side = nullptr;                    // copies the slots' count words to the host
    bool pending = false;                          // a speculative window not yet verified (settle_allgather)
    uint64_t pend_slot = 0;                        // its slot size S
    uint32_t* pend_buf = nullptr;                  // its export (the tail pairs [S, n) are sent from it)
    uint64_t last_delta = 0;                       // the largest delta of the last verified window
    std::vector<uint64_t> gslot;                   // gather: every sender's speculative slot (empty: exact round next)
    uint64_t win = 0;                              // prefilter: windows since the stream's start (broadcast schedule)
    uint32_t* bword = nullptr;                     // prefilter: the broadcast giant slot words (device, 2)
    // prefilter, asynchronous filter-state broadcasts (after the first kBcastSync closes): their own
    // communicator (RCCL: split from the main one at bind; in-process: the same group) and stream
    ncclComm_t nccl_side = nullptr;
    hipStream_t bside = nullptr;
    uint32_t* bstage = nullptr;                    // rank 0: a snapshot [gbits | 2 giant words]; senders: 2 slots
    uint64_t bslot_words = 0;                      // 32-bit words per slot
    hipEvent_t ev_bmain = nullptr;                 // senders: a slot is free (its install ran); rank 0: the
                                                   // last broadcast has read the snapshot
    hipEvent_t ev_brecv[2] = {nullptr, nullptr};   // senders: slot k has arrived; rank 0 ([0]): snapshot taken
    int64_t bpend[2] = {-1, -1};                   // senders: the window whose state slot k holds (-1: none)
    uint64_t bytes_sent = 0, bytes_recv = 0, exchanges = 0, overflows = 0;
};

namespace {

int nccl_fail(ncclResult_t r, const char* what) {
    return fail(GS_ERR_COMM, "%s failed: %s", what, ncclGetErrorString(r));
}
#define GS_NCCL(expr)                                                                        \
    do {                                                                                     \
        ncclResult_t r_ = (expr);                                                            \
        if (r_ != ncclSuccess) return nccl_fail(r_, #expr);                                  \
    } while (0)

// ---- the three collective primitives the exchanges need ----
int allgather(gs_comm_t* c, const void* send, void* recv, size_t bytes, hipStream_t s) {
    if (c->nccl) {
        GS_NCCL(ncclAllGather(send, recv, bytes, ncclUint8, c->nccl, s));
        return GS_OK;
    }
    LocalGroup& g = *c->local;
    GS_HIP(hipEventRecord(c->ev_ready, s));
    g.send[c->rank] = send;
    g.ev[c->rank] = c->ev_ready;
    if (!g.barrier()) return fail(GS_ERR_COMM, "in-process group: a peer's exchange failed");   // buffers published
    for (int q = 0; q < c->world; ++q) {
        if (q != c->rank) GS_HIP(hipStreamWaitEvent(s, g.ev[q], 0));
        GS_HIP(hipMemcpyAsync(static_cast<char*>(recv) + (size_t)q * bytes, g.send[q], bytes, hipMemcpyDeviceToDevice, s));
    }
    GS_HIP(hipEventRecord(c->ev_done, s));
    g.done[c->rank] = c->ev_done;
    if (!g.barrier()) return fail(GS_ERR_COMM, "in-process group: a peer's exchange failed");   // reads enqueued
    for (int q = 0; q < c->world; ++q)             // a send buffer is rewritten only after the
        if (q != c->rank) GS_HIP(hipStreamWaitEvent(s, g.done[q], 0));   // peers' reads of it
    return GS_OK;
}

int send(gs_comm_t* c, const void* p, size_t bytes, int peer, hipStream_t s) {
    if (c->nccl) {
        GS_NCCL(ncclSend(p, bytes, ncclUint8, peer, c->nccl, s));
        return GS_OK;
    }
    LocalGroup& g = *c->local;
    LocalGroup::Box& b = g.box[(size_t)c->rank * c->world + peer];
    GS_HIP(hipEventRecord(c->ev_ready, s));
    std::unique_lock<std::mutex> lk(g.mu);
    b.p = p;
    b.bytes = bytes;
    b.ready = c->ev_ready;
    b.state = 1;
    g.cv.notify_all();
    g.cv.wait(lk, [&] { return b.state == 2 || g.failed; });   // the receiver has enqueued its copy
    if (b.state != 2) return fail(GS_ERR_COMM, "in-process group: a peer's exchange failed");
    b.state = 0;
    const hipEvent_t taken = b.taken;
    lk.unlock();
    if (!taken) return fail(GS_ERR_COMM, "local send of %zu bytes to rank %d: the receiver refused it", bytes, peer);
    GS_HIP(hipStreamWaitEvent(s, taken, 0));       // p is reused only after the copy ran
    return GS_OK;
}

int recv(gs_comm_t* c, void* p, size_t bytes, int peer, hipStream_t s) {
    if (c->nccl) {
        GS_NCCL(ncclRecv(p, bytes, ncclUint8, peer, c->nccl, s));
        return GS_OK;
    }
    LocalGroup& g = *c->local;
    LocalGroup::Box& b = g.box[(size_t)peer * c->world + c->rank];
    std::unique_lock<std::mutex> lk(g.mu);
    g.cv.wait(lk, [&] { return b.state == 1 || g.failed; });
    if (b.state != 1) return fail(GS_ERR_COMM, "in-process group: a peer's exchange failed");
    if (b.bytes != bytes) {
        b.taken = nullptr;
        b.state = 2;
        g.cv.notify_all();
        return fail(GS_ERR_COMM, "local recv of %zu bytes from rank %d, %zu sent", bytes, peer, b.bytes);
    }
    GS_HIP(hipStreamWaitEvent(s, b.ready, 0));
    GS_HIP(hipMemcpyAsync(p, b.p, bytes, hipMemcpyDeviceToDevice, s));
    GS_HIP(hipEventRecord(c->ev_done, s));
    b.taken = c->ev_done;
    b.state = 2;
    g.cv.notify_all();
    return GS_OK;
}

// rank 0's buffer into every rank's buffer of the same address role, in place (side: on the
// prefilter's broadcast communicator; the in-process group serves both, its host barriers order them)
int bcast(gs_comm_t* c, void* buf, size_t bytes, hipStream_t s, bool side = false) {
    if (c->nccl) {
        GS_NCCL(ncclBroadcast(buf, buf, bytes, ncclUint8, 0, side ? c->nccl_side : c->nccl, s));
        return GS_OK;
    }
    LocalGroup& g = *c->local;
    GS_HIP(hipEventRecord(c->ev_ready, s));
    g.send[c->rank] = buf;
    g.ev[c->rank] = c->ev_ready;
    if (!g.barrier()) return fail(GS_ERR_COMM, "in-process group: a peer's exchange failed");
    if (c->rank != 0) {
        GS_HIP(hipStreamWaitEvent(s, g.ev[0], 0));
        GS_HIP(hipMemcpyAsync(buf, g.send[0], bytes, hipMemcpyDeviceToDevice, s));
    }
    GS_HIP(hipEventRecord(c->ev_done, s));
    g.done[c->rank] = c->ev_done;
    if (!g.barrier()) return fail(GS_ERR_COMM, "in-process group: a peer's exchange failed");
    if (c->rank == 0)                              // rank 0's buffer changes only after the copies
        for (int q = 1; q < c->world; ++q) GS_HIP(hipStreamWaitEvent(s, g.done[q], 0));
    return GS_OK;
}

struct Group {                                     // ncclGroupStart/End around p2p batches
    gs_comm_t* c;
    explicit Group(gs_comm_t* c_) : c(c_) { if (c->nccl) (void)ncclGroupStart(); }
    int end() {
        if (c->nccl) GS_NCCL(ncclGroupEnd());
        c = nullptr;
        return GS_OK;
    }
    ~Group() { if (c && c->nccl) (void)ncclGroupEnd(); }
};

// Grows a device buffer. Folds already enqueued on the stream may still read the old one (a
// receive buffer is read by the fold kernels that follow its collective), so the stream drains
// before the free.
int ensure(void** p, size_t* have, size_t need, hipStream_t s) {
    if (*have >= need) return GS_OK;
    if (*p) {
        GS_HIP(hipStreamSynchronize(s));
        GS_HIP(hipFree(*p));
        *p = nullptr;
        *have = 0;
    }
    if (hipMalloc(p, need) != hipSuccess) { (void)hipGetLastError(); return fail(GS_ERR_NOMEM, "hipMalloc(%zu) failed", need); }
    *have = need;
    return GS_OK;
}

int prepare(gs_comm_t* c, gs_cc_t* h, CcInfo* info, int mode) {
    GS_TRY(cc_info(h, info));
    if (mode == GS_MERGE_PREFILTER && info->sparse)
        return fail(GS_ERR_UNSUPPORTED, "GS_MERGE_PREFILTER: dense ids only");
    if (!info->marks && mode != GS_MERGE_PREFILTER)     // (the pre-filter exports no deltas)
        return fail(GS_ERR_UNSUPPORTED, "gs_cc_merge_window: handle created without GS_CC_TRACK_MARKS");
    if (info->device != c->device) return fail(GS_ERR_INVALID, "gs_cc_merge_window: handle on device %d, communicator on %d",
                                               info->device, c->device);
    const uint64_t need = 2ull * info->cap;        // an export never exceeds 2 x capacity pairs
    if (c->cap_pairs < need || c->pair_bytes != pbytes(*info)) {
        if (c->sendbuf) (void)hipFree(c->sendbuf);
        if (c->sendbuf2) (void)hipFree(c->sendbuf2);
        c->sendbuf = c->sendbuf2 = nullptr;
        if (hipMalloc(&c->sendbuf, (size_t)(need + 1) * pbytes(*info)) != hipSuccess ||      // + a count word
            hipMalloc(&c->sendbuf2, (size_t)(need + 1) * pbytes(*info)) != hipSuccess) {
            (void)hipGetLastError();
            c->cap_pairs = 0;
            return fail(GS_ERR_NOMEM, "exchange buffers of %llu pairs", (unsigned long long)need);
        }
        c->cap_pairs = need;
        c->send_pairs = need + 1;
        c->pair_bytes = pbytes(*info);
    }
    return GS_OK;
}

// GS_MERGE_PREFILTER sender: room for every edge of a slice of m edges to survive (a slice can be
// larger than the 2 x capacity pairs the deltas are sized for). Nothing is pending here (the
// window was settled before merge_prefilter), so the old buffers are free once the stream drains.
int ensure_send(gs_comm_t* c, uint64_t m, hipStream_t s) {
    if (m + 1 <= c->send_pairs) return GS_OK;
    GS_HIP(hipStreamSynchronize(s));
    if (c->sendbuf) (void)hipFree(c->sendbuf);
    if (c->sendbuf2) (void)hipFree(c->sendbuf2);
    c->sendbuf = c->sendbuf2 = nullptr;
    c->pend_buf = nullptr;
    c->send_pairs = 0;
    const uint64_t want = std::max<uint64_t>(m + 1, c->cap_pairs + 1);
    if (hipMalloc(&c->sendbuf, (size_t)want * 8) != hipSuccess || hipMalloc(&c->sendbuf2, (size_t)want * 8) != hipSuccess) {
        (void)hipGetLastError();
        return fail(GS_ERR_NOMEM, "prefilter send buffers of %llu pairs", (unsigned long long)want);
    }
    c->send_pairs = want;
    return GS_OK;
}

// Folds deltas laid out in slots of m pairs (slot q: counts[q] real pairs, then copies of its
// first pair; skip[q] = do not fold). While the deltas are big (young windows: components not yet
// joined) each slot is its own fold call, whose short head launch makes the big joins first
// (cc_api.hip kMergeHead); otherwise runs of slots go in one call.
constexpr uint64_t kBulkDeltaPairs = 1ull << 21;
int fold_slots(gs_cc_t* h, const CcInfo& in, const uint32_t* buf, uint64_t m, const std::vector<uint64_t>& cnt,
               const std::vector<char>& skip) {
    const int P = (int)cnt.size();
    const uint64_t pw = pwords(in);
    uint64_t mx = 0;
    for (int q = 0; q < P; ++q) if (!skip[q]) mx = std::max(mx, cnt[q]);
    if (mx == 0) return GS_OK;
    if (mx > kBulkDeltaPairs) {
        for (int q = 0; q < P; ++q)
            if (!skip[q] && cnt[q]) GS_TRY(cc_fold_pairs_any(h, buf + pw * (uint64_t)q * m, cnt[q]));
        return GS_OK;
    }
    int q = 0;
    while (q < P) {
        if (skip[q] || cnt[q] == 0) { ++q; continue; }
        int e = q;
        while (e + 1 < P && !skip[e + 1] && cnt[e + 1]) ++e;
        const uint64_t npairs = (uint64_t)(e - q) * m + cnt[e];     // the last slot: its real pairs only
        GS_TRY(cc_fold_pairs_any(h, buf + pw * (uint64_t)q * m, npairs));
        q = e + 1;
    }
    return GS_OK;
}

// One exact exchange round of the replicated summary: counts all-gathered and read by the host,
// deltas padded to the largest count and all-gathered, the others' slots folded with marking
// paused. *maxc = the largest delta.
int exchange_exact(gs_comm_t* c, gs_cc_t* h, const CcInfo& in, uint64_t* maxc) {
    const int P = c->world;
    hipStream_t s = in.stream;
    GS_TRY(cc_export_async(h, c->sendbuf, c->cap_pairs, c->dcnt + P));
    GS_TRY(allgather(c, c->dcnt + P, c->dcnt, sizeof(unsigned long long), s));
    GS_HIP(hipMemcpyAsync(c->hcnt, c->dcnt, P * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    GS_HIP(hipStreamSynchronize(s));               // the slot size is the largest delta
    std::vector<uint64_t> cnt(P);
    uint64_t m = 0;
    for (int q = 0; q < P; ++q) { cnt[q] = c->hcnt[q]; m = std::max(m, cnt[q]); }
    *maxc = m;
    if (m) {
        const uint64_t n = cnt[c->rank];
        if (n && n < m) pad_pairs(in.sparse, c->sendbuf, n, m, s);
        GS_HIP(hipGetLastError());
        GS_TRY(ensure(reinterpret_cast<void**>(&c->recvbuf), &c->recv_bytes, (size_t)P * m * pbytes(in), s));
        GS_TRY(allgather(c, c->sendbuf, c->recvbuf, m * pbytes(in), s));
        std::vector<char> skip(P, 0);
        skip[c->rank] = 1;
        GS_TRY(gs_cc_set_marking(h, 0));           // the others' deltas are theirs to export
        const int rc = fold_slots(h, in, c->recvbuf, m, cnt, skip);
        GS_TRY(gs_cc_set_marking(h, in.marking ? 1 : 0));   // the caller's marking state back
        GS_TRY(rc);
        c->bytes_sent += m * pbytes(in) * (P - 1);
        c->bytes_recv += m * pbytes(in) * (P - 1);
    }
    return GS_OK;
}

// The slot size of the next speculative exchange: twice the largest delta just seen (at least 4K
// pairs), the same on every rank (every rank saw every count).
uint64_t next_slot(const gs_comm_t* c, uint64_t maxc) {
    uint64_t S = std::max<uint64_t>(2 * maxc, 4096);
    S = (S + 1023) & ~(uint64_t)1023;
    return std::min<uint64_t>(S, c->cap_pairs - 1);
}

// Replicated global summary: every rank folds the others' deltas, so every rank's giant filter is
// the global one and its next delta holds only connectivity new to the whole job.
// Speculative single-collective round (once a slot size S is known): every rank exports its WHOLE
// delta behind a count word, right after its own fold, and the first S pairs of every rank are
// all-gathered in ONE RCCL call; the others' slots are folded and the window is closed with the
// counts read on the device. The host does NOT wait for the counts here: the window is left
// pending (settle_allgather) and verified at the start of the next merge_window, or by any call
// that consumes the emission first (cc_settle: stats, checksum, emit_*, find, sync, ...), by
// which time the counts are long on the host — so the host can enqueue the next window's fold
// while this window's exchange and close still run. A delta larger than S (every rank sees every
// count, so all agree) has its tail sent in one more all-gather, from the same export: the pairs
// must be the exporter's state right after its own fold — re-exported after folding the others'
// slots (marking paused), a root of its own that a foreign pair hooked would vanish from its
// pairs. A tail folded after the next window's local fold is still exact for every emission a
// caller can observe: the next emission closes after it, and the pending window's own emission is
// only readable through a call that settles first. The first window of a stream runs the exact
// round and sizes S.
int settle_allgather(gs_comm_t* c, bool close) {
    if (!c->pending) return GS_OK;
    c->pending = false;
    gs_cc_t* h = c->bound;
    CcInfo in;
    GS_TRY(cc_info(h, &in));
    DeviceGuard g(in.device);
    const int P = c->world;
    hipStream_t s = in.stream;
    const uint64_t S = c->pend_slot;
    uint32_t* send = c->pend_buf;
    GS_HIP(hipEventSynchronize(c->ev_counts));      // normally complete long ago
    std::vector<uint64_t> tail(P, 0);
    uint64_t folded = 0, mt = 0, maxc = 0;
    for (int q = 0; q < P; ++q) {
        const uint64_t n = c->hcnt[q];
        if (n > c->cap_pairs - 1) return fail(GS_ERR_CAPACITY, "rank %d delta of %llu pairs past the export buffer", q,
                                              (unsigned long long)n);
        maxc = std::max<uint64_t>(maxc, n);
        tail[q] = n > S ? n - S : 0;
        mt = std::max<uint64_t>(mt, tail[q]);
        if (q != c->rank) folded += n;
    }
    cc_count_folded(h, folded);
    if (mt) {                                                   // tails past S: one more all-gather
        ++c->overflows;
        uint32_t* t = send + 2 + pwords(in) * S;                // this rank's pairs [S, n)
        const uint64_t n = tail[c->rank];
        if (n && n < mt) pad_pairs(in.sparse, t, n, mt, s);
        GS_HIP(hipGetLastError());
        GS_TRY(ensure(reinterpret_cast<void**>(&c->recvbuf), &c->recv_bytes, (size_t)P * mt * pbytes(in), s));
        GS_TRY(allgather(c, t, c->recvbuf, mt * pbytes(in), s));
        std::vector<char> skip(P, 0);
        skip[c->rank] = 1;
        GS_TRY(gs_cc_set_marking(h, 0));
        const int rc = fold_slots(h, in, c->recvbuf, mt, tail, skip);
        GS_TRY(gs_cc_set_marking(h, in.marking ? 1 : 0));
        GS_TRY(rc);
        c->bytes_sent += mt * pbytes(in) * (P - 1);
        c->bytes_recv += mt * pbytes(in) * (P - 1);
        if (close) GS_TRY(gs_cc_close_window(h));              // (from merge_window: its close follows)
    }
    c->spec_slot = next_slot(c, maxc);
    c->last_delta = maxc;
    return GS_OK;
}

int abort_exchange(gs_comm_t* c, int rc);

// GSGPU_PREFILTER_LOG=1: a sender's survivor count per window on stderr (once known: at once in
// the exact rounds, at the settle of a speculative one) — the real staleness of the broadcast
// bitmap, which tools/sim_ranks.py's filter against the Merger's current state cannot show
void log_survivors(const gs_comm_t* c, uint64_t n) {
    static const bool on = [] { const char* e = getenv("GSGPU_PREFILTER_LOG"); return e && atoi(e) != 0; }();
    if (on) fprintf(stderr, "[gsgpu prefilter] rank %d survivors %llu\n", c->rank, (unsigned long long)n);
}

// cc_settle's callback: a failed verification fails the group (peers may be in the tail round)
int settle_gather(gs_comm_t* c, bool close);
int settle_cb(void* ctx) {
    gs_comm_t* c = static_cast<gs_comm_t*>(ctx);
    const int rc = (c->mode == GS_MERGE_GATHER || c->mode == GS_MERGE_PREFILTER) ? settle_gather(c, true)
                                                                                 : settle_allgather(c, true);
    return rc == GS_OK ? rc : abort_exchange(c, rc);
}

int merge_allgather(gs_comm_t* c, gs_cc_t* h, const CcInfo& in) {
    const int P = c->world;
    hipStream_t s = in.stream;
    uint64_t maxc = 0;
    if (c->spec_slot == 0 && !c->pending) {
        GS_TRY(exchange_exact(c, h, in, &maxc));
        GS_TRY(gs_cc_close_window(h));
        c->spec_slot = next_slot(c, maxc);
        c->last_delta = maxc;
        return GS_OK;
    }
    // 1. this window's export, into the buffer the pending window does not use: its roots are
    //    this rank's forest right after its own fold (the pending window's tails, foreign pairs
    //    folded with marking paused, must not be under them: a root of its own they hooked would
    //    vanish from its pairs)
    uint32_t* send = (c->pending && c->pend_buf == c->sendbuf) ? c->sendbuf2 : c->sendbuf;
    GS_TRY(cc_export_async(h, send + 2, c->cap_pairs - 1, reinterpret_cast<unsigned long long*>(send), 2 * c->last_delta));
    // 2. the previous window's verification (its tail round, if any, is the next collective on
    //    every rank); it sizes this window's slot
    if (c->pending) {
        cc_set_settle(h, nullptr, nullptr);
        GS_TRY(settle_allgather(c, false));
    }
    const uint64_t S = c->spec_slot;
    const uint64_t slot_words = 2 + pwords(in) * S;              // [u64 count][S pairs]
    GS_TRY(ensure(reinterpret_cast<void**>(&c->slotbuf), &c->slot_bytes, (size_t)P * slot_words * 4, s));
    GS_TRY(allgather(c, send, c->slotbuf, slot_words * 4, s));
    // the count words (one per slot, strided) go to the host on a side stream, so the slots' fold
    // and the close start right after the collective; settle_allgather reads them (the next
    // window's collective is enqueued only after that, so the slots are not overwritten under it)
    GS_HIP(hipEventRecord(c->ev_slots, s));
    GS_HIP(hipStreamWaitEvent(c->side, c->ev_slots, 0));
    GS_HIP(hipMemcpy2DAsync(c->hcnt, sizeof(unsigned long long), c->slotbuf, slot_words * 4, sizeof(unsigned long long), P,
                            hipMemcpyDeviceToHost, c->side));
    GS_HIP(hipEventRecord(c->ev_counts, c->side));
    GS_TRY(cc_fold_slots(h, c->slotbuf, slot_words, P, c->rank, S));
    GS_TRY(gs_cc_close_window(h));                              // optimistic: no delta exceeded S
    c->bytes_sent += slot_words * 4 * (P - 1);
    c->bytes_recv += slot_words * 4 * (P - 1);
    c->pending = true;                                          // verified by settle_allgather
    c->pend_slot = S;
    c->pend_buf = send;
    cc_set_settle(h, settle_cb, c);
    return GS_OK;
}

// windowAll: every other rank sends its delta straight to rank 0 (the Merger), which folds them
// all and emits; the other ranks only close their own summaries (their giant filters).
// The exact round (the first window of a stream): counts sent first and read by the host, then
// exactly the pairs. It sizes every sender's speculative slot (gslot).
int merge_gather_exact(gs_comm_t* c, gs_cc_t* h, const CcInfo& in) {
    const int P = c->world;
    hipStream_t s = in.stream;
    c->gslot.assign(P, 0);
    if (c->rank != 0) {
        GS_TRY(cc_export_async(h, c->sendbuf, c->cap_pairs, c->dcnt + P));
        GS_HIP(hipMemcpyAsync(c->hcnt + P, c->dcnt + P, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        GS_HIP(hipStreamSynchronize(s));
        const uint64_t n = c->hcnt[P];
        GS_TRY(send(c, c->dcnt + P, sizeof(unsigned long long), 0, s));
        if (n) GS_TRY(send(c, c->sendbuf, n * pbytes(in), 0, s));
        c->bytes_sent += n * pbytes(in);
        c->gslot[c->rank] = next_slot(c, n);
        c->last_delta = n;
        return gs_cc_close_window(h);
    }
    if (!c->root_marking_off) {                    // rank 0 never exports
        GS_TRY(gs_cc_set_marking(h, 0));
        c->root_marking_off = true;
    }
    {
        Group g(c);
        for (int q = 1; q < P; ++q) GS_TRY(recv(c, c->dcnt + q, sizeof(unsigned long long), q, s));
        GS_TRY(g.end());
    }
    GS_HIP(hipMemcpyAsync(c->hcnt, c->dcnt, P * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    GS_HIP(hipStreamSynchronize(s));
    std::vector<uint64_t> cnt(P, 0);
    uint64_t total = 0, mx = 0;
    for (int q = 1; q < P; ++q) {
        cnt[q] = c->hcnt[q];
        total += cnt[q];
        mx = std::max(mx, cnt[q]);
        c->gslot[q] = next_slot(c, cnt[q]);
    }
    if (total) {
        GS_TRY(ensure(reinterpret_cast<void**>(&c->recvbuf), &c->recv_bytes, (size_t)total * pbytes(in), s));
        {
            Group g(c);
            uint64_t off = 0;
            for (int q = 1; q < P; ++q) {
                if (cnt[q]) GS_TRY(recv(c, c->recvbuf + pwords(in) * off, cnt[q] * pbytes(in), q, s));
                off += cnt[q];
            }
            GS_TRY(g.end());
        }
        if (mx > kBulkDeltaPairs) {                // big deltas one call each (head launch first)
            uint64_t off = 0;
            for (int q = 1; q < P; ++q) {
                if (cnt[q]) GS_TRY(cc_fold_pairs_any(h, c->recvbuf + pwords(in) * off, cnt[q]));
                off += cnt[q];
            }
        } else {
            GS_TRY(cc_fold_pairs_any(h, c->recvbuf, total));
        }
        c->bytes_recv += total * pbytes(in);
    }
    c->last_delta = mx;
    return gs_cc_close_window(h);
}

// The speculative gather's verification (as settle_allgather): a sender whose delta outgrew its
// slot sends the tail [S, n) from the same export; rank 0 knows which senders overflowed from the
// count words of their slots (on the host by now), receives those tails, folds them and, when
// called from cc_settle (an emission read), closes again. Each side then sizes that sender's next
// slot from the same count, so both agree without another message.
int settle_gather(gs_comm_t* c, bool close) {
    if (!c->pending) return GS_OK;
    c->pending = false;
    gs_cc_t* h = c->bound;
    CcInfo in;
    GS_TRY(cc_info(h, &in));
    DeviceGuard g(in.device);
    const int P = c->world;
    hipStream_t s = in.stream;
    GS_HIP(hipEventSynchronize(c->ev_counts));      // normally complete long ago
    if (c->rank != 0) {
        const uint64_t n = c->hcnt[P], S = c->pend_slot;
        if (n > c->send_pairs - 1) return fail(GS_ERR_CAPACITY, "delta of %llu pairs past the export buffer", (unsigned long long)n);
        if (n > S) {
            ++c->overflows;
            GS_TRY(send(c, c->pend_buf + 2 + pwords(in) * S, (n - S) * pbytes(in), 0, s));
            c->bytes_sent += (n - S) * pbytes(in);
        }
        c->gslot[c->rank] = next_slot(c, n);
        c->last_delta = n;
        if (c->mode == GS_MERGE_PREFILTER) log_survivors(c, n);
        return GS_OK;
    }
    std::vector<uint64_t> tail(P, 0);
    uint64_t total = 0, mx = 0, folded = 0;
    for (int q = 1; q < P; ++q) {
        const uint64_t n = c->hcnt[q];
        // (a prefilter sender's survivors are bounded by its slice, which its buffers hold)
        if (c->mode != GS_MERGE_PREFILTER && n > c->cap_pairs - 1)
            return fail(GS_ERR_CAPACITY, "rank %d delta of %llu pairs past the export buffer", q, (unsigned long long)n);
        tail[q] = n > c->gslot[q] ? n - c->gslot[q] : 0;
        folded += n - tail[q];
        total += tail[q];
        mx = std::max(mx, n);
        c->gslot[q] = next_slot(c, n);
    }
    cc_count_folded(h, folded);
    c->last_delta = mx;
    if (total) {
        ++c->overflows;
        GS_TRY(ensure(reinterpret_cast<void**>(&c->recvbuf), &c->recv_bytes, (size_t)total * pbytes(in), s));
        {
            Group gr(c);
            uint64_t off = 0;
            for (int q = 1; q < P; ++q) {
                if (tail[q]) GS_TRY(recv(c, c->recvbuf + pwords(in) * off, tail[q] * pbytes(in), q, s));
                off += tail[q];
            }
            GS_TRY(gr.end());
        }
        GS_TRY(cc_fold_pairs_any(h, c->recvbuf, total));
        c->bytes_recv += total * pbytes(in);
        if (close) GS_TRY(gs_cc_close_window(h));
    }
    return GS_OK;
}

// Speculative gather (from the second window of a stream): each sender exports its whole delta
// behind a count word and sends [count | S_q pairs] in ONE message, S_q sized from its own last
// delta; rank 0 receives every slot, folds them with the counts read on the device and closes —
// no host wait on either side (verified lazily by settle_gather, as the all-gather is).
int merge_gather(gs_comm_t* c, gs_cc_t* h, const CcInfo& in) {
    const int P = c->world;
    hipStream_t s = in.stream;
    if (c->gslot.empty() || P > kMaxSlotCaps) return merge_gather_exact(c, h, in);
    if (c->rank != 0) {
        uint32_t* send_buf = (c->pend_buf == c->sendbuf) ? c->sendbuf2 : c->sendbuf;
        const uint64_t S = c->gslot[c->rank];
        GS_TRY(cc_export_async(h, send_buf + 2, c->cap_pairs - 1, reinterpret_cast<unsigned long long*>(send_buf),
                               2 * c->last_delta));
        GS_TRY(send(c, send_buf, (2 + pwords(in) * S) * 4, 0, s));
        GS_HIP(hipEventRecord(c->ev_slots, s));                 // the count word to the host, aside
        GS_HIP(hipStreamWaitEvent(c->side, c->ev_slots, 0));
        GS_HIP(hipMemcpyAsync(c->hcnt + P, send_buf, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->side));
        GS_HIP(hipEventRecord(c->ev_counts, c->side));
        c->bytes_sent += (2 + pwords(in) * S) * 4;
        GS_TRY(gs_cc_close_window(h));
        c->pending = true;
        c->pend_slot = S;
        c->pend_buf = send_buf;
        cc_set_settle(h, settle_cb, c);
        return GS_OK;
    }
    uint64_t smax = 0;
    for (int q = 1; q < P; ++q) smax = std::max(smax, c->gslot[q]);
    const uint64_t slot_words = 2 + pwords(in) * smax;
    GS_TRY(ensure(reinterpret_cast<void**>(&c->slotbuf), &c->slot_bytes, (size_t)P * slot_words * 4, s));
    {
        Group g(c);
        for (int q = 1; q < P; ++q)
            GS_TRY(recv(c, c->slotbuf + (uint64_t)q * slot_words, (2 + pwords(in) * c->gslot[q]) * 4, q, s));
        GS_TRY(g.end());
    }
    GS_HIP(hipEventRecord(c->ev_slots, s));
    GS_HIP(hipStreamWaitEvent(c->side, c->ev_slots, 0));
    GS_HIP(hipMemcpy2DAsync(c->hcnt, sizeof(unsigned long long), c->slotbuf, slot_words * 4, sizeof(unsigned long long), P,
                            hipMemcpyDeviceToHost, c->side));
    GS_HIP(hipEventRecord(c->ev_counts, c->side));
    GS_TRY(cc_fold_slots(h, c->slotbuf, slot_words, P, 0, smax, c->gslot.data()));
    GS_TRY(gs_cc_close_window(h));                              // optimistic: no delta outgrew its slot
    for (int q = 1; q < P; ++q) c->bytes_recv += (2 + pwords(in) * c->gslot[q]) * 4;
    c->pending = true;
    cc_set_settle(h, settle_cb, c);
    return GS_OK;
}

// ---- GS_MERGE_PREFILTER: the partitions filter, the Merger unions ----
// SummaryBulkAggregation.java:76-83: every partition folds its slice of a window (UpdateCC) and the
// window's partials go to the parallelism-1 Merger, which combines them and emits. Here ranks
// 1..P-1 keep no forest: a rank runs only the giant FILTER of the fold over its slice, against the
// giant bitmap and root rank 0 broadcasts (a stale bitmap is safe: components only merge until
// reset), with its own LDS hot / L2 warm sets, and sends the survivors — plain (u, v) edges — to
// rank 0 in the gather's count-headed slots. Rank 0 folds its own slice and every rank's survivors,
// closes and emits. The filter (the fold's expensive, read-only part) runs on P - 1 GPUs in
// parallel; the unions, the close and the emission stay on the Merger, whose per-window work is the
// survivors (~3.5 % of a steady RMAT-26 window) instead of every rank's full delta fold.
// The first kExactYoung windows of a stream are exact rounds (counts to the host first): their
// survivors are large (a padded speculative slot would move twice their bytes), and rank 0 folds
// them in one call through the young fold. Then speculative slots sized from each sender's last
// count, verified lazily (settle_gather), as the gather. The bitmap and the giant words go out
// after rank 0's closes on the schedule below. A rank may fold no slice of its own (n == 0): every
// rank still runs every window's exchange (the window count is agreed per call, gs_cc_fold_windows).
constexpr uint64_t kExactYoung = 16;
// Filter-state broadcasts (round 6). After the first kBcastSync closes the broadcast is on the
// critical path, as before: the next window's filter waits for it (window 2 needs the giant window 1
// formed; with no bitmap at all every edge of window 2 would go to rank 0). After that they are
// asynchronous (window 3 filters against close 0's bitmap: 3.5 M survivors at the 8-rank RMAT-26
// layout instead of 2.3 M, but its filter overlaps rank 0's window 2; rank model P = 8 2.23 -> 2.27x,
// P = 4 1.77 -> 1.84x with one synchronous broadcast instead of two, profiles/r06_k_sim_ab.txt): rank 0 snapshots
// [gbits | giant words] right after the close and broadcasts the snapshot on a side stream over a
// communicator of their own, while it folds the next windows; a sender receives into one of two
// staging slots on its side stream and installs the state before its filter two windows later
// (a staler bitmap only lets more edges survive: components only merge until reset). While the
// giant grows (windows < kBcastAsyncYoung) every window's state goes out, then every
// kBcastAsyncEvery-th (8 MiB at 2^26 ids, ~130 us of link time at 64 GB/s).
constexpr uint64_t kBcastSync = 1;
constexpr uint64_t kBcastAsyncYoung = 16;
constexpr uint64_t kBcastAsyncEvery = 4;
constexpr uint64_t kBcastLag = 2;                  // installed before the filter of window j + kBcastLag
bool bcast_sync(uint64_t win) { return win < kBcastSync; }
bool bcast_async(uint64_t win) {
    return win >= kBcastSync && (win < kBcastAsyncYoung || win % kBcastAsyncEvery == kBcastAsyncEvery - 1);
}

// side stream, events and staging of the asynchronous broadcasts (first use)
int bside_init(gs_comm_t* c, uint64_t slot_words) {
    if (c->bstage) return GS_OK;                     // (the last piece: everything before it exists)
    // a failed attempt keeps what it created (gs_comm_destroy frees it) and the next one goes on
    if ((!c->bside && hipStreamCreateWithFlags(&c->bside, hipStreamNonBlocking) != hipSuccess) ||
        (!c->ev_bmain && hipEventCreateWithFlags(&c->ev_bmain, hipEventDisableTiming) != hipSuccess) ||
        (!c->ev_brecv[0] && hipEventCreateWithFlags(&c->ev_brecv[0], hipEventDisableTiming) != hipSuccess) ||
        (!c->ev_brecv[1] && hipEventCreateWithFlags(&c->ev_brecv[1], hipEventDisableTiming) != hipSuccess) ||
        hipMalloc(&c->bstage, (size_t)slot_words * 4 * (c->rank == 0 ? 1 : 2)) != hipSuccess) {
        (void)hipGetLastError();
        c->bstage = nullptr;
        return fail(GS_ERR_NOMEM, "prefilter broadcast staging");
    }
    c->bslot_words = slot_words;
    c->bpend[0] = c->bpend[1] = -1;
    return GS_OK;
}

// rank 0, after close(win): the snapshot and its broadcast, off the handle's stream
int bcast_async_send(gs_comm_t* c, gs_cc_t* h, hipStream_t s) {
    uint32_t *gb = nullptr, *words = nullptr;
    uint64_t gbytes = 0;
    GS_TRY(cc_filter_state(h, &gb, &gbytes, &words));
    GS_TRY(bside_init(c, gbytes / 4 + 2));
    // the snapshot is taken on the handle's stream, right after the close: a copy on the side stream
    // could overlap the next close, and a giant switch there (the bitmap rebuilt for another
    // component) would mix two components' bits (8 MiB at 2^26 ids: a few us). The previous
    // broadcast must have read the buffer first.
    GS_HIP(hipStreamWaitEvent(s, c->ev_bmain, 0));
    GS_HIP(hipMemcpyAsync(c->bstage, gb, gbytes, hipMemcpyDeviceToDevice, s));
    GS_HIP(hipMemcpyAsync(c->bstage + gbytes / 4, words, 2 * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    GS_HIP(hipEventRecord(c->ev_brecv[0], s));                  // the snapshot is complete
    GS_HIP(hipStreamWaitEvent(c->bside, c->ev_brecv[0], 0));
    GS_TRY(bcast(c, c->bstage, gbytes + 8, c->bside, true));
    GS_HIP(hipEventRecord(c->ev_bmain, c->bside));              // the buffer may be rewritten after this
    c->bytes_sent += (gbytes + 8) * (c->world - 1);
    return GS_OK;
}

// sender, in the call of window win: receive the state rank 0 broadcasts after close(win) into a slot
int bcast_async_recv(gs_comm_t* c, gs_cc_t* h, uint64_t win) {
    uint32_t *gb = nullptr, *words = nullptr;
    uint64_t gbytes = 0;
    GS_TRY(cc_filter_state(h, &gb, &gbytes, &words));
    GS_TRY(bside_init(c, gbytes / 4 + 2));
    const int k = (int)(win & 1);
    // (the slot's last install was recorded in ev_bmain, which the side stream waits for)
    GS_HIP(hipStreamWaitEvent(c->bside, c->ev_bmain, 0));
    GS_TRY(bcast(c, c->bstage + (size_t)k * c->bslot_words, gbytes + 8, c->bside, true));
    GS_HIP(hipEventRecord(c->ev_brecv[k], c->bside));
    c->bpend[k] = (int64_t)win;
    c->bytes_recv += gbytes + 8;
    return GS_OK;
}

// sender, before the filter of window win: install the state of window win - kBcastLag if it was sent
int bcast_async_install(gs_comm_t* c, gs_cc_t* h, uint64_t win, hipStream_t s) {
    if (win < kBcastLag) return GS_OK;
    const uint64_t j = win - kBcastLag;
    const int k = (int)(j & 1);
    if (c->bpend[k] != (int64_t)j) return GS_OK;
    uint32_t *gb = nullptr, *words = nullptr;
    uint64_t gbytes = 0;
    GS_TRY(cc_filter_state(h, &gb, &gbytes, &words));
    const uint32_t* slot = c->bstage + (size_t)k * c->bslot_words;
    GS_HIP(hipStreamWaitEvent(s, c->ev_brecv[k], 0));
    GS_HIP(hipMemcpyAsync(gb, slot, gbytes, hipMemcpyDeviceToDevice, s));
    GS_TRY(cc_install_giant(h, slot + gbytes / 4));
    GS_HIP(hipEventRecord(c->ev_bmain, s));                      // slot k free for the next receive
    c->bpend[k] = -1;
    return GS_OK;
}

int bcast_filter_state(gs_comm_t* c, gs_cc_t* h, hipStream_t s) {
    uint32_t *gb = nullptr, *words = nullptr;
    uint64_t gbytes = 0;
    GS_TRY(cc_filter_state(h, &gb, &gbytes, &words));
    if (!c->bword) {
        if (hipMalloc(&c->bword, 2 * sizeof(uint32_t)) != hipSuccess) {
            (void)hipGetLastError();
            return fail(GS_ERR_NOMEM, "broadcast words");
        }
    }
    if (c->rank == 0) GS_HIP(hipMemcpyAsync(c->bword, words, 2 * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    {
        Group g(c);
        GS_TRY(bcast(c, gb, gbytes, s));
        GS_TRY(bcast(c, c->bword, 2 * sizeof(uint32_t), s));
        GS_TRY(g.end());
    }
    if (c->rank != 0) GS_TRY(cc_install_giant(h, c->bword));
    if (c->rank == 0) c->bytes_sent += (gbytes + 8) * (c->world - 1);
    else c->bytes_recv += gbytes + 8;
    return GS_OK;
}

int merge_prefilter(gs_comm_t* c, gs_cc_t* h, const CcInfo& in, const void* a, const void* b, uint64_t m) {
    const int P = c->world;
    hipStream_t s = in.stream;
    const uint64_t win = c->win++;
    const bool exact = win < kExactYoung || c->gslot.empty() || P > kMaxSlotCaps;
    if (c->gslot.empty()) c->gslot.assign(P, 0);
    if (c->rank != 0) {
        GS_TRY(ensure_send(c, m, s));
        GS_TRY(bcast_async_install(c, h, win, s));
        if (exact) {
            GS_TRY(cc_filter_async(h, a, b, m, c->sendbuf + 2, c->send_pairs - 1, reinterpret_cast<unsigned long long*>(c->sendbuf)));
            GS_HIP(hipMemcpyAsync(c->hcnt + P, c->sendbuf, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
            GS_HIP(hipStreamSynchronize(s));
            const uint64_t n = c->hcnt[P];
            GS_TRY(send(c, c->sendbuf, sizeof(unsigned long long), 0, s));
            if (n) GS_TRY(send(c, c->sendbuf + 2, n * 8, 0, s));
            c->bytes_sent += n * 8 + 8;
            c->gslot[c->rank] = next_slot(c, n);
            c->last_delta = n;
            c->pend_buf = c->sendbuf;
            log_survivors(c, n);
        } else {
            uint32_t* send_buf = (c->pend_buf == c->sendbuf) ? c->sendbuf2 : c->sendbuf;
            const uint64_t S = c->gslot[c->rank];
            GS_TRY(cc_filter_async(h, a, b, m, send_buf + 2, c->send_pairs - 1, reinterpret_cast<unsigned long long*>(send_buf)));
            GS_TRY(send(c, send_buf, (2 + 2 * S) * 4, 0, s));
            GS_HIP(hipEventRecord(c->ev_slots, s));                 // the count word to the host, aside
            GS_HIP(hipStreamWaitEvent(c->side, c->ev_slots, 0));
            GS_HIP(hipMemcpyAsync(c->hcnt + P, send_buf, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->side));
            GS_HIP(hipEventRecord(c->ev_counts, c->side));
            c->bytes_sent += (2 + 2 * S) * 4;
            c->pending = true;
            c->pend_slot = S;
            c->pend_buf = send_buf;
            cc_set_settle(h, settle_cb, c);
        }
        if (bcast_sync(win)) GS_TRY(bcast_filter_state(c, h, s));
        if (bcast_async(win)) GS_TRY(bcast_async_recv(c, h, win));
        return GS_OK;
    }
    if (!c->root_marking_off) {                    // the Merger never exports
        GS_TRY(gs_cc_set_marking(h, 0));
        c->root_marking_off = true;
    }
    if (exact) {
        {
            Group g(c);
            for (int q = 1; q < P; ++q) GS_TRY(recv(c, c->dcnt + q, sizeof(unsigned long long), q, s));
            GS_TRY(g.end());
        }
        GS_HIP(hipMemcpyAsync(c->hcnt, c->dcnt, P * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        GS_HIP(hipStreamSynchronize(s));
        std::vector<uint64_t> cnt(P, 0);
        uint64_t total = 0, mx = 0;
        for (int q = 1; q < P; ++q) {
            cnt[q] = c->hcnt[q];                 // (at most the sender's slice: its buffers hold it)
            total += cnt[q];
            mx = std::max(mx, cnt[q]);
            c->gslot[q] = next_slot(c, cnt[q]);
        }
        if (total) {
            GS_TRY(ensure(reinterpret_cast<void**>(&c->recvbuf), &c->recv_bytes, (size_t)total * 8, s));
            {
                Group g(c);
                uint64_t off = 0;
                for (int q = 1; q < P; ++q) {
                    if (cnt[q]) GS_TRY(recv(c, c->recvbuf + 2 * off, cnt[q] * 8, q, s));
                    off += cnt[q];
                }
                GS_TRY(g.end());
            }
            // every survivor in one fold call, through the young fold (its internal giant split
            // included): one call per slice cost ~7 dependent launches per young window
            GS_TRY(cc_fold_pairs_any(h, c->recvbuf, total));
            c->bytes_recv += total * 8 + 8 * (P - 1);
        }
        c->last_delta = mx;
        GS_TRY(gs_cc_close_window(h));
    } else {
        uint64_t smax = 0;
        for (int q = 1; q < P; ++q) smax = std::max(smax, c->gslot[q]);
        const uint64_t slot_words = 2 + 2 * smax;
        GS_TRY(ensure(reinterpret_cast<void**>(&c->slotbuf), &c->slot_bytes, (size_t)P * slot_words * 4, s));
        {
            Group g(c);
            for (int q = 1; q < P; ++q)
                GS_TRY(recv(c, c->slotbuf + (uint64_t)q * slot_words, (2 + 2 * c->gslot[q]) * 4, q, s));
            GS_TRY(g.end());
        }
        GS_HIP(hipEventRecord(c->ev_slots, s));
        GS_HIP(hipStreamWaitEvent(c->side, c->ev_slots, 0));
        GS_HIP(hipMemcpy2DAsync(c->hcnt, sizeof(unsigned long long), c->slotbuf, slot_words * 4, sizeof(unsigned long long), P,
                                hipMemcpyDeviceToHost, c->side));
        GS_HIP(hipEventRecord(c->ev_counts, c->side));
        GS_TRY(cc_fold_slots(h, c->slotbuf, slot_words, P, 0, smax, c->gslot.data()));
        GS_TRY(gs_cc_close_window(h));                          // optimistic: no sender outgrew its slot
        for (int q = 1; q < P; ++q) c->bytes_recv += (2 + 2 * c->gslot[q]) * 4;
        c->pending = true;
        cc_set_settle(h, settle_cb, c);
    }
    if (bcast_sync(win)) GS_TRY(bcast_filter_state(c, h, s));
    if (bcast_async(win)) GS_TRY(bcast_async_send(c, h, s));
    return GS_OK;
}

// ConnectedComponentsTree's pairwise rounds (SummaryTreeReduce.enhance): in round r (step 2^r)
// rank i + step sends its delta to rank i (i % 2^(r+1) == 0), which folds it with marking on (it
// forwards what it gained in a later round). After ceil(log2 P) rounds rank 0 holds every edge.
int merge_tree(gs_comm_t* c, gs_cc_t* h, const CcInfo& in) {
    const int P = c->world;
    hipStream_t s = in.stream;
    if (c->rank == 0 && !c->root_marking_off) {
        GS_TRY(gs_cc_set_marking(h, 0));
        c->root_marking_off = true;
    }
    for (int step = 1; step < P; step *= 2) {
        if (c->rank % (2 * step) == step) {        // sender: done for this window after this
            GS_TRY(cc_export_async(h, c->sendbuf, c->cap_pairs, c->dcnt + P));
            GS_HIP(hipMemcpyAsync(c->hcnt + P, c->dcnt + P, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
            GS_HIP(hipStreamSynchronize(s));
            const uint64_t n = c->hcnt[P];
            const int peer = c->rank - step;
            GS_TRY(send(c, c->dcnt + P, sizeof(unsigned long long), peer, s));
            if (n) GS_TRY(send(c, c->sendbuf, n * pbytes(in), peer, s));
            c->bytes_sent += n * pbytes(in);
            break;
        }
        if (c->rank % (2 * step) == 0 && c->rank + step < P) {
            const int peer = c->rank + step;
            GS_TRY(recv(c, c->dcnt, sizeof(unsigned long long), peer, s));
            GS_HIP(hipMemcpyAsync(c->hcnt, c->dcnt, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
            GS_HIP(hipStreamSynchronize(s));
            const uint64_t n = c->hcnt[0];
            if (n) {
                GS_TRY(ensure(reinterpret_cast<void**>(&c->recvbuf), &c->recv_bytes, (size_t)n * pbytes(in), s));
                GS_TRY(recv(c, c->recvbuf, n * pbytes(in), peer, s));
                GS_TRY(cc_fold_pairs_any(h, c->recvbuf, n));
            }
            c->bytes_recv += n * pbytes(in);
        }
    }
    return gs_cc_close_window(h);
}

int alloc_common(gs_comm_t* c) {
    if (hipEventCreateWithFlags(&c->ev_ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_counts, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_slots, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->dcnt, (c->world + 1) * sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc(&c->hcnt, (c->world + 1) * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return fail(GS_ERR_NOMEM, "communicator scratch allocation failed");
    }
    GS_HIP(hipMemset(c->dcnt, 0, (c->world + 1) * sizeof(unsigned long long)));
    return GS_OK;
}

}  // namespace

extern "C" {

int gs_comm_unique_id(void* id, uint64_t id_bytes) {
    if (!id || id_bytes < sizeof(ncclUniqueId)) return fail(GS_ERR_INVALID, "gs_comm_unique_id: need %zu bytes", sizeof(ncclUniqueId));
    ncclUniqueId u;
    GS_NCCL(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof(u));
    return GS_OK;
}

int gs_comm_create(gs_comm_t** out, const void* unique_id, int rank, int world, int device) {
    if (!out || !unique_id) return fail(GS_ERR_INVALID, "gs_comm_create: null argument");
    *out = nullptr;
    if (world < 1 || rank < 0 || rank >= world) return fail(GS_ERR_INVALID, "gs_comm_create: rank %d of %d", rank, world);
    DeviceGuard g(device);
    if (!g.ok) return fail(GS_ERR_HIP, "gs_comm_create: hipSetDevice(%d) failed", device);
    std::unique_ptr<gs_comm_t> c(new gs_comm_t());
    c->rank = rank;
    c->world = world;
    c->device = device;
    GS_TRY(alloc_common(c.get()));
    ncclUniqueId u;
    memcpy(&u, unique_id, sizeof(u));
    const ncclResult_t r = ncclCommInitRank(&c->nccl, world, u, rank);
    if (r != ncclSuccess) {
        c->nccl = nullptr;
        const int rc = nccl_fail(r, "ncclCommInitRank");
        gs_comm_destroy(c.release());
        return rc;
    }
    *out = c.release();
    return GS_OK;
}

int gs_comm_create_local(gs_comm_t** comms, int world, int device) {
    if (!comms || world < 1) return fail(GS_ERR_INVALID, "gs_comm_create_local: bad arguments");
    DeviceGuard g(device);
    if (!g.ok) return fail(GS_ERR_HIP, "gs_comm_create_local: hipSetDevice(%d) failed", device);
    auto grp = std::make_shared<LocalGroup>(world);
    for (int r = 0; r < world; ++r) comms[r] = nullptr;
    for (int r = 0; r < world; ++r) {
        gs_comm_t* c = new gs_comm_t();
        c->rank = r;
        c->world = world;
        c->device = device;
        c->local = grp;
        comms[r] = c;
        const int rc = alloc_common(c);
        if (rc != GS_OK) {
            for (int q = 0; q <= r; ++q) { gs_comm_destroy(comms[q]); comms[q] = nullptr; }
            return rc;
        }
    }
    return GS_OK;
}

int gs_comm_destroy(gs_comm_t* c) {
    if (!c) return GS_OK;
    DeviceGuard g(c->device);
    if (c->pending && c->bound) {                   // verify the last window (peers may be in its tail
        cc_set_settle(c->bound, nullptr, nullptr);  // round), then the handle forgets this communicator
        if (!c->broken) (void)settle_cb(c);
    }
    (void)hipDeviceSynchronize();
    if (c->nccl_side) (void)ncclCommDestroy(c->nccl_side);
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    if (c->bside) (void)hipStreamDestroy(c->bside);
    if (c->ev_bmain) (void)hipEventDestroy(c->ev_bmain);
    for (hipEvent_t e : c->ev_brecv)
        if (e) (void)hipEventDestroy(e);
    if (c->bstage) (void)hipFree(c->bstage);
    if (c->ev_ready) (void)hipEventDestroy(c->ev_ready);
    if (c->ev_done) (void)hipEventDestroy(c->ev_done);
    if (c->ev_counts) (void)hipEventDestroy(c->ev_counts);
    if (c->ev_slots) (void)hipEventDestroy(c->ev_slots);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->sendbuf) (void)hipFree(c->sendbuf);
    if (c->sendbuf2) (void)hipFree(c->sendbuf2);
    if (c->recvbuf) (void)hipFree(c->recvbuf);
    if (c->slotbuf) (void)hipFree(c->slotbuf);
    if (c->bword) (void)hipFree(c->bword);
    if (c->dcnt) (void)hipFree(c->dcnt);
    if (c->hcnt) (void)hipHostFree(c->hcnt);
    delete c;
    return GS_OK;
}

int gs_comm_info(gs_comm_t* c, int* rank, int* world, uint64_t* bytes_sent, uint64_t* bytes_recv, uint64_t* exchanges,
                 uint64_t* overflows) {
    if (!c) return fail(GS_ERR_INVALID, "null communicator");
    // (a pending window's overflow round is counted when it is verified: the next merge_window or
    // any call that consumes the emission)
    if (overflows) *overflows = c->overflows;
    if (rank) *rank = c->rank;
    if (world) *world = c->world;
    if (bytes_sent) *bytes_sent = c->bytes_sent;
    if (bytes_recv) *bytes_recv = c->bytes_recv;
    if (exchanges) *exchanges = c->exchanges;
    return GS_OK;
}

namespace {
// A rank that fails inside an exchange would leave its peers blocked in the next collective: tear
// the communicator down so they fail too (RCCL: ncclCommAbort; in-process: wake every waiter).
int abort_exchange(gs_comm_t* c, int rc) {
    const std::string msg = last_error();
    c->broken = true;
    if (c->nccl_side) {
        (void)ncclCommAbort(c->nccl_side);
        c->nccl_side = nullptr;
    }
    if (c->nccl) {
        (void)ncclCommAbort(c->nccl);
        c->nccl = nullptr;
    }
    if (c->local) c->local->fail_all();
    last_error() = msg;
    return rc;
}

int merge_window(gs_cc_t* h, gs_comm_t* c, int mode, const void* a = nullptr, const void* b = nullptr, uint64_t m = 0) {
    CcInfo in;
    GS_TRY(prepare(c, h, &in, mode));
    // a communicator carries per-stream state (the speculative slot size, rank 0's paused
    // marking): it serves one handle in one mode; a reset of that handle starts a new stream
    if (c->bound && (c->bound != h || c->mode != mode))
        return fail(GS_ERR_INVALID, "gs_cc_merge_window: this communicator serves another handle or mode "
                                    "(one communicator per summary and mode)");
    if (!c->bound) {
        // every rank sizes its exchange buffers from its own handle, and the speculative slots are
        // sized from them on the sending and the receiving side alike (next_slot): agree once, when
        // the communicator is bound, that every rank's capacity and pair width are the same
        // (every rank sees every word, so all fail together on a mismatch)
        const int P = c->world;
        const unsigned long long mine = (unsigned long long)c->cap_pairs << 8 | c->pair_bytes;
        c->hcnt[P] = mine;                           // (pinned: the copy reads it when it runs)
        GS_HIP(hipMemcpyAsync(c->dcnt + P, c->hcnt + P, sizeof(mine), hipMemcpyHostToDevice, in.stream));
        GS_TRY(allgather(c, c->dcnt + P, c->dcnt, sizeof(unsigned long long), in.stream));
        GS_HIP(hipMemcpyAsync(c->hcnt, c->dcnt, P * sizeof(unsigned long long), hipMemcpyDeviceToHost, in.stream));
        GS_HIP(hipStreamSynchronize(in.stream));
        for (int q = 0; q < P; ++q)
            if (c->hcnt[q] != mine)
                return fail(GS_ERR_INVALID, "gs_cc_merge_window: rank %d's summary has %llu-pair / %llu-byte exchange "
                            "buffers, rank %d's %llu / %llu: every rank needs the same vertex capacity and id mode",
                            q, c->hcnt[q] >> 8, c->hcnt[q] & 0xFF, c->rank, (unsigned long long)c->cap_pairs,
                            (unsigned long long)c->pair_bytes);
        if (mode == GS_MERGE_PREFILTER && c->nccl && !c->nccl_side)   // (collective: every rank binds here)
            GS_NCCL(ncclCommSplit(c->nccl, 0, c->rank, &c->nccl_side, nullptr));
        c->bound = h;
        c->mode = mode;
        c->reset_gen = in.reset_gen;
    }
    if (mode != GS_MERGE_ALLGATHER) GS_TRY(cc_settle(h));   // (allgather settles after its export)
    if (in.reset_gen != c->reset_gen) {              // the handle was reset: a new stream
        c->reset_gen = in.reset_gen;
        c->spec_slot = 0;                            // its first window runs the exact round again
        c->gslot.clear();
        c->win = 0;
        c->bpend[0] = c->bpend[1] = -1;              // (broadcasts in flight land, unused)
    }
    DeviceGuard g(in.device);
    switch (mode) {
    case GS_MERGE_ALLGATHER: return merge_allgather(c, h, in);
    case GS_MERGE_GATHER: return merge_gather(c, h, in);
    case GS_MERGE_PREFILTER: return merge_prefilter(c, h, in, a, b, m);
    default: return merge_tree(c, h, in);
    }
}
}  // namespace

extern "C++" {
namespace gsgpu {
int cc_comm_rank(const gs_comm_t* c) { return c ? c->rank : 0; }

// GS_MERGE_PREFILTER (gs_cc_fold_windows): every window is an exchange with rank 0, so every rank
// must run the same number of them. Each rank's slice of a short last global window may be empty,
// a rank's whole slice may be empty: the ranks agree on the largest window count (one all-gather of
// a word per call) and a rank past its own edges runs empty windows (a rank with n == 0
// used to skip the exchange and leave its peers waiting in it).
int cc_agree_windows(gs_cc_t* h, gs_comm_t* c, uint64_t mine, uint64_t* most) {
    if (!c) return fail(GS_ERR_INVALID, "null communicator");
    if (c->broken) return fail(GS_ERR_COMM, "the communicator failed in an earlier exchange");
    CcInfo in;
    GS_TRY(cc_info(h, &in));
    GS_TRY(cc_settle(h));                            // (nothing is pending between calls: settled at their end)
    DeviceGuard g(in.device);
    const int P = c->world;
    auto run = [&]() -> int {
        c->hcnt[P] = mine;                           // (pinned: the copy reads it when it runs)
        GS_HIP(hipMemcpyAsync(c->dcnt + P, c->hcnt + P, sizeof(unsigned long long), hipMemcpyHostToDevice, in.stream));
        GS_TRY(allgather(c, c->dcnt + P, c->dcnt, sizeof(unsigned long long), in.stream));
        GS_HIP(hipMemcpyAsync(c->hcnt, c->dcnt, P * sizeof(unsigned long long), hipMemcpyDeviceToHost, in.stream));
        GS_HIP(hipStreamSynchronize(in.stream));
        uint64_t mx = 0;
        for (int q = 0; q < P; ++q) mx = std::max<uint64_t>(mx, c->hcnt[q]);
        *most = mx;
        return GS_OK;
    };
    const int rc = run();
    return rc == GS_OK ? rc : abort_exchange(c, rc);
}

// gs_cc_fold_windows with GS_MERGE_PREFILTER: the window's own edges go to the exchange (rank 0
// has folded them already; the other ranks filter them there)
int cc_merge_edges(gs_cc_t* h, gs_comm_t* c, int mode, const void* a, const void* b, uint64_t m) {
    if (!c) return fail(GS_ERR_INVALID, "null communicator");
    if (c->broken) return fail(GS_ERR_COMM, "the communicator failed in an earlier exchange");
    const int rc = merge_window(h, c, mode, a, b, m);
    if (rc == GS_OK) {
        ++c->exchanges;
        return rc;
    }
    return abort_exchange(c, rc);
}
}  // namespace gsgpu
}  // extern "C++"

int gs_cc_merge_window(gs_cc_t* h, gs_comm_t* c, int mode) {
    if (!c) return fail(GS_ERR_INVALID, "gs_cc_merge_window: null communicator");
    if (c->broken) return fail(GS_ERR_COMM, "gs_cc_merge_window: the communicator failed in an earlier exchange");
    int rc;
    if (!h) rc = fail(GS_ERR_INVALID, "gs_cc_merge_window: null handle");
    else if (mode == GS_MERGE_PREFILTER)
        rc = fail(GS_ERR_INVALID, "gs_cc_merge_window: GS_MERGE_PREFILTER needs the window's edges (gs_cc_fold_windows)");
    else if (mode != GS_MERGE_ALLGATHER && mode != GS_MERGE_GATHER && mode != GS_MERGE_TREE)
        rc = fail(GS_ERR_INVALID, "gs_cc_merge_window: mode %d", mode);
    else rc = merge_window(h, c, mode);
    if (rc == GS_OK) {
        ++c->exchanges;
        return rc;
    }
    // any failure on one rank (a bad argument included) fails the whole group: its peers are
    // (or will be) waiting for this rank in a collective
    return abort_exchange(c, rc);
}

}  // extern "C"
