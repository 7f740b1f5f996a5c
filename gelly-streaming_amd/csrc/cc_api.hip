// cc_api.hip — the extern "C" boundary of libgsgpu.so (declared in include/gsgpu.h).
// Host-side orchestration of one DisjointSet summary per handle: staging of host buffers,
// kernel launches on the handle's stream, deferred device error reporting, instrumentation.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <mutex>
#include <vector>

#include <hip/hip_ext.h>

#include "cc_internal.hpp"
#include "cc_kernels.hpp"
#include "sparse_ids.hpp"

#include <hipcub/hipcub.hpp>

namespace gsgpu {

std::string& last_error() {
    static thread_local std::string s;
    return s;
}

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    last_error() = buf;
    return code;
}

bool is_device_pointer(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable host memory is unknown to the runtime
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged || a.isManaged;
}

static size_t mark_bytes(uint32_t cap) { return (((size_t)cap + 31) / 32) * 4; }

static unsigned grid_for(uint64_t items, uint64_t per_block, unsigned cap_blocks) {
    uint64_t b = (items + per_block - 1) / per_block;
    if (b == 0) b = 1;
    return (unsigned)(b < cap_blocks ? b : cap_blocks);
}

}  // namespace gsgpu

using namespace gsgpu;

struct gs_cc {
    gs_cc_config cfg{};
    uint32_t cap = 0;
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr;
    uint32_t* parent = nullptr;          // dense summary / label array
    uint32_t* mark = nullptr;            // hook log while marking (GS_CC_TRACK_MARKS), else null
    uint32_t* mark_buf = nullptr;        // the hook log: 2 x capacity entries (cc_kernels.hpp log_append)
    unsigned long long* mark_ctr = nullptr;   // [log length, export cursor], a 128-B line of its own
    uint32_t* gbits = nullptr;           // giant-component filter bitmap (1 bit per vertex)
    uint32_t* sbits = nullptr;           // seen bitmap (1 bit per vertex), set on first touch
    uint32_t* cbits = nullptr;           // ring folds: first touches claimed under the giant root
    uint32_t* hkbits[2] = {nullptr, nullptr}; // roots hooked before any giant exists, by close parity
    bool hkbits_ok = true;               // every fold since the last close marked its hooked roots
    uint32_t* dbits = nullptr;           // delta emission: vertices a close may have relabelled since the last delta
    // list-mode closes (cc_kernels.hpp ListCtl): control words, the NGL (seen vertices outside the
    // giant) and the touch log, each double-buffered by close parity
    uint32_t* lctl = nullptr;
    uint2* ngl[2] = {nullptr, nullptr};
    uint32_t* tlog[2] = {nullptr, nullptr};
    uint32_t ngl_sub = 0;
    bool ilist_ok = true;                // every fold since the last close logged its first touches
    uint32_t ilist_folds = 0;            // logged folds since the last close
    uint32_t ilist_slots = 0;            // touch-log slots they took (one per wave)
    bool list_prev = false;              // the last close built an NGL (list_next)
    bool list_kernel = false;            // the last close ran k_compress_list (its control words are current)
    uint32_t* elab = nullptr;            // delta emission: the labels last emitted (kInvalid: never)
    uint32_t* derr = nullptr;            // derr[0] deferred device error flags; derr[1..5] giant state
    uint32_t* psamp = nullptr;           // 2 x kPickSamples labels a full-pass close recorded (k_compress)
    // a multi-GPU window whose exchange is still to be verified (comm.hip: the speculative
    // all-gather's delta sizes are checked lazily, so the host never waits for them per window):
    // every call that consumes the emission runs it first (cc_settle)
    int (*settle_fn)(void*) = nullptr;
    void* settle_ctx = nullptr;
    unsigned long long* dscratch = nullptr;  // reduction outputs (8 words)
    unsigned long long* hscratch = nullptr;  // pinned mirror
    void* stage = nullptr;               // host->device staging: 2 slots x (src, dst) x staging_edges ids
    size_t stage_bytes = 0;
    hipStream_t copy = nullptr;          // H2D copies of host-buffer folds (double-buffered staging)
    hipEvent_t staged[2] = {nullptr, nullptr}, freed[2] = {nullptr, nullptr};
    void* tmp = nullptr;                 // emission temporaries
    size_t tmp_bytes = 0;
    // delta emission (gs_cc_emit_delta[_async]): two slots of packed pairs; an async emission's
    // slot is copied out on estream (k_delta_copy: device / pinned buffers) or at gs_cc_emit_wait
    struct EmitSlot { void* mem = nullptr; size_t bytes = 0; hipEvent_t staged = nullptr, done = nullptr; };
    EmitSlot eslot[2];
    unsigned long long* ecount = nullptr;    // pinned: the size of each slot's delta
    hipStream_t estream = nullptr;
    struct EmitPend { int slot; uint64_t* n_out; uint64_t cap; void* vertices; void* labels; bool kcopy; };
    EmitPend epend[2];                   // async emissions not yet waited for, oldest first
    int n_epend = 0;
    uint32_t enext = 0;                  // slot of the next emission
    bool compressed = true;
    bool sbits_stale = false;            // a young launch skipped the seen bits: the next close rebuilds them
    uint64_t edges_since_reset = 0;      // drives the young-forest launch split (fold_impl)
    uint64_t ring_launches = 0;          // ring fold launches since reset (hot-set admission cadence)
    uint64_t closes = 0;                 // compressions since reset (giant re-sampled every kPickEvery)
    uint64_t pick_edges = 0;             // edges_since_reset at the last forced giant re-pick
    uint64_t reset_gen = 0;              // gs_cc_reset calls (a communicator's per-stream state follows it)
    unsigned long long* dstats = nullptr;    // GSGPU_FOLD_STATS=1: per-window fold counters
    unsigned ring_clock_groups = 0;          // ... and the last k_fold_ring launch's clocks (its grid)
    uint2* hot = nullptr;                // LDS hot set master copy (kHotBuckets uint2), steady folds
    uint32_t hot_bits = 0;               // ids < 2^hot_bits
    uint32_t* hot_cand = nullptr;        // hot-set admission candidates (2^kHotCandBits ids)
    uint32_t* warm = nullptr;            // warm set (2^warm_bits words, L2-resident), steady folds
    uint32_t warm_bits = 0;
    uint32_t* wkeys = nullptr;           // warm build: sampled endpoint key slots
    uint16_t* wpart = nullptr;           // warm build: keys by hash bucket
    unsigned long long* wctl = nullptr;  // warm build: [0] edges counted, then bucket fills (u32)
    uint64_t warm_sample = 0;            // edges a warm count launch samples
    uint32_t warm_bcap = 0;              // keys per hash bucket
    int cus = 0;                         // compute units: k_fold_ring grid
    void* ingest = nullptr;              // streaming text ingestion state (parse.hip), freed by ingest_free
    uint2* fscratch = nullptr;           // partition pre-filter: per-workgroup survivor regions
    size_t fscratch_bytes = 0;
    void* fstage = nullptr;              // ... and the device copy of host edge batches
    size_t fstage_bytes = 0;
    void (*ingest_free)(void*) = nullptr;
    // GS_CC_SPARSE_IDS: id -> slot table; cap (above) = slots = 2^hbits + 1
    bool sparse = false;
    int64_t* keys = nullptr;             // 2^hbits slot keys (INT64_MIN = empty)
    uint32_t hbits = 0;
    unsigned long long* nkeys = nullptr; // distinct ids inserted
    int64_t* minkey = nullptr;           // per root: minimum id of its component (emission)
    bool minkey_valid = false;
    // instrumentation
    bool timing = false;
    uint32_t timing_mask = ~0u;          // kernels timed while timing (bit GS_K_*)
    int fold_timer = GS_K_FOLD;          // GS_K_MERGE while folding an exported partial summary
    struct Pend { int k; hipEvent_t a, b; uint64_t units; };
    std::vector<Pend> pending;
    std::vector<hipEvent_t> pool;
    double total_ms[GS_K_COUNT] = {};
    uint64_t launches[GS_K_COUNT] = {};
    uint64_t units[GS_K_COUNT] = {};     // edges (folds, merges) or vertices (closes) the timed launches took
};

namespace {

int check(gs_cc_t* h) {
    if (!h) return fail(GS_ERR_INVALID, "null handle");
    return GS_OK;
}

int ensure_buf(void** p, size_t* have, size_t need) {
    if (*have >= need) return GS_OK;
    if (*p) { GS_HIP(hipFree(*p)); *p = nullptr; *have = 0; }
    if (hipMalloc(p, need) != hipSuccess) { (void)hipGetLastError(); return fail(GS_ERR_NOMEM, "hipMalloc(%zu) failed", need); }
    *have = need;
    return GS_OK;
}

hipEvent_t get_event(gs_cc_t* h) {
    if (!h->pool.empty()) { hipEvent_t e = h->pool.back(); h->pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

// Times one span of launches of kernel class k (HIP events on the launch stream). Launch the
// span's first kernel with start() and its last with stop() through klaunch().
// the current giant-state slot (cc_kernels.hpp): derr[1 + 2 * (closes & 1)] = giant, [+1] = built;
// close c reads slot c & 1 and writes slot (c + 1) & 1; derr[5] = hot set owner, derr[6] = hot
// set admission budget, derr[7] = warm set valid
inline uint32_t* giant_state(gs_cc_t* h) { return h->derr + 1 + 2 * (h->closes & 1); }
// derr[kWorkWord..+1]: the young k_fold's dynamic chunk counter, an atomicAdd per chunk from every
// workgroup: on a 128-B line of its own, away from the giant state every union reads (sharing
// its line made a hoisted read of the giant root 2.6x slower in window 1, profiles/r02_h)
constexpr uint32_t kWorkWord = 32;
constexpr size_t kDerrBytes = 256;

// The events ride on the kernel dispatches themselves (hipExtLaunchKernelGGL start/stop events):
// separate hipEventRecord marker packets are barrier packets, ~10 us of idle GPU each on gfx950
// (profiles/r01_v3).
struct KTimer {
    gs_cc_t* h; int k; hipEvent_t a = nullptr, b = nullptr; uint64_t units;
    KTimer(gs_cc_t* h_, int k_, uint64_t units_ = 0) : h(h_), k(k_), units(units_) {
        if (!h->timing || !(h->timing_mask & (1u << k))) return;
        a = get_event(h);
        b = get_event(h);
    }
    hipEvent_t start() const { return a; }
    hipEvent_t stop() const { return b; }
    ~KTimer() {
        if (a) h->pending.push_back({k, a, b, units});
    }
};

// hipLaunchKernelGGL with optional start/stop events attached to the dispatch
template <typename F, typename... Args>
inline void klaunch(F kernel, dim3 grid, dim3 block, hipStream_t s, hipEvent_t start, hipEvent_t stop, Args... args) {
    if (start || stop) hipExtLaunchKernelGGL(kernel, grid, block, 0, s, start, stop, 0, args...);
    else hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
}

int resolve_timing(gs_cc_t* h) {
    for (auto& p : h->pending) {
        GS_HIP(hipEventSynchronize(p.b));
        float ms = 0.f;
        GS_HIP(hipEventElapsedTime(&ms, p.a, p.b));
        h->total_ms[p.k] += ms;
        h->launches[p.k] += 1;
        h->units[p.k] += p.units;
        h->pool.push_back(p.a);
        h->pool.push_back(p.b);
    }
    h->pending.clear();
    return GS_OK;
}

int sync_and_check(gs_cc_t* h) {
    uint32_t* hflag = reinterpret_cast<uint32_t*>(h->hscratch + 7);
    GS_HIP(hipMemcpyAsync(hflag, h->derr, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
    GS_HIP(hipStreamSynchronize(h->stream));
    if (*hflag) {
        const uint32_t f = *hflag;
        *hflag = 0;
        GS_HIP(hipMemsetAsync(h->derr, 0, sizeof(uint32_t), h->stream));
        if (f & 2u)
            return fail(GS_ERR_CAPACITY, "more than %llu distinct ids were folded into a sparse-id summary",
                        (unsigned long long)h->cfg.vertex_capacity);
        return fail(GS_ERR_RANGE, "a vertex id outside [0, %u) was folded; such edges were skipped", h->cap);
    }
    return GS_OK;
}

// ---- tuning constants (MI355X, RMAT-26 EF16, 2^24-edge windows unless noted) ----
// Young forest (fewer than capacity/4 edges folded since reset): ONE launch of k_fold with a
// dynamic chunk counter, kYoungBlocksPerCu workgroups per CU, kYoungEpt edges per thread (edges in
// flight = CUs x 2 x 256 x 2 is what bounds the hub contention): window 1 64 launches of 2^18
// edges 1746 us, one launch 2/CU 1403 us, 4/CU 2265 us; EPT 4 -> 2: 1873 -> 1715 us.
constexpr int kYoungEpt = 2;
constexpr unsigned kYoungBlocksPerCu = 2;
// the first young launch after reset: at most 1/kYoungFirstDiv of its edges in flight (headline
// RMAT-26 sweep of the divisor 16 / 32 / 64 / 128 / 256: 16.29 / 16.25 / 16.47 / 17.03 / 18.19 ms
// per step, profiles/r03_yfirst_sweep.txt; at 2^22 edges 16 keeps the 2-per-CU grid)
constexpr uint64_t kYoungFirstDiv = 16;
// ... and at least this many workgroups (config 2's 2^18-edge first launch: floor 8 / 16 / 32 / 64
// -> 0.613 / 0.610 / 0.608 / 0.566 ms per step, profiles/r03_yfloor.txt; launches of 2^19 edges and
// more, configs 3 and 4, are above the floor)
constexpr uint64_t kYoungFirstMinWg = 64;
// Folding a partial summary (AOS pairs: fold_pairs / the multi-GPU merge): the pairs (v, R) of one
// component all name its root R; while R's component is not yet joined to the receiver's, every
// pair in flight CASes the same word (RMAT-26 window-1 deltas: 5-14 ms for 6M pairs). A head
// launch of kMergeHead pairs makes the big joins first (8 ranks' window-1 merges: 32 ms in one
// launch each, 2.1 ms with a 2^10 head; 2^14: 2.6, 2^17: 6.5), then the rest in one launch.
constexpr uint64_t kMergeHead = 1u << 10;
constexpr uint64_t kMergeBulk = 1ull << 20;   // smaller batches: one launch (a delta of a mature
                                              // summary rarely joins big components)
// k_compress grid: the incremental close is a bitmap scan; 16384 workgroups cost 140 us more per
// 64-window step than 2048 (young closes: 8192-65536 gave the same sum as 2048)
constexpr unsigned kCompressGrid = 2048;          // 1024-8192 swept: 2048 fastest (r02_bl/bm)
// Steady ring fold and its warm set from ids >= 2^kRingMinBits (gbits outgrows an XCD's 4 MiB L2):
// with gbits L2-resident the hot set's 128 KiB LDS fill per workgroup costs more than it saves
// (RMAT-20 2^20-edge windows: ring 83 us, plain 61 us; ER 2^24: 141 vs 126 us).
constexpr uint32_t kRingMinBits = 25;
// warm set: counted in ring launch kWarmAt after reset (the first warm_sample edges: kWarmSample,
// at most capacity/8) and re-checked every kWarmEvery-th launch (rebuilt only when invalid for the
// current giant). Launch 2 (RMAT-26 window 4): windows 2-12 35 us less than launch 3, as launch 0
// or 1 (profiles/r02_ab_experiments.txt r02_w); 2^24-edge samples gained nothing (r02_u)
constexpr uint64_t kWarmAt = 2, kWarmEvery = 64, kWarmSample = 1ull << 23;   // every 16 -> 64: r02_bg
constexpr uint32_t kWarmBucketsMaxBits = 18;
                                                    // slower per steady window, r02_u)
constexpr uint32_t kHotThresh = 3;                  // sightings before hot-set admission (233 -> 229 us)
// Young split: inside the young forest, close internally (compress + giant pick: no emission,
// labels stay canonical) after S edges, so the rest of the young window folds with the giant
// filter on. Round 2 measured it at capacity/16 edges: RMAT-26 window 1 1487 -> 1297 us. Round 5,
// with the young fold's claims and the seen-bit skip since: 16.452-16.481 ms per step without it
// against 16.572-16.589 with it, three alternations on one box (profiles/r05_young_split_ab.txt) —
// off by default, GSGPU_YOUNG_SPLIT=S turns it on (the variant tests run it).
// kYoungSplitDiv: a young launch of >= capacity/kYoungSplitDiv edges skips the seen bitmap (below).
constexpr uint32_t kYoungSplitDiv = 16;
// Small plain folds (config 5's 2^16-edge windows): one edge per thread, so a launch spreads over
// more workgroups and each thread's chain of dependent unions is one union long (a 2^16-edge launch
// at 4 edges per thread filled 64 workgroups). Config 5: 3.94 -> 5.09 G edges/s, per-window latency
// p50 29.9 -> 23.5 us; at 2^20 edges per launch config 2 +3 %, config 4 -1.5 % (profiles/r03_small)
constexpr uint64_t kSmallFoldEdges = 1u << 18;
// Pair / survivor folds (AOS: the prefilter Merger's survivors, exported partial summaries) take one
// edge per thread up to this many pairs: a mature window's survivors (0.2-3.5 M at the 8-rank
// RMAT-26 layout) are latency chains (gbits lookups, walks, a CAS), and four per thread ran them
// four deep. One-GPU rank model at P = 8: the Merger's survivor folds 5.26 -> 4.33 ms per step,
// window 5's 300 -> 141 us, the model 2.01 -> 2.20x (profiles/r06_f_sim_p8_*.txt)
constexpr uint64_t kSmallPairFold = 1ull << 22;
// list-mode closes: one-edge-per-thread folds log their first touches into one touch-log slot per
// wave, up to kTlogSlots slots per window (2^18 edges; beyond: the close is a bitmap or full one)
constexpr uint32_t kTlogSlots = 4096;
constexpr int kSmallEpt = 1;

// ---- debug variables (read once per process; none is needed in production) ----
//   GSGPU_FOLD_STATS=1       per-window fold counters on stderr (STATS kernel variants; same results)
//   GSGPU_RING_CLOCKS=1      per-workgroup phase clocks of the window's last k_fold_ring launch on stderr
//   GSGPU_FOLD_MODE=plain|ring|auto   force the steady fold variant (parity tests of each variant)
//   GSGPU_RING_MIN_BITS=B    ring fold + warm set from ids >= 2^B instead of 2^25 (tests at small sizes)
//   GSGPU_YOUNG_SPLIT=S      young split after S edges (default: none; tests and A/B)
//   GSGPU_PAIR_COMBINE=0     pair / survivor folds without wave-combined hooks (A/B)
enum FoldMode { kFoldPlain = 0, kFoldRing = 1, kFoldAuto = 2 };
struct DebugEnv {
    bool fold_stats = false;
    int ring_clocks = 0;                            // GSGPU_RING_CLOCKS=1: k_fold_ring phase clocks on stderr (2: per XCD)
    int fold_mode = kFoldAuto;
    uint32_t ring_min_bits = kRingMinBits;
    uint64_t young_split = ~0ull;                   // ~0: the production rule
    uint64_t small_fold = kSmallFoldEdges;          // GSGPU_SMALL_FOLD: plain folds of at most this many edges...
    int small_ept = kSmallEpt;                      // GSGPU_SMALL_EPT: ...take this many edges per thread
    uint64_t young_first_min = kYoungFirstMinWg;    // GSGPU_YOUNG_FIRST_MIN: workgroup floor of the first young launch
    bool list_close = true;                         // GSGPU_LIST_CLOSE=0: no list-mode closes (A/B)
    bool small_claim = true;                        // GSGPU_SMALL_CLAIM=0: small k_fold launches without claims (A/B)
    bool pair_combine = true;                       // GSGPU_PAIR_COMBINE=0: pair folds without combined hooks (A/B)
    uint32_t pair_halve = 1;                        // GSGPU_PAIR_HALVE=0: pair folds walk read-only (A/B)
    DebugEnv() {
        const char* e = getenv("GSGPU_FOLD_STATS");
        fold_stats = e && atoi(e) != 0;
        e = getenv("GSGPU_RING_CLOCKS");
        ring_clocks = e ? atoi(e) : 0;
        e = getenv("GSGPU_FOLD_MODE");
        if (e && !strcmp(e, "plain")) fold_mode = kFoldPlain;
        if (e && !strcmp(e, "ring")) fold_mode = kFoldRing;
        e = getenv("GSGPU_RING_MIN_BITS");
        if (e && *e) ring_min_bits = (uint32_t)strtoul(e, nullptr, 0);
        e = getenv("GSGPU_YOUNG_SPLIT");
        if (e && *e) young_split = strtoull(e, nullptr, 0);
        e = getenv("GSGPU_SMALL_FOLD");
        if (e && *e) small_fold = strtoull(e, nullptr, 0);
        e = getenv("GSGPU_YOUNG_FIRST_MIN");
        if (e && *e) young_first_min = std::max<uint64_t>(1, strtoull(e, nullptr, 0));
        e = getenv("GSGPU_SMALL_EPT");
        if (e && *e) small_ept = atoi(e) == 1 ? 1 : (atoi(e) == 2 ? 2 : 4);
        e = getenv("GSGPU_LIST_CLOSE");
        if (e && *e) list_close = atoi(e) != 0;
        e = getenv("GSGPU_SMALL_CLAIM");
        if (e && *e) small_claim = atoi(e) != 0;
        e = getenv("GSGPU_PAIR_COMBINE");
        if (e && *e) pair_combine = atoi(e) != 0;
        e = getenv("GSGPU_PAIR_HALVE");
        if (e && *e) pair_halve = atoi(e) != 0 ? 1u : 0u;

    }
};
static const DebugEnv& dbg() {
    static const DebugEnv d;
    return d;
}

static void ensure_stats(gs_cc_t* h) {
    if (dbg().fold_stats && !h->dstats) {
        (void)hipMalloc(&h->dstats, 8 * sizeof(unsigned long long));
        (void)hipMemsetAsync(h->dstats, 0, 8 * sizeof(unsigned long long), h->stream);
    }
}

// Vertices a ring fold claims straight under the giant root go to their own bitmap (cbits); the
// next incremental close sets their gbits bits without reading parent[]: closes -165 us per 40
// RMAT-26 windows, folds unchanged (profiles/r02_ab_experiments.txt r02_bd)
constexpr bool kUseCbits = true;
static WarmBuild warm_build_args(gs_cc_t* h);
static void launch_warm_build(gs_cc_t* h, hipEvent_t stop, hipStream_t s);


template <typename IdT, bool AOS>
void launch_fold(gs_cc_t* h, const void* a, const void* b, uint64_t n, bool young = false) {
    const uint64_t small = AOS ? std::max<uint64_t>(kSmallPairFold, dbg().small_fold) : dbg().small_fold;
    const int ept = young ? kYoungEpt : (n <= small ? dbg().small_ept : kEdgesPerThread);
    const bool persist = young && h->cus > 0;
    // The first young launch after reset folds into an EMPTY forest: every hub's first hooks and
    // the giant root's repeated re-hooks collide there, so it keeps at most ~1/16 of its edges in
    // flight (>= 32 workgroups). BASELINE config 2 (RMAT-20, the whole 2^18-edge launch in flight
    // at 2/CU): 0.97 -> 0.64 ms per step; configs 3-5 unchanged (profiles/r03_ygrid2).
    const uint64_t ycap = h->edges_since_reset ? ~0ull
                                               : std::max<uint64_t>(dbg().young_first_min, n / (kYoungFirstDiv * kFoldThreads * kYoungEpt));
    const unsigned grid = persist ? (unsigned)std::min<uint64_t>(std::min<uint64_t>((uint64_t)h->cus * kYoungBlocksPerCu, ycap),
                                                                  grid_for((n + ept - 1) / ept, kFoldThreads, 1u << 20))
                                  : grid_for((n + ept - 1) / ept, kFoldThreads, 16384);
    ensure_stats(h);
    FoldArgs f{n, h->parent, h->mark, h->sbits, h->gbits, giant_state(h), RangeCheck{h->cap, h->derr}, h->dstats};
    f.mark_len = h->mark_ctr;
    f.combine = (AOS && dbg().pair_combine) ? 1u : 0u;   // pair / survivor folds (combine_hooks)
    if (AOS) f.halve = dbg().pair_halve;
    // hooked roots marked (while no giant exists, k_fold) by mature SoA launches only: in the young
    // forest the marks would cost an atomic per hook for a close whose grandparent reads hit L2
    // anyway (an RMAT window 1's non-roots hang under a few hub roots)
    if (!young && !AOS && h->hkbits[0]) f.hbits = h->hkbits[h->closes & 1];
    else h->hkbits_ok = false;
    // a big young launch (>= capacity/16 edges, i.e. window 1 of the headline) leaves the seen
    // bitmap to the close that follows it — a full pass in any case while the forest is this
    // young — and saves one device-scope atomic per new vertex (window 1: ~6.4M)
    if (young && !AOS && n >= h->cap / kYoungSplitDiv) {
        f.sbits = nullptr;
        h->sbits_stale = true;
    }
    // one-edge-per-thread mature SoA folds log their first touches (touch-log slots) for a list-mode
    // close; any other fold makes the next close a bitmap or full one
    const uint32_t waves = grid * (kFoldThreads / 64);
    const uint32_t claim = (!young && ept == 1 && dbg().small_claim) ? 1u : 0u;
    if (h->lctl && !young && !AOS && !h->dbits && dbg().list_close && ept == 1 && !persist &&
        (uint64_t)grid * kFoldThreads >= n && h->ilist_slots + waves <= kTlogSlots) {
        f.tlog = h->tlog[h->closes & 1] + (size_t)h->ilist_slots * kSlotWords;
        ++h->ilist_folds;
        h->ilist_slots += waves;
    } else {
        h->ilist_ok = false;
    }
    if (persist) {
        f.work = reinterpret_cast<unsigned long long*>(h->derr + kWorkWord);
        (void)hipMemsetAsync(f.work, 0, sizeof(unsigned long long), h->stream);
    }
    const bool vec = std::is_same<IdT, uint32_t>::value && !AOS &&
                     ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0;
    KTimer t(h, h->fold_timer, n);
#define GS_LAUNCH_FOLD(MARKV, VECV, EPTV, STV)                                                                       \
    klaunch((k_fold<IdT, AOS, MARKV, VECV, EPTV, STV>), dim3(grid), dim3(kFoldThreads), h->stream, t.start(), t.stop(), \
            (const IdT*)a, (const IdT*)b, f, claim)
    if (h->dstats) { if (h->mark) GS_LAUNCH_FOLD(true, false, 4, true); else GS_LAUNCH_FOLD(false, false, 4, true); }
    else if (ept == kYoungEpt) { if (h->mark) GS_LAUNCH_FOLD(true, false, kYoungEpt, false); else GS_LAUNCH_FOLD(false, false, kYoungEpt, false); }
    else if (ept == 1) { if (h->mark) GS_LAUNCH_FOLD(true, false, 1, false); else GS_LAUNCH_FOLD(false, false, 1, false); }
    else if (h->mark) { if (vec) GS_LAUNCH_FOLD(true, true, 4, false); else GS_LAUNCH_FOLD(true, false, 4, false); }
    else { if (vec) GS_LAUNCH_FOLD(false, true, 4, false); else GS_LAUNCH_FOLD(false, false, 4, false); }
#undef GS_LAUNCH_FOLD
}

// Steady-state fold (mature forest, aligned device uint32 SoA): k_fold_ring (LDS hot set + warm set
// + survivor rings, one persistent launch) once gbits outgrows an XCD's L2, else k_fold as for
// young windows (GSGPU_FOLD_MODE forces either)
static bool use_ring(const gs_cc_t* h) {
    const int m = dbg().fold_mode;
    return m == kFoldRing || (m == kFoldAuto && h->hot_bits >= dbg().ring_min_bits);
}

static void launch_warm_build(gs_cc_t* h, hipEvent_t stop, hipStream_t s) {
    const WarmBuild w = warm_build_args(h);
    klaunch(k_warm_part, dim3((unsigned)((w.keys_cap + kWarmPartTile - 1) / kWarmPartTile)), dim3(1024), s, nullptr,
            nullptr, w);
    klaunch(k_warm_count, dim3(w.nbk), dim3(1024), s, nullptr, nullptr, w);
    klaunch(k_warm_done, dim3(1), dim3(1024), s, nullptr, stop, w, h->derr + 7);
}

static WarmBuild warm_build_args(gs_cc_t* h) {
    WarmBuild w;
    w.keys = h->wkeys;
    w.ctl = h->wctl;
    w.cur = reinterpret_cast<uint32_t*>(h->wctl + 1);
    w.part = h->wpart;
    w.keys_cap = 2 * h->warm_sample;
    w.cap = h->warm_bcap;
    w.B = h->hot_bits;
    w.nbk = 1u << (h->hot_bits - kWarmLocalBits);
    w.warm = h->warm;
    w.wb = h->warm_bits;
    w.valid = h->derr + 7;
    return w;
}

// The hot-set / warm-set arguments of a steady-fold launch (k_fold_ring, k_filter), in launch order:
// admission cadence and warm-build schedule follow h->ring_launches. *build: this launch counts the
// warm set's sample (the build kernels follow it on the same stream).
static HotArgs ring_hot_args(gs_cc_t* h, bool* build_out) {
    HotArgs hot{h->hot, h->hot_bits, h->hot_cand};
    hot.sample_edges = kHotSampleEdges;
    hot.budget = h->derr + 6;
    hot.periodic = (h->ring_launches % kHotAdmitEvery == kHotAdmitEvery - 1) ? 1u : 0u;
    ++h->ring_launches;
    hot.five = (h->hot_bits <= kHotBucketBits + 12) ? 1u : 0u;
    hot.thresh = kHotThresh;
    const uint64_t launch_no = h->ring_launches - 1;
    const bool build = h->warm && launch_no >= kWarmAt && (launch_no - kWarmAt) % kWarmEvery == 0;
    hot.warm = h->warm;
    hot.warm_bits = h->warm_bits;
    hot.warm_valid = h->derr + 7;
    hot.wkeys = build ? h->wkeys : nullptr;
    hot.wctl = h->wctl;
    hot.count_edges = build ? h->warm_sample : 0;
    hot.clocks = dbg().ring_clocks ? 1u : 0u;
    *build_out = build;
    return hot;
}

template <typename IdT>
void launch_fold_ring(gs_cc_t* h, const IdT* a, const IdT* b, uint64_t n) {
    ensure_stats(h);
    // admission: while the device budget lasts (cc_kernels.hpp), plus every kHotAdmitEvery-th launch;
    // warm set: counted in this launch, then built (k_warm_part / count / insert), at ring launch
    // kWarmAt after reset and every kWarmEvery-th after it, each time only if the set is not valid
    // for the current giant (device-gated)
    bool build = false;
    const HotArgs hot = ring_hot_args(h, &build);
    FoldArgs f{n, h->parent, h->mark, h->sbits, h->gbits, giant_state(h), RangeCheck{h->cap, h->derr}, h->dstats};
    f.mark_len = h->mark_ctr;
    f.cbits = kUseCbits ? h->cbits : nullptr;
    if (h->hkbits[0]) f.hbits = h->hkbits[h->closes & 1];
    else h->hkbits_ok = false;
    h->ilist_ok = false;
    KTimer t(h, h->fold_timer == GS_K_FOLD ? GS_K_RING : h->fold_timer, n);
    const bool st = h->dstats != nullptr;
    const dim3 grid(grid_for(n / 4, kHotThreads, (unsigned)std::max(h->cus, 1)));
    hipEvent_t stop = build ? nullptr : t.stop();
    hipEvent_t start = t.start();
    if (hot.clocks) {                                // GSGPU_RING_CLOCKS: the instrumented instance
        if (h->mark) klaunch(k_fold_ring<IdT, true, false, true>, grid, dim3(kHotThreads), h->stream, start, stop, a, b, f, hot);
        else klaunch(k_fold_ring<IdT, false, false, true>, grid, dim3(kHotThreads), h->stream, start, stop, a, b, f, hot);
    } else if (h->mark) {
        if (st) klaunch(k_fold_ring<IdT, true, true>, grid, dim3(kHotThreads), h->stream, start, stop, a, b, f, hot);
        else klaunch(k_fold_ring<IdT, true, false>, grid, dim3(kHotThreads), h->stream, start, stop, a, b, f, hot);
    } else {
        if (st) klaunch(k_fold_ring<IdT, false, true>, grid, dim3(kHotThreads), h->stream, start, stop, a, b, f, hot);
        else klaunch(k_fold_ring<IdT, false, false>, grid, dim3(kHotThreads), h->stream, start, stop, a, b, f, hot);
    }
    if (hot.clocks) h->ring_clock_groups = std::min<unsigned>(grid.x, kRingPhaseGroups);
    if (build) launch_warm_build(h, t.stop(), h->stream);
}

// Young-forest split points (dense ids, SoA folds): one internal close at capacity/16 edges since
// reset where gbits outgrows L2 (ids >= 2^kRingMinBits), or at GSGPU_YOUNG_SPLIT
static uint64_t next_young_split(const gs_cc_t* h, uint64_t done) {
    uint64_t s = dbg().young_split;
    if (s == ~0ull) s = 0;                           // production: no split (above)
    return (s && done < s) ? s : 0;
}

int compress_impl(gs_cc_t* h);

// A fold call longer than this many edges (past the young forest) closes internally between
// chunks (compress + giant follow: no emission; labels stay canonical), so the giant filter keeps
// up inside one huge window as it does across windows (one 2^30-edge window: 40.8 ms in one
// launch with the filter frozen at 2^22 edges)
constexpr uint64_t kInternalCloseEdges = 1ull << 24;

static void internal_close(gs_cc_t* h) {
    h->compressed = false;
    (void)compress_impl(h);
    h->compressed = false;
}

// UpdateCC over a batch of dense ids, cut into launches: young-forest launches (up to the young
// limit, cut at the young split point, which closes internally), then mature launches of at most
// kInternalCloseEdges edges with internal closes between them — the ring fold for aligned device
// SoA batches where use_ring() holds, else k_fold. Partial summaries (AOS pairs) fold a short head
// launch first, then the rest in one launch.
template <typename IdT, bool AOS>
int launch_fold_split(gs_cc_t* h, const char* a, const char* b, uint64_t n, size_t esz) {
    // window 1 of the headline stays in k_fold after its young split: the ring fold there (hot set
    // empty, the giant root hooked again and again) took 2.06 ms instead of 1.19 (r02_n)
    const uint64_t young_limit = h->cap / 4;
    const size_t stride = AOS ? 2 * esz : esz;
    const bool aligned = ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0;
    uint64_t off = 0;
    while (off < n) {
        uint64_t m = n - off;
        const bool young = h->edges_since_reset < young_limit;
        if (young) {
            m = std::min(m, young_limit - h->edges_since_reset);
            uint64_t sp = 0;
            if (!AOS && !h->sparse) {
                sp = next_young_split(h, h->edges_since_reset);
                if (sp) m = std::min(m, sp - h->edges_since_reset);
            }
            launch_fold<IdT, AOS>(h, a + off * stride, b ? b + off * esz : nullptr, m, true);
            h->edges_since_reset += m;
            off += m;
            if (sp && h->edges_since_reset == sp && off < n) internal_close(h);
            continue;
        }
        if (AOS) {
            if (off == 0 && n > kMergeBulk) m = std::min(m, kMergeHead);
            launch_fold<IdT, AOS>(h, a + off * stride, nullptr, m, false);
            h->edges_since_reset += m;
            off += m;
            continue;
        }
        m = std::min(m, kInternalCloseEdges);
        if (h->hot && use_ring(h) && aligned && m >= 4) {
            m &= ~(uint64_t)3;                          // the ring fold takes groups of 4 edges
            launch_fold_ring<IdT>(h, reinterpret_cast<const IdT*>(a + off * esz), reinterpret_cast<const IdT*>(b + off * esz), m);
        } else {
            launch_fold<IdT, AOS>(h, a + off * stride, b + off * esz, m, false);
        }
        h->edges_since_reset += m;
        off += m;
        if (off < n && n - off >= 4) internal_close(h);   // (a tail of < 4 edges folds unclosed)
    }
    return GS_OK;
}

SparseArgs sparse_args(gs_cc_t* h) {
    return SparseArgs{h->keys, h->hbits, h->nkeys, h->cfg.vertex_capacity, h->derr};
}

// UpdateCC over arbitrary int64 ids (GS_CC_SPARSE_IDS), young-forest split as for dense ids
// (young sparse folds in launches of kSparseYoungChunk edges: later edges see earlier unions)
constexpr uint64_t kSparseYoungChunk = 1ull << 18;
void launch_fold_sparse(gs_cc_t* h, const int64_t* a, const int64_t* b, uint64_t n, bool aos) {
    const SparseArgs sa = sparse_args(h);
    h->hkbits_ok = false;
    h->ilist_ok = false;
    const uint64_t young_limit = h->cfg.vertex_capacity / 4;
    uint64_t off = 0;
    while (off < n) {
        uint64_t m = n - off;
        if (h->edges_since_reset < young_limit)
            m = std::min(m, std::max<uint64_t>(std::min(kSparseYoungChunk, young_limit - h->edges_since_reset), 1));
        FoldArgs f{m, h->parent, h->mark, h->sbits, h->gbits, giant_state(h), RangeCheck{h->cap, h->derr}, h->dstats};
        f.mark_len = h->mark_ctr;
        const unsigned grid = grid_for((m + 1) / 2, 256, 16384);
        KTimer t(h, h->fold_timer);
        const int64_t* pa = a + (aos ? 2 * off : off);
        const int64_t* pb = aos ? nullptr : b + off;
        if (aos) {
            if (h->mark) klaunch(k_fold_sparse<true, true>, dim3(grid), dim3(256), h->stream, t.start(), t.stop(), pa, pb, f, sa);
            else klaunch(k_fold_sparse<true, false>, dim3(grid), dim3(256), h->stream, t.start(), t.stop(), pa, pb, f, sa);
        } else {
            if (h->mark) klaunch(k_fold_sparse<false, true>, dim3(grid), dim3(256), h->stream, t.start(), t.stop(), pa, pb, f, sa);
            else klaunch(k_fold_sparse<false, false>, dim3(grid), dim3(256), h->stream, t.start(), t.stop(), pa, pb, f, sa);
        }
        h->edges_since_reset += m;
        off += m;
    }
}

int launch_fold_any(gs_cc_t* h, const void* a, const void* b, uint64_t n, bool aos, uint32_t id_bits) {
    if (h->sparse) {
        launch_fold_sparse(h, static_cast<const int64_t*>(a), static_cast<const int64_t*>(b), n, aos);
        return GS_OK;
    }
    const char* ca = static_cast<const char*>(a);
    const char* cb = static_cast<const char*>(b);
    if (id_bits == 32) {
        if (aos) return launch_fold_split<uint32_t, true>(h, ca, nullptr, n, 4);
        return launch_fold_split<uint32_t, false>(h, ca, cb, n, 4);
    }
    if (aos) return launch_fold_split<int64_t, true>(h, ca, nullptr, n, 8);
    return launch_fold_split<int64_t, false>(h, ca, cb, n, 8);
}

// host-buffer folds: edges per staging chunk (one window of the headline workload)
constexpr uint64_t kStagingEdges = 1ull << 24;

// dev_known: 1 = the caller has checked that both buffers are device memory (gs_cc_fold_windows,
// once per call: two pointer-attribute queries per window are ~2-4 us of host time, the order of
// a small window's GPU time), -1 = query here
int fold_impl(gs_cc_t* h, const void* a, const void* b, uint64_t n, bool aos, uint32_t id_bits, int dev_known = -1) {
    GS_TRY(check(h));
    if (n == 0) return GS_OK;
    if (!a || (!aos && !b)) return fail(GS_ERR_INVALID, "fold: null edge buffer");
    DeviceGuard g(h->device);
    if (h->sparse && id_bits != 64) return fail(GS_ERR_UNSUPPORTED, "fold: a sparse-id summary takes 64-bit ids");
    const size_t esz = id_bits / 8;
    const bool dev = dev_known >= 0 ? dev_known != 0 : (is_device_pointer(a) && (aos || is_device_pointer(b)));
    h->compressed = false;
    h->minkey_valid = false;
    if (dev) {
        GS_TRY(launch_fold_any(h, a, b, n, aos, id_bits));
        GS_HIP(hipGetLastError());
        return GS_OK;
    }
    // host buffers (pinned: DMA at the PCIe rate; pageable: through the runtime's bounce buffers):
    // double-buffered staging. Chunk i is copied into slot i & 1 on the copy stream while chunk
    // i - 1 folds on the handle's stream; a slot is refilled only after the fold that read it.
    const uint64_t chunk = h->cfg.staging_edges ? h->cfg.staging_edges : kStagingEdges;
    GS_TRY(ensure_buf(&h->stage, &h->stage_bytes, (size_t)chunk * esz * 4));
    if (!h->copy) {
        GS_HIP(hipStreamCreateWithFlags(&h->copy, hipStreamNonBlocking));
        for (int k = 0; k < 2; ++k) {
            GS_HIP(hipEventCreateWithFlags(&h->staged[k], hipEventDisableTiming));
            GS_HIP(hipEventCreateWithFlags(&h->freed[k], hipEventDisableTiming));
        }
    }
    GS_HIP(hipEventRecord(h->freed[0], h->stream));      // folds queued before this call may still read
    GS_HIP(hipEventRecord(h->freed[1], h->stream));      // the slots
    uint64_t i = 0;
    for (uint64_t off = 0; off < n; off += chunk, ++i) {
        const uint64_t m = (n - off < chunk) ? (n - off) : chunk;
        const int k = (int)(i & 1);
        char* s0 = static_cast<char*>(h->stage) + (size_t)k * chunk * esz * 2;
        char* s1 = s0 + (size_t)chunk * esz;
        GS_HIP(hipStreamWaitEvent(h->copy, h->freed[k], 0));
        if (aos) {
            GS_HIP(hipMemcpyAsync(s0, static_cast<const char*>(a) + off * esz * 2, m * esz * 2, hipMemcpyHostToDevice, h->copy));
        } else {
            GS_HIP(hipMemcpyAsync(s0, static_cast<const char*>(a) + off * esz, m * esz, hipMemcpyHostToDevice, h->copy));
            GS_HIP(hipMemcpyAsync(s1, static_cast<const char*>(b) + off * esz, m * esz, hipMemcpyHostToDevice, h->copy));
        }
        GS_HIP(hipEventRecord(h->staged[k], h->copy));
        GS_HIP(hipStreamWaitEvent(h->stream, h->staged[k], 0));
        GS_TRY(launch_fold_any(h, s0, s1, m, aos, id_bits));
        GS_HIP(hipGetLastError());
        GS_HIP(hipEventRecord(h->freed[k], h->stream));
    }
    return GS_OK;
}

void report_fold_stats(gs_cc_t* h) {
    if (!h->dstats) return;
    unsigned long long c[8];
    if (hipMemcpyAsync(c, h->dstats, sizeof(c), hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
        hipStreamSynchronize(h->stream) != hipSuccess) return;
    fprintf(stderr, "[gsgpu fold-stats] valid=%llu filtered=%llu early=%llu hooks=%llu casfail=%llu inits=%llu hot_hits=%llu warm_hits=%llu\n",
            c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
    (void)hipMemsetAsync(h->dstats, 0, sizeof(c), h->stream);
}

void report_ring_clocks(gs_cc_t* h) {
    const unsigned ng = h->ring_clock_groups;
    h->ring_clock_groups = 0;
    if (!ng) return;
    // the last ring launch's phases, in wall_clock64 ticks (100 MHz) relative to the first entry:
    // entry skew, hot-set fill, main loop, final flush (medians and maxima over workgroups)
    std::vector<unsigned long long> ph(4ull * ng);
    if (hipStreamSynchronize(h->stream) != hipSuccess ||
        hipMemcpyFromSymbol(ph.data(), HIP_SYMBOL(g_ring_phase), ph.size() * 8, 0, hipMemcpyDeviceToHost) != hipSuccess) return;
    unsigned long long t0 = ~0ull, tend = 0;
    std::vector<double> d[4];
    for (unsigned g = 0; g < ng; ++g) t0 = std::min(t0, ph[4 * g]);
    for (unsigned g = 0; g < ng; ++g) {
        const unsigned long long* p = &ph[4 * g];
        tend = std::max(tend, p[3]);
        d[0].push_back((p[0] - t0) * 0.01);
        d[1].push_back((p[1] - p[0]) * 0.01);
        d[2].push_back((p[2] - p[1]) * 0.01);
        d[3].push_back((p[3] - p[2]) * 0.01);
    }
    for (auto& x : d) std::sort(x.begin(), x.end());
    fprintf(stderr, "[gsgpu ring-clocks] groups=%u span=%.2fus entry(med/max)=%.2f/%.2f fill=%.2f/%.2f loop=%.2f/%.2f final=%.2f/%.2f\n",
            ng, (tend - t0) * 0.01, d[0][ng / 2], d[0][ng - 1], d[1][ng / 2], d[1][ng - 1], d[2][ng / 2], d[2][ng - 1],
            d[3][ng / 2], d[3][ng - 1]);
    // per XCD (workgroups are dispatched round-robin over the 8 XCDs): mean / max end time
    if (dbg().ring_clocks > 1) {
        double sum[8] = {0}, mx[8] = {0};
        unsigned cntx[8] = {0};
        for (unsigned g = 0; g < ng; ++g) {
            const double e = (ph[4 * g + 3] - t0) * 0.01;
            sum[g & 7] += e; mx[g & 7] = std::max(mx[g & 7], e); ++cntx[g & 7];
        }
        fprintf(stderr, "[gsgpu ring-xcd]");
        for (int x = 0; x < 8; ++x) fprintf(stderr, " %.1f/%.1f", cntx[x] ? sum[x] / cntx[x] : 0.0, mx[x]);
        fprintf(stderr, "\n");
    }
}

constexpr uint64_t kEarlyPicks = 4;
constexpr uint64_t kPickMinEdges = 1ull << 22;

int compress_impl(gs_cc_t* h) {
    report_fold_stats(h);
    report_ring_clocks(h);
    if (h->compressed) return GS_OK;
    {
        KTimer t(h, GS_K_COMPRESS, h->cap);
        // re-sample the giant every kPickEvery closes (and, while there may be none yet, before
        // each of the first kEarlyPicks closes); otherwise k_compress follows it itself. (Early
        // picks before the first 16 closes cost 66 us per RMAT-26 step in no-op launches: r02_az.)
        // small windows: at most one forced re-pick per kPickMinEdges folded edges (config 5's
        // 2^16-edge windows re-picked every 16th close spent ~9 us per pick, 4.5 % of the step;
        // a pick only aims the filter, any giant is correct)
        const bool force = h->closes % kPickEvery == 0 &&
                           (h->closes == 0 || h->edges_since_reset - h->pick_edges >= kPickMinEdges);
        const bool pick = force || h->closes < kEarlyPicks;
        if (force) h->pick_edges = h->edges_since_reset;
        ListClose lc;
        unsigned grid = grid_for(h->cap, 1024, kCompressGrid);
        if (h->lctl) {
            const uint64_t c = h->closes;
            lc.ctl = h->lctl;
            lc.ngl_in = h->ngl[c & 1];
            lc.ngl_out = h->ngl[(c + 1) & 1];
            lc.ngl_sub = h->ngl_sub;
            lc.tlog = h->tlog[c & 1];
            lc.nslots = h->ilist_slots;
            lc.c3 = (uint32_t)(c % 3);
            lc.n3 = (uint32_t)((c + 1) % 3);
            lc.z3 = (uint32_t)((c + 2) % 3);
            lc.unlogged = (!h->ilist_ok || h->dbits) ? 1u : 0u;
            lc.list_next = (h->ilist_ok && h->ilist_folds > 0 && !h->dbits && dbg().list_close) ? 1u : 0u;
            grid = (grid + kListSub - 1) / kListSub * kListSub;      // whole sets of list workgroups
        }
        h->ilist_ok = true;
        h->ilist_folds = 0;
        h->ilist_slots = 0;
        uint32_t* in = giant_state(h);
        const uint32_t* samp_in = h->psamp + (h->closes & 1) * kPickSamples;
        uint32_t* samp_out = h->psamp + ((h->closes + 1) & 1) * kPickSamples;
        if (pick)
            klaunch(k_pick_giant, dim3(1), dim3(1024), h->stream, t.start(), nullptr, (const uint32_t*)h->parent, h->cap,
                    in, (int)force);
        ++h->closes;
        // (the close about to run is number closes - 1 now: it reads the marks of its parity)
        const uint32_t* hb_in = (h->hkbits[0] && h->hkbits_ok) ? h->hkbits[(h->closes - 1) & 1] : nullptr;
        uint32_t* hb_next = h->hkbits[0] ? h->hkbits[h->closes & 1] : nullptr;
        // k_compress_list while lists are in use: the last close built an NGL (this one may be a list
        // close) or this one builds one. Its control words are stale after plain closes: cleared
        // (LVALID 0, counts 0) when it starts again
        const bool lists = lc.ctl && (h->list_prev || lc.list_next);
        h->list_prev = lc.list_next != 0;
        if (lists) {
            if (!h->list_kernel) GS_HIP(hipMemsetAsync(h->lctl, 0, ListCtl::kWords * sizeof(uint32_t), h->stream));
            klaunch(k_compress_list, dim3(grid), dim3(256), h->stream, pick ? nullptr : t.start(), t.stop(),
                    h->parent, h->cap, h->gbits, h->sbits, (const uint32_t*)in, giant_state(h), h->derr + 5, h->hot,
                    (int)h->sbits_stale, kUseCbits ? h->cbits : nullptr, h->dbits, samp_in, samp_out, hb_in, hb_next, lc);
        } else {
            klaunch(k_compress, dim3(grid_for(h->cap, 1024, kCompressGrid)), dim3(256), h->stream, pick ? nullptr : t.start(),
                    t.stop(), h->parent, h->cap, h->gbits, h->sbits, (const uint32_t*)in, giant_state(h), h->derr + 5,
                    h->hot, (int)h->sbits_stale, kUseCbits ? h->cbits : nullptr, h->dbits, samp_in, samp_out, hb_in, hb_next);
        }
        h->list_kernel = lists;
        h->sbits_stale = false;
        h->hkbits_ok = true;
    }
    GS_HIP(hipGetLastError());
    h->compressed = true;
    return GS_OK;
}

// sparse ids: close the window, then minkey[root] = minimum id of every component
int ensure_minkey(gs_cc_t* h) {
    GS_TRY(compress_impl(h));
    if (h->minkey_valid) return GS_OK;
    const SparseArgs sa = sparse_args(h);
    const dim3 grid(grid_for(h->cap, 256, 16384));
    hipLaunchKernelGGL(k_minkey_init, grid, dim3(256), 0, h->stream, (const uint32_t*)h->parent, h->cap, sa, h->minkey);
    hipLaunchKernelGGL(k_minkey_reduce, grid, dim3(256), 0, h->stream, (const uint32_t*)h->parent, h->cap, sa,
                       (const uint32_t*)(giant_state(h) + 1), h->minkey);
    GS_HIP(hipGetLastError());
    h->minkey_valid = true;
    return GS_OK;
}

int stats_impl(gs_cc_t* h, bool checksum, uint64_t* nv, uint64_t* nc, uint64_t* sum) {
    if (h->sparse && checksum) {
        GS_TRY(ensure_minkey(h));
        GS_HIP(hipMemsetAsync(h->dscratch, 0, 3 * sizeof(unsigned long long), h->stream));
        hipLaunchKernelGGL(k_stats_sparse, dim3(grid_for(h->cap, 256, 4096)), dim3(256), 0, h->stream,
                           (const uint32_t*)h->parent, h->cap, sparse_args(h), (const int64_t*)h->minkey, h->dscratch);
        GS_HIP(hipGetLastError());
        GS_HIP(hipMemcpyAsync(h->hscratch, h->dscratch, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream));
        GS_TRY(sync_and_check(h));
        if (nv) *nv = h->hscratch[0];
        if (nc) *nc = h->hscratch[1];
        if (sum) *sum = h->hscratch[2];
        return GS_OK;
    }
    GS_HIP(hipMemsetAsync(h->dscratch, 0, 3 * sizeof(unsigned long long), h->stream));
    const dim3 grid(grid_for(h->cap, 256, 4096));
    if (checksum) hipLaunchKernelGGL(k_stats<true>, grid, dim3(256), 0, h->stream, h->parent, h->cap, h->dscratch);
    else hipLaunchKernelGGL(k_stats<false>, grid, dim3(256), 0, h->stream, h->parent, h->cap, h->dscratch);
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(h->hscratch, h->dscratch, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream));
    GS_TRY(sync_and_check(h));
    if (nv) *nv = h->hscratch[0];
    if (nc) *nc = h->hscratch[1];
    if (sum) *sum = h->hscratch[2];
    return GS_OK;
}

// copy n bytes of device data to dst (device or host)
int copy_out(gs_cc_t* h, void* dst, const void* src, size_t n) {
    GS_HIP(hipMemcpyAsync(dst, src, n, is_device_pointer(dst) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, h->stream));
    return GS_OK;
}

int emit_pairs_sparse(gs_cc_t* h, void* vertices, void* labels, uint64_t cap, uint64_t* n_out) {
    GS_TRY(ensure_minkey(h));
    uint64_t nv = 0;
    GS_TRY(stats_impl(h, false, &nv, nullptr, nullptr));
    *n_out = nv;
    const uint64_t w = nv < cap ? nv : cap;
    if (nv) {
        // tmp: [counter][keys in][labels in][keys out][labels out][radix-sort temp]
        size_t sort_bytes = 0;
        GS_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const int64_t*)nullptr, (int64_t*)nullptr,
                                                   (const int64_t*)nullptr, (int64_t*)nullptr, (int)nv, 0, 64, h->stream));
        const size_t arr = ((nv * 8) + 255) & ~(size_t)255;
        GS_TRY(ensure_buf(&h->tmp, &h->tmp_bytes, 256 + 4 * arr + sort_bytes));
        char* base = static_cast<char*>(h->tmp);
        auto* counter = reinterpret_cast<unsigned long long*>(base);
        auto* ki = reinterpret_cast<int64_t*>(base + 256);
        auto* li = reinterpret_cast<int64_t*>(base + 256 + arr);
        auto* ko = reinterpret_cast<int64_t*>(base + 256 + 2 * arr);
        auto* lo = reinterpret_cast<int64_t*>(base + 256 + 3 * arr);
        void* st = base + 256 + 4 * arr;
        GS_HIP(hipMemsetAsync(counter, 0, 8, h->stream));
        hipLaunchKernelGGL(k_emit_sparse, dim3(grid_for(h->cap, 256, 16384)), dim3(256), 0, h->stream,
                           (const uint32_t*)h->parent, h->cap, sparse_args(h), (const int64_t*)h->minkey, ki, li, counter);
        GS_HIP(hipGetLastError());
        GS_HIP(hipcub::DeviceRadixSort::SortPairs(st, sort_bytes, (const int64_t*)ki, ko, (const int64_t*)li, lo, (int)nv,
                                                   0, 64, h->stream));
        if (w) {
            GS_TRY(copy_out(h, vertices, ko, w * 8));
            GS_TRY(copy_out(h, labels, lo, w * 8));
        }
    }
    GS_TRY(sync_and_check(h));
    if (nv > cap) return fail(GS_ERR_CAPACITY, "gs_cc_emit_pairs: %llu pairs, capacity %llu",
                              (unsigned long long)nv, (unsigned long long)cap);
    return GS_OK;
}

int find_sparse(gs_cc_t* h, const int64_t* ids, int64_t* roots, uint8_t* found, uint64_t n) {
    GS_TRY(ensure_minkey(h));
    const bool dev = is_device_pointer(ids) && is_device_pointer(roots) && (!found || is_device_pointer(found));
    const int64_t* di = ids;
    int64_t* dr = roots;
    uint8_t* df = found;
    if (!dev) {
        GS_TRY(ensure_buf(&h->tmp, &h->tmp_bytes, 2 * n * 8 + n));
        di = static_cast<const int64_t*>(h->tmp);
        dr = static_cast<int64_t*>(h->tmp) + n;
        df = found ? reinterpret_cast<uint8_t*>(static_cast<int64_t*>(h->tmp) + 2 * n) : nullptr;
        GS_HIP(hipMemcpyAsync(const_cast<int64_t*>(di), ids, n * 8,
                              is_device_pointer(ids) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, h->stream));
    }
    hipLaunchKernelGGL(k_find_sparse, dim3(grid_for(n, 256, 16384)), dim3(256), 0, h->stream, di, dr, df, n,
                       (const uint32_t*)h->parent, sparse_args(h), (const int64_t*)h->minkey);
    GS_HIP(hipGetLastError());
    if (!dev) {
        GS_TRY(copy_out(h, roots, dr, n * 8));
        if (found) GS_TRY(copy_out(h, found, df, n));
    }
    return sync_and_check(h);
}

}  // namespace

namespace gsgpu {
// internal accessors for comm.hip (cc_internal.hpp)
int cc_info(gs_cc_t* h, CcInfo* out) {
    GS_TRY(check(h));
    *out = CcInfo{h->cap, h->device, h->stream, h->mark_buf != nullptr, h->sparse, h->mark != nullptr, h->reset_gen,
                  h->cfg.id_bits};
    return GS_OK;
}
static int export_launch(gs_cc_t* h, void* out, uint64_t cap, unsigned long long* counter, uint64_t expect = ~0ull);
// Fold the slots of a speculative all-gather (comm.hip): every slot but `skip`, pairs up to
// min(count, cap) read on the device; marking is off for these folds (the others' deltas are theirs
// to export). Big slots (young windows: components not yet joined) fold a short head of every
// slot first (see kMergeHead), then the rest.
int cc_fold_slots(gs_cc_t* h, const uint32_t* slots, uint64_t slot_words, int nslots, int skip, uint64_t cap,
                  const uint64_t* caps) {
    GS_TRY(check(h));
    DeviceGuard g(h->device);
    if (nslots <= 1 || cap == 0) return GS_OK;
    SlotCaps sc;
    if (caps) {
        if (nslots > kMaxSlotCaps) return fail(GS_ERR_INVALID, "cc_fold_slots: %d slots with capacities (at most %d)", nslots, kMaxSlotCaps);
        sc.n = (uint32_t)nslots;
        for (int q = 0; q < nslots; ++q) sc.v[q] = caps[q];
    }
    h->compressed = false;
    h->minkey_valid = false;
    FoldArgs f{0, h->parent, nullptr, h->sbits, h->gbits, giant_state(h), RangeCheck{h->cap, h->derr}, nullptr};
    f.combine = dbg().pair_combine ? 1u : 0u;        // (combine_hooks)
    f.halve = dbg().pair_halve;
    KTimer t(h, GS_K_MERGE);
    h->hkbits_ok = false;
    h->ilist_ok = false;
    if (h->sparse) {                                 // (id, id) int64 pairs, hashed to slots
        const dim3 grid(grid_for(cap, 256, (unsigned)std::max(64, 4096 / nslots)), (unsigned)nslots);
        klaunch(k_fold_slots_sparse, grid, dim3(256), h->stream, t.start(), t.stop(), slots, slot_words, skip, (uint64_t)0,
                cap, f, sparse_args(h), sc);
        GS_HIP(hipGetLastError());
        return GS_OK;
    }
    const uint64_t head = cap > kMergeBulk ? std::min<uint64_t>(cap, kMergeHead) : 0;
    if (head) {
        const dim3 grid(grid_for(head, 256, 64), (unsigned)nslots);
        klaunch(k_fold_slots, grid, dim3(256), h->stream, t.start(), nullptr, slots, slot_words, skip, (uint64_t)0, head, f, sc);
    }
    const dim3 grid(grid_for(cap - head, 256, (unsigned)std::max(64, 4096 / nslots)), (unsigned)nslots);
    klaunch(k_fold_slots, grid, dim3(256), h->stream, head ? nullptr : t.start(), t.stop(), slots, slot_words, skip, head, cap, f, sc);
    GS_HIP(hipGetLastError());
    return GS_OK;
}
void cc_count_folded(gs_cc_t* h, uint64_t n) { h->edges_since_reset += n; }

// Partition pre-filter (comm.hip GS_MERGE_PREFILTER senders, gs_cc_filter_edges): the survivors of
// the SoA edges (a[i], b[i]), i < n, against this handle's giant filter, appended as (u, v) uint32
// pairs to out (cap pairs) behind the u64 count word *dcount, which is zeroed first. Launches of at
// most kFilterChunk edges, each workgroup's survivors staged in its region of h->fscratch.
constexpr uint64_t kFilterChunk = 1ull << 24;     // 2^22 cost 156 vs ~110 us per 9.4M-edge slice (launch ramps)
int cc_filter_async(gs_cc_t* h, const void* a, const void* b, uint64_t n, void* out, uint64_t cap,
                    unsigned long long* dcount) {
    GS_TRY(check(h));
    if (h->sparse) return fail(GS_ERR_UNSUPPORTED, "partition pre-filter: dense ids only");
    if (n > cap) return fail(GS_ERR_CAPACITY, "partition pre-filter: %llu edges, room for %llu survivors",
                             (unsigned long long)n, (unsigned long long)cap);
    DeviceGuard g(h->device);
    GS_HIP(hipMemsetAsync(dcount, 0, sizeof(unsigned long long), h->stream));
    if (n == 0) return GS_OK;
    const unsigned grid = grid_for((std::min(n, kFilterChunk) + 3) / 4, kHotThreads, (unsigned)std::max(h->cus, 1));
    const uint64_t stride = (uint64_t)grid * kHotThreads;                       // groups per round
    // edges per workgroup of the largest launch (the first): its rounds x 4096
    const uint64_t region = (((std::min(n, kFilterChunk) + 3) / 4 + stride - 1) / stride) * (uint64_t)kHotThreads * 4;
    const size_t need = (size_t)grid * region * sizeof(uint2);
    if (h->fscratch_bytes < need) {
        if (h->fscratch) {
            GS_HIP(hipStreamSynchronize(h->stream));
            GS_HIP(hipFree(h->fscratch));
            h->fscratch = nullptr;
            h->fscratch_bytes = 0;
        }
        if (hipMalloc(&h->fscratch, need) != hipSuccess) {
            (void)hipGetLastError();
            return fail(GS_ERR_NOMEM, "partition pre-filter scratch of %zu bytes", need);
        }
        h->fscratch_bytes = need;
    }
    const size_t esz = h->cfg.id_bits / 8;
    const bool hot_on = h->hot && use_ring(h);
    uint2* o = static_cast<uint2*>(out);
    if (!is_device_pointer(a) || !is_device_pointer(b)) {
        // host edges: staged through a device copy of the batch (the pre-filter reads device memory)
        const size_t bytes = (size_t)n * esz;
        if (h->fstage_bytes < 2 * bytes) {
            if (h->fstage) {
                GS_HIP(hipStreamSynchronize(h->stream));
                GS_HIP(hipFree(h->fstage));
                h->fstage = nullptr;
                h->fstage_bytes = 0;
            }
            if (hipMalloc(&h->fstage, 2 * bytes) != hipSuccess) {
                (void)hipGetLastError();
                return fail(GS_ERR_NOMEM, "partition pre-filter staging of %zu bytes", 2 * bytes);
            }
            h->fstage_bytes = 2 * bytes;
        }
        char* da = static_cast<char*>(h->fstage);
        GS_HIP(hipMemcpyAsync(da, a, bytes, hipMemcpyHostToDevice, h->stream));
        GS_HIP(hipMemcpyAsync(da + bytes, b, bytes, hipMemcpyHostToDevice, h->stream));
        a = da;
        b = da + bytes;
    }
    for (uint64_t off = 0; off < n; off += kFilterChunk) {
        const uint64_t m = std::min(kFilterChunk, n - off);
        const char* pa = static_cast<const char*>(a) + off * esz;
        const char* pb = static_cast<const char*>(b) + off * esz;
        const int aligned = ((reinterpret_cast<uintptr_t>(pa) | reinterpret_cast<uintptr_t>(pb)) & 15) == 0;
        FoldArgs f{m, h->parent, nullptr, nullptr, h->gbits, giant_state(h), RangeCheck{h->cap, h->derr}, nullptr};
        bool build = false;
        HotArgs hot{};
        if (hot_on) hot = ring_hot_args(h, &build);
        const dim3 gd(grid_for((m + 3) / 4, kHotThreads, (unsigned)std::max(h->cus, 1)));
        KTimer t(h, GS_K_RING, m);
        hipEvent_t stop = build ? nullptr : t.stop();
#define GS_LAUNCH_FILTER(IDT, HOTV)                                                                                \
    klaunch(k_filter_out<IDT, HOTV>, gd, dim3(kHotThreads), h->stream, t.start(), stop, (const IDT*)pa, (const IDT*)pb, \
            f, hot, h->fscratch, region, o, dcount, aligned)
        if (h->cfg.id_bits == 32) { if (hot_on) GS_LAUNCH_FILTER(uint32_t, true); else GS_LAUNCH_FILTER(uint32_t, false); }
        else { if (hot_on) GS_LAUNCH_FILTER(int64_t, true); else GS_LAUNCH_FILTER(int64_t, false); }
#undef GS_LAUNCH_FILTER
        GS_HIP(hipGetLastError());
        if (build) launch_warm_build(h, t.stop(), h->stream);
    }
    return GS_OK;
}

int cc_fold_pairs_any(gs_cc_t* h, const void* pairs, uint64_t n) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));
    h->fold_timer = GS_K_MERGE;
    const int rc = fold_impl(h, pairs, nullptr, n, true, h->sparse ? 64 : 32);
    h->fold_timer = GS_K_FOLD;
    return rc;
}

int cc_filter_state(gs_cc_t* h, uint32_t** gbits, uint64_t* gbits_bytes, uint32_t** giant_words) {
    GS_TRY(check(h));
    if (h->sparse || !h->gbits) return fail(GS_ERR_UNSUPPORTED, "giant filter state: dense ids only");
    *gbits = h->gbits;
    *gbits_bytes = (((uint64_t)h->cap + 31) >> 5) * 4;
    *giant_words = giant_state(h);
    return GS_OK;
}

int cc_install_giant(gs_cc_t* h, const uint32_t* words) {
    GS_TRY(check(h));
    DeviceGuard g(h->device);
    hipLaunchKernelGGL(k_install_giant, dim3(1), dim3(1024), 0, h->stream, words, giant_state(h), h->derr + 5,
                       (h->hot && use_ring(h)) ? h->hot : nullptr);
    GS_HIP(hipGetLastError());
    return GS_OK;
}

void* cc_ingest_get(gs_cc_t* h) { return h->ingest; }
void cc_ingest_set(gs_cc_t* h, void* p, void (*free_fn)(void*)) {
    if (h->ingest && h->ingest_free && h->ingest != p) h->ingest_free(h->ingest);
    h->ingest = p;
    h->ingest_free = free_fn;
}

void cc_set_settle(gs_cc_t* h, int (*fn)(void*), void* ctx) {
    h->settle_fn = fn;
    h->settle_ctx = ctx;
}

int cc_settle(gs_cc_t* h) {
    if (!h || !h->settle_fn) return GS_OK;
    int (*fn)(void*) = h->settle_fn;
    void* ctx = h->settle_ctx;
    h->settle_fn = nullptr;                          // the settle itself folds and closes
    h->settle_ctx = nullptr;
    return fn(ctx);
}

int cc_export_async(gs_cc_t* h, void* pairs, uint64_t cap, unsigned long long* dcount, uint64_t expect) {
    GS_TRY(check(h));
    if (!h->mark_buf) return fail(GS_ERR_UNSUPPORTED, "export: no marks on this handle");
    // (cap may be smaller than the log: the pending tail stays for the next export; the count word
    // receives the whole pending number, so the caller can tell)
    DeviceGuard g(h->device);
    return export_launch(h, pairs, cap, dcount, expect);
}
}  // namespace gsgpu

extern "C" {

int gs_version(void) { return GSGPU_VERSION; }
const char* gs_last_error(void) { return last_error().c_str(); }

int gs_cc_create(gs_cc_t** out, const gs_cc_config* cfg) {
    if (!out || !cfg) return fail(GS_ERR_INVALID, "gs_cc_create: null argument");
    *out = nullptr;
    if (cfg->struct_size != sizeof(gs_cc_config))
        return fail(GS_ERR_INVALID, "gs_cc_create: struct_size %u != %zu", cfg->struct_size, sizeof(gs_cc_config));
    if (cfg->id_bits != 32 && cfg->id_bits != 64) return fail(GS_ERR_INVALID, "gs_cc_create: id_bits must be 32 or 64");
    const bool sparse = (cfg->flags & GS_CC_SPARSE_IDS) != 0;
    if (sparse && cfg->id_bits != 64) return fail(GS_ERR_INVALID, "gs_cc_create: GS_CC_SPARSE_IDS needs id_bits 64");
    if (sparse && (cfg->vertex_capacity == 0 || cfg->vertex_capacity > (1ull << 30)))
        return fail(GS_ERR_INVALID, "gs_cc_create: sparse vertex_capacity must be in [1, 2^30]");
    if (cfg->vertex_capacity == 0 || cfg->vertex_capacity > 0xFFFFFFFFull)
        return fail(GS_ERR_INVALID, "gs_cc_create: vertex_capacity must be in [1, 2^32-1]");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return fail(GS_ERR_HIP, "gs_cc_create: no HIP device available");
    }
    if (cfg->device < 0 || cfg->device >= ndev) return fail(GS_ERR_INVALID, "gs_cc_create: device %d of %d", cfg->device, ndev);
    DeviceGuard g(cfg->device);
    if (!g.ok) return fail(GS_ERR_HIP, "gs_cc_create: hipSetDevice(%d) failed", cfg->device);
    gs_cc_t* h = new gs_cc_t();
    h->cfg = *cfg;
    h->cap = (uint32_t)cfg->vertex_capacity;
    h->device = cfg->device;
    if (sparse) {                        // slots: 2^hbits >= 2 x capacity, + the INT64_MIN slot
        h->sparse = true;
        h->hbits = 4;
        while ((1ull << h->hbits) < 2 * cfg->vertex_capacity) ++h->hbits;
        h->cap = (1u << h->hbits) + 1;
    }
    auto bail = [&](int rc) { gs_cc_destroy(h); return rc; };
    if (hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking) != hipSuccess) return bail(fail(GS_ERR_HIP, "hipStreamCreate failed"));
    h->stream = h->own;
    if (hipMalloc(&h->parent, (size_t)h->cap * sizeof(uint32_t)) != hipSuccess) { (void)hipGetLastError(); return bail(fail(GS_ERR_NOMEM, "parent[%u] allocation failed", h->cap)); }
    if (cfg->flags & GS_CC_TRACK_MARKS) {
        if (hipMalloc(&h->mark_buf, (size_t)h->cap * 2 * sizeof(uint32_t)) != hipSuccess) { (void)hipGetLastError(); return bail(fail(GS_ERR_NOMEM, "hook log allocation failed")); }
        if (hipMalloc(&h->mark_ctr, 128) != hipSuccess) { (void)hipGetLastError(); return bail(fail(GS_ERR_NOMEM, "hook log counter allocation failed")); }
        h->mark = h->mark_buf;
    }
    if (hipMalloc(&h->gbits, mark_bytes(h->cap)) != hipSuccess || hipMalloc(&h->sbits, mark_bytes(h->cap)) != hipSuccess ||
        hipMalloc(&h->cbits, mark_bytes(h->cap)) != hipSuccess ||
        hipMalloc(&h->derr, kDerrBytes) != hipSuccess || hipMalloc(&h->psamp, 2 * kPickSamples * sizeof(uint32_t)) != hipSuccess || hipMalloc(&h->dscratch, 8 * sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc(&h->hscratch, 8 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return bail(fail(GS_ERR_NOMEM, "scratch allocation failed"));
    }
    std::memset(h->hscratch, 0, 8 * sizeof(unsigned long long));
    if (!sparse && (hipMalloc(&h->hkbits[0], mark_bytes(h->cap)) != hipSuccess ||
                    hipMalloc(&h->hkbits[1], mark_bytes(h->cap)) != hipSuccess)) {
        (void)hipGetLastError();
        return bail(fail(GS_ERR_NOMEM, "hooked-root bitmaps allocation failed"));
    }
    if (!sparse) {
        // NGL: up to capacity/64 vertices outside the giant (more: bitmap closes); touch log:
        // kTlogSlots slots per interval
        h->ngl_sub = (uint32_t)std::min<uint64_t>(4096, std::max<uint64_t>(64, (uint64_t)h->cap / 64 / kListSub));
        if (hipMalloc(&h->lctl, ListCtl::kWords * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&h->ngl[0], (size_t)kListSub * h->ngl_sub * sizeof(uint2)) != hipSuccess ||
            hipMalloc(&h->ngl[1], (size_t)kListSub * h->ngl_sub * sizeof(uint2)) != hipSuccess ||
            hipMalloc(&h->tlog[0], (size_t)kTlogSlots * kSlotWords * 4) != hipSuccess ||
            hipMalloc(&h->tlog[1], (size_t)kTlogSlots * kSlotWords * 4) != hipSuccess) {
            (void)hipGetLastError();
            return bail(fail(GS_ERR_NOMEM, "list-close buffers allocation failed"));
        }
    }
    if (sparse && (hipMalloc(&h->keys, sizeof(int64_t) << h->hbits) != hipSuccess ||
                   hipMalloc(&h->minkey, sizeof(int64_t) * (size_t)h->cap) != hipSuccess ||
                   hipMalloc(&h->nkeys, sizeof(unsigned long long)) != hipSuccess)) {
        (void)hipGetLastError();
        return bail(fail(GS_ERR_NOMEM, "sparse id table (2^%u slots) allocation failed", h->hbits));
    }
    if (hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, cfg->device) != hipSuccess) h->cus = 0;
    {
        uint32_t bits = 0;
        while (bits < 32 && (1ull << bits) < (uint64_t)h->cap) ++bits;
        if (!sparse && bits >= 20 && bits <= kHotBucketBits + 15) {     // remainders fit 15 bits (+1 in 16)
            if (hipMalloc(&h->hot, kHotBuckets * sizeof(uint2)) != hipSuccess ||
                hipMalloc(&h->hot_cand, sizeof(uint32_t) << kHotCandBits) != hipSuccess) {
                (void)hipGetLastError();
                if (h->hot) (void)hipFree(h->hot);
                if (h->hot_cand) (void)hipFree(h->hot_cand);
                h->hot = nullptr;
                h->hot_cand = nullptr;
            }
            h->hot_bits = bits;
            // warm set: only where gbits outgrows an XCD's 4 MiB L2 (with the ring fold), its table
            // L2-resident and at most 1/8 of gbits (8-bit slots need at least 2^(B-8) buckets)
            h->warm_bits = std::min<uint32_t>(kWarmBucketsMaxBits, bits - 6);
            if (h->hot && bits >= dbg().ring_min_bits && bits <= h->warm_bits + 8 && bits >= kWarmLocalBits &&
                bits - kWarmLocalBits <= 13 && bits - h->warm_bits <= kWarmLocalBits) {
                h->warm_sample = std::min<uint64_t>(kWarmSample, h->cap / 8);
                const uint32_t nbk = 1u << (bits - kWarmLocalBits);
                h->warm_sample = (h->warm_sample + 255) / 256 * 256;        // whole wave steps
                const uint64_t keys = 2 * h->warm_sample;
                h->warm_bcap = (uint32_t)((keys / nbk + keys / nbk / 2 + 1024 + 7) & ~7ull);  // 1.5 x the mean bucket
                const size_t ctl = sizeof(unsigned long long) + (size_t)nbk * 4;
                if (hipMalloc(&h->warm, (size_t)4 << h->warm_bits) != hipSuccess ||
                    hipMalloc(&h->wkeys, keys * 4) != hipSuccess ||
                    hipMalloc(&h->wpart, (size_t)nbk * h->warm_bcap * 2) != hipSuccess ||
                    hipMalloc(&h->wctl, ctl) != hipSuccess || hipMemsetAsync(h->wctl, 0, ctl, h->stream) != hipSuccess) {
                    (void)hipGetLastError();
                    if (h->warm) (void)hipFree(h->warm);
                    if (h->wkeys) (void)hipFree(h->wkeys);
                    if (h->wpart) (void)hipFree(h->wpart);
                    if (h->wctl) (void)hipFree(h->wctl);
                    h->warm = nullptr;
                    h->wkeys = nullptr;
                    h->wpart = nullptr;
                    h->wctl = nullptr;
                }
            }
        }
    }
    if (hipMemsetAsync(h->derr, 0, kDerrBytes, h->stream) != hipSuccess) return bail(fail(GS_ERR_HIP, "memset failed"));
    int rc = gs_cc_reset(h);
    if (rc != GS_OK) return bail(rc);
    if (hipStreamSynchronize(h->stream) != hipSuccess) return bail(fail(GS_ERR_HIP, "stream sync failed"));
    *out = h;
    return GS_OK;
}

int gs_cc_destroy(gs_cc_t* h) {
    if (!h) return GS_OK;
    (void)cc_settle(h);                          // peers may wait for this rank in a tail round
    DeviceGuard g(h->device);
    if (h->own) (void)hipStreamSynchronize(h->own);
    if (h->stream && h->stream != h->own) (void)hipStreamSynchronize(h->stream);
    for (auto& p : h->pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto e : h->pool) (void)hipEventDestroy(e);
    if (h->parent) (void)hipFree(h->parent);
    if (h->mark_buf) (void)hipFree(h->mark_buf);
    if (h->mark_ctr) (void)hipFree(h->mark_ctr);
    if (h->derr) (void)hipFree(h->derr);
    if (h->psamp) (void)hipFree(h->psamp);
    if (h->gbits) (void)hipFree(h->gbits);
    if (h->sbits) (void)hipFree(h->sbits);
    if (h->cbits) (void)hipFree(h->cbits);
    for (auto* hb : h->hkbits) if (hb) (void)hipFree(hb);
    if (h->lctl) (void)hipFree(h->lctl);
    for (auto* q : h->ngl) if (q) (void)hipFree(q);
    for (auto* q : h->tlog) if (q) (void)hipFree(q);
    if (h->dbits) (void)hipFree(h->dbits);
    if (h->elab) (void)hipFree(h->elab);
    if (h->dstats) (void)hipFree(h->dstats);
    if (h->fscratch) (void)hipFree(h->fscratch);
    if (h->fstage) (void)hipFree(h->fstage);
    if (h->hot) (void)hipFree(h->hot);
    if (h->hot_cand) (void)hipFree(h->hot_cand);
    if (h->warm) (void)hipFree(h->warm);
    if (h->wkeys) (void)hipFree(h->wkeys);
    if (h->wpart) (void)hipFree(h->wpart);
    if (h->wctl) (void)hipFree(h->wctl);
    if (h->keys) (void)hipFree(h->keys);
    if (h->minkey) (void)hipFree(h->minkey);
    if (h->nkeys) (void)hipFree(h->nkeys);
    if (h->dscratch) (void)hipFree(h->dscratch);
    if (h->hscratch) (void)hipHostFree(h->hscratch);
    if (h->stage) (void)hipFree(h->stage);
    if (h->copy) (void)hipStreamSynchronize(h->copy);
    for (int k = 0; k < 2; ++k) {
        if (h->staged[k]) (void)hipEventDestroy(h->staged[k]);
        if (h->freed[k]) (void)hipEventDestroy(h->freed[k]);
    }
    if (h->copy) (void)hipStreamDestroy(h->copy);
    if (h->estream) (void)hipStreamSynchronize(h->estream);
    for (auto& s : h->eslot) {
        if (s.mem) (void)hipFree(s.mem);
        if (s.staged) (void)hipEventDestroy(s.staged);
        if (s.done) (void)hipEventDestroy(s.done);
    }
    if (h->ecount) (void)hipHostFree(h->ecount);
    if (h->estream) (void)hipStreamDestroy(h->estream);
    if (h->tmp) (void)hipFree(h->tmp);
    if (h->ingest && h->ingest_free) h->ingest_free(h->ingest);
    if (h->own) (void)hipStreamDestroy(h->own);
    delete h;
    return GS_OK;
}

int gs_cc_reset(gs_cc_t* h) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));                      // a pending multi-GPU window first (comm.hip)
    DeviceGuard g(h->device);
    GS_HIP(hipMemsetAsync(h->parent, 0xFF, (size_t)h->cap * sizeof(uint32_t), h->stream));
    if (h->mark_ctr) GS_HIP(hipMemsetAsync(h->mark_ctr, 0, 3 * sizeof(unsigned long long), h->stream));
    GS_HIP(hipMemsetAsync(h->gbits, 0, mark_bytes(h->cap), h->stream));
    GS_HIP(hipMemsetAsync(h->sbits, 0, mark_bytes(h->cap), h->stream));
    GS_HIP(hipMemsetAsync(h->cbits, 0, mark_bytes(h->cap), h->stream));
    for (auto* hb : h->hkbits) if (hb) GS_HIP(hipMemsetAsync(hb, 0, mark_bytes(h->cap), h->stream));
    h->hkbits_ok = true;
    h->list_prev = false;
    h->list_kernel = false;
    if (h->lctl) GS_HIP(hipMemsetAsync(h->lctl, 0, ListCtl::kWords * sizeof(uint32_t), h->stream));
    h->ilist_ok = true;
    h->ilist_folds = 0;
    h->ilist_slots = 0;
    if (h->elab) {                       // a new stream: the next delta is the whole emission
        GS_HIP(hipMemsetAsync(h->elab, 0xFF, (size_t)h->cap * 4, h->stream));
        GS_HIP(hipMemsetAsync(h->dbits, 0, mark_bytes(h->cap), h->stream));
    }
    // giant state (cc_kernels.hpp, giant_state()): both slots no giant / gbits built for none,
    // hot set owner none
    GS_HIP(hipMemsetAsync(h->derr + 1, 0xFF, 5 * sizeof(uint32_t), h->stream));
    {
        static const uint32_t budget = kHotAdmitLaunches;   // derr[6]
        GS_HIP(hipMemcpyAsync(h->derr + 6, &budget, sizeof(uint32_t), hipMemcpyHostToDevice, h->stream));
    }
    GS_HIP(hipMemsetAsync(h->derr + 7, 0, sizeof(uint32_t), h->stream));      // warm set: not built
    GS_HIP(hipMemsetAsync(h->psamp, 0xFF, 2 * kPickSamples * sizeof(uint32_t), h->stream));   // no samples yet
    if (h->hot) GS_HIP(hipMemsetAsync(h->hot, 0, kHotBuckets * sizeof(uint2), h->stream));
    if (h->hot_cand) GS_HIP(hipMemsetAsync(h->hot_cand, 0xFF, sizeof(uint32_t) << kHotCandBits, h->stream));
    if (h->sparse) {
        hipLaunchKernelGGL(k_fill64, dim3(grid_for(1ull << h->hbits, 256, 4096)), dim3(256), 0, h->stream, h->keys,
                           (uint64_t)1 << h->hbits, kEmptyKey);
        GS_HIP(hipGetLastError());
        GS_HIP(hipMemsetAsync(h->nkeys, 0, sizeof(unsigned long long), h->stream));
    }
    h->compressed = true;
    h->sbits_stale = false;
    h->minkey_valid = false;
    h->edges_since_reset = 0;
    h->closes = 0;
    h->pick_edges = 0;
    h->ring_launches = 0;
    ++h->reset_gen;
    return GS_OK;
}

int gs_cc_set_stream(gs_cc_t* h, void* s) {
    GS_TRY(check(h));
    h->stream = static_cast<hipStream_t>(s);     // NULL = the HIP null stream, like any HIP API
    return GS_OK;
}

int gs_cc_get_stream(gs_cc_t* h, void** s) {
    GS_TRY(check(h));
    if (!s) return fail(GS_ERR_INVALID, "null out");
    *s = h->stream;
    return GS_OK;
}

int gs_cc_sync(gs_cc_t* h) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));                      // a pending multi-GPU window first (comm.hip)
    DeviceGuard g(h->device);
    GS_TRY(sync_and_check(h));
    return gs_cc_emit_wait(h, 0);              // and every async delta emission
}

// A fold settles a pending multi-GPU window first: its tail pairs (foreign unions folded with marking
// paused) must land before this fold's hooks are exported, or not under their roots at all
// (comm.hip merge_allgather). gs_cc_fold_windows folds without it: its merge_window exports the new
// window's hooks BEFORE settling the previous window, so its host never waits per window.
int gs_cc_fold(gs_cc_t* h, const void* src, const void* dst, uint64_t n) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));
    return fold_impl(h, src, dst, n, false, h->cfg.id_bits);
}

int gs_cc_fold_pairs(gs_cc_t* h, const void* pairs, uint64_t n) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));
    return fold_impl(h, pairs, nullptr, n, true, h->cfg.id_bits);
}

int gs_cc_fold_pairs32(gs_cc_t* h, const void* pairs, uint64_t n) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));
    h->fold_timer = GS_K_MERGE;          // a partial summary: timed as CombineCC, not UpdateCC
    const int rc = fold_impl(h, pairs, nullptr, n, true, 32);
    h->fold_timer = GS_K_FOLD;
    return rc;
}

int gs_cc_merge(gs_cc_t* into, gs_cc_t* from) {
    GS_TRY(check(into));
    GS_TRY(check(from));
    GS_TRY(cc_settle(into));
    GS_TRY(cc_settle(from));
    if (into == from) return GS_OK;
    if (into->device != from->device) return fail(GS_ERR_UNSUPPORTED, "gs_cc_merge: summaries on different devices");
    if (into->sparse != from->sparse) return fail(GS_ERR_UNSUPPORTED, "gs_cc_merge: sparse-id and dense-id summaries do not mix");
    if (!into->sparse && from->cap > into->cap)
        return fail(GS_ERR_RANGE, "gs_cc_merge: source capacity %u exceeds target %u", from->cap, into->cap);
    DeviceGuard g(into->device);
    if (from->stream != into->stream) {
        hipEvent_t e = get_event(into);
        GS_HIP(hipEventRecord(e, from->stream));
        GS_HIP(hipStreamWaitEvent(into->stream, e, 0));
        into->pool.push_back(e);
    }
    into->compressed = false;
    into->minkey_valid = false;
    into->hkbits_ok = false;
    into->ilist_ok = false;
    if (into->sparse) {
        KTimer t(into, GS_K_MERGE);
        const dim3 grid(grid_for(from->cap, 256, 16384));
        FoldArgs f{0, into->parent, into->mark, into->sbits, into->gbits, giant_state(into), RangeCheck{into->cap, into->derr}, nullptr};
        f.mark_len = into->mark_ctr;
        if (into->mark) klaunch(k_merge_sparse<true>, grid, dim3(256), into->stream, t.start(), t.stop(), (const uint32_t*)from->parent, sparse_args(from), f, sparse_args(into));
        else klaunch(k_merge_sparse<false>, grid, dim3(256), into->stream, t.start(), t.stop(), (const uint32_t*)from->parent, sparse_args(from), f, sparse_args(into));
    } else {
        KTimer t(into, GS_K_MERGE);
        const dim3 grid(grid_for(from->cap, 256, 16384));
        if (into->mark) klaunch(k_merge_dense<true>, grid, dim3(256), into->stream, t.start(), t.stop(), (const uint32_t*)from->parent, from->cap, into->parent, into->mark, into->mark_ctr, into->sbits);
        else klaunch(k_merge_dense<false>, grid, dim3(256), into->stream, t.start(), t.stop(), (const uint32_t*)from->parent, from->cap, into->parent, into->mark, into->mark_ctr, into->sbits);
    }
    GS_HIP(hipGetLastError());
    if (from->stream != into->stream) {   // `from` must not be reused before the merge read it
        hipEvent_t e = get_event(into);
        GS_HIP(hipEventRecord(e, into->stream));
        GS_HIP(hipStreamWaitEvent(from->stream, e, 0));
        into->pool.push_back(e);
    }
    return GS_OK;
}

int gs_cc_combine(gs_cc_t* s1, gs_cc_t* s2, gs_cc_t** result) {
    GS_TRY(check(s1));
    GS_TRY(check(s2));
    GS_TRY(cc_settle(s1));
    GS_TRY(cc_settle(s2));
    if (!result) return fail(GS_ERR_INVALID, "gs_cc_combine: null result");
    uint64_t c1 = 0, c2 = 0;
    GS_TRY(gs_cc_stats(s1, &c1, nullptr));
    GS_TRY(gs_cc_stats(s2, &c2, nullptr));
    if (c1 <= c2) { GS_TRY(gs_cc_merge(s2, s1)); *result = s2; }
    else { GS_TRY(gs_cc_merge(s1, s2)); *result = s1; }
    return GS_OK;
}

int gs_cc_close_window(gs_cc_t* h) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));                      // a pending multi-GPU window first (comm.hip)
    DeviceGuard g(h->device);
    return compress_impl(h);
}

// The per-window host loop of gs_cc_fold_windows (fold, then close or merge), enqueued on h->stream.
// (Round 5 measured a split of the steady fold here — a read-only giant filter run one window ahead
// on a stream of its own, the ordered unions after it — and removed it: DESIGN.md §4.)
static int fold_windows_loop(gs_cc_t* h, gs_comm_t* comm, int mode, const char* a, const char* b, uint64_t n,
                             uint64_t window_edges, uint64_t* windows_out) {
    const size_t esz = h->cfg.id_bits / 8;
    const int dev = (n && is_device_pointer(a) && is_device_pointer(b)) ? 1 : 0;
    // GS_MERGE_PREFILTER: only the Merger (rank 0) folds; the exchange takes the window's edges.
    // Every window is an exchange, so the ranks first agree on the window count: a rank past its
    // own edges (a short last global window, an empty slice) runs empty windows
    const bool pre = comm && mode == GS_MERGE_PREFILTER;
    const bool fold_here = !pre || cc_comm_rank(comm) == 0;
    uint64_t nw = (n + window_edges - 1) / window_edges;
    if (pre) GS_TRY(cc_agree_windows(h, comm, nw, &nw));
    for (uint64_t w = 0; w < nw; ++w) {
        const uint64_t off = std::min(n, w * window_edges);
        const uint64_t m = std::min(window_edges, n - off);
        if (fold_here) GS_TRY(fold_impl(h, a + off * esz, b + off * esz, m, false, h->cfg.id_bits, dev));   // (no settle: above)
        if (pre) GS_TRY(cc_merge_edges(h, comm, mode, a + off * esz, b + off * esz, m));
        else GS_TRY(comm ? gs_cc_merge_window(h, comm, mode) : gs_cc_close_window(h));
        if (windows_out) *windows_out = w + 1;
    }
    return GS_OK;
}

int gs_cc_fold_windows(gs_cc_t* h, gs_comm_t* comm, int mode, const void* src, const void* dst, uint64_t n,
                       uint64_t window_edges, uint64_t* windows_out) {
    GS_TRY(check(h));
    if (windows_out) *windows_out = 0;
    if (window_edges == 0) return fail(GS_ERR_INVALID, "gs_cc_fold_windows: window_edges must be > 0");
    if (n && (!src || !dst)) return fail(GS_ERR_INVALID, "gs_cc_fold_windows: null edge buffer");
    const char* a = static_cast<const char*>(src);
    const char* b = static_cast<const char*>(dst);
    GS_TRY(fold_windows_loop(h, comm, mode, a, b, n, window_edges, windows_out));
    GS_TRY(cc_settle(h));                            // the last window's exchange verified
    // a pre-filtering sender folds nothing: its filters' range-error flag is reported here
    if (comm && mode == GS_MERGE_PREFILTER && cc_comm_rank(comm) != 0) return sync_and_check(h);
    return GS_OK;
}

int gs_cc_stats(gs_cc_t* h, uint64_t* nv, uint64_t* nc) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));                      // a pending multi-GPU window first (comm.hip)
    DeviceGuard g(h->device);
    return stats_impl(h, false, nv, nc, nullptr);
}

int gs_cc_checksum(gs_cc_t* h, uint64_t* sum, uint64_t* nv, uint64_t* nc) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));                      // a pending multi-GPU window first (comm.hip)
    DeviceGuard g(h->device);
    GS_TRY(compress_impl(h));
    return stats_impl(h, true, nv, nc, sum);
}

int gs_cc_emit_dense(gs_cc_t* h, void* labels, uint64_t n) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));                      // a pending multi-GPU window first (comm.hip)
    if (n && !labels) return fail(GS_ERR_INVALID, "gs_cc_emit_dense: null output");
    if (h->sparse) return fail(GS_ERR_UNSUPPORTED, "gs_cc_emit_dense: sparse-id summary (use gs_cc_emit_pairs)");
    DeviceGuard g(h->device);
    GS_TRY(compress_impl(h));
    const uint64_t m = n < h->cap ? n : h->cap;
    const size_t esz = h->cfg.id_bits / 8;
    if (h->cfg.id_bits == 32) {
        GS_TRY(copy_out(h, labels, h->parent, m * 4));
    } else if (is_device_pointer(labels)) {
        hipLaunchKernelGGL(k_widen, dim3(grid_for(m, 256, 16384)), dim3(256), 0, h->stream, h->parent, (int64_t*)labels, m);
        GS_HIP(hipGetLastError());
    } else {
        GS_TRY(ensure_buf(&h->tmp, &h->tmp_bytes, m * 8 + 8));
        hipLaunchKernelGGL(k_widen, dim3(grid_for(m, 256, 16384)), dim3(256), 0, h->stream, h->parent, (int64_t*)h->tmp, m);
        GS_HIP(hipGetLastError());
        GS_TRY(copy_out(h, labels, h->tmp, m * 8));
    }
    if (n > m) {   // ids beyond the capacity are never in the summary: -1
        char* tail = static_cast<char*>(labels) + m * esz;
        if (is_device_pointer(labels)) GS_HIP(hipMemsetAsync(tail, 0xFF, (n - m) * esz, h->stream));
        else { GS_TRY(sync_and_check(h)); std::memset(tail, 0xFF, (n - m) * esz); }
    }
    return sync_and_check(h);
}

int gs_cc_emit_pairs(gs_cc_t* h, void* vertices, void* labels, uint64_t cap, uint64_t* n_out) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));                      // a pending multi-GPU window first (comm.hip)
    if (!n_out) return fail(GS_ERR_INVALID, "gs_cc_emit_pairs: null n_out");
    if (cap && (!vertices || !labels)) return fail(GS_ERR_INVALID, "gs_cc_emit_pairs: null output");
    DeviceGuard g(h->device);
    if (h->sparse) return emit_pairs_sparse(h, vertices, labels, cap, n_out);
    GS_TRY(compress_impl(h));
    const uint32_t ntiles = (uint32_t)((h->cap + kTile - 1) / kTile);
    const size_t esz = h->cfg.id_bits / 8;
    // layout of tmp: [tile counts u32 x ntiles][offsets u64 x ntiles+1][vertices][labels]
    const size_t cnt_b = ((size_t)ntiles * 4 + 15) & ~(size_t)15;
    const size_t off_b = ((size_t)(ntiles + 1) * 8 + 15) & ~(size_t)15;
    GS_TRY(ensure_buf(&h->tmp, &h->tmp_bytes, cnt_b + off_b));
    uint32_t* cnt = static_cast<uint32_t*>(h->tmp);
    uint64_t* off = reinterpret_cast<uint64_t*>(static_cast<char*>(h->tmp) + cnt_b);
    hipLaunchKernelGGL(k_tile_count, dim3(ntiles), dim3(kTileThreads), 0, h->stream, h->parent, h->cap, cnt);
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, h->stream, cnt, off, ntiles, (unsigned long long*)nullptr);
    GS_HIP(hipGetLastError());
    GS_HIP(hipMemcpyAsync(h->hscratch, off + ntiles, 8, hipMemcpyDeviceToHost, h->stream));
    GS_TRY(sync_and_check(h));
    const uint64_t total = h->hscratch[0];
    *n_out = total;
    const uint64_t w = total < cap ? total : cap;
    if (w) {
        const bool dev = is_device_pointer(vertices) && is_device_pointer(labels);
        void* vo = vertices;
        void* lo = labels;
        if (!dev) {
            GS_TRY(ensure_buf(&h->tmp, &h->tmp_bytes, cnt_b + off_b + 2 * w * esz));
            cnt = static_cast<uint32_t*>(h->tmp);
            off = reinterpret_cast<uint64_t*>(static_cast<char*>(h->tmp) + cnt_b);
            // ensure_buf may have reallocated: recompute the offsets
            hipLaunchKernelGGL(k_tile_count, dim3(ntiles), dim3(kTileThreads), 0, h->stream, h->parent, h->cap, cnt);
            hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, h->stream, cnt, off, ntiles, (unsigned long long*)nullptr);
            vo = static_cast<char*>(h->tmp) + cnt_b + off_b;
            lo = static_cast<char*>(vo) + w * esz;
        }
        if (h->cfg.id_bits == 32)
            hipLaunchKernelGGL(k_tile_scatter<uint32_t>, dim3(ntiles), dim3(kTileThreads), 0, h->stream, h->parent, h->cap, off,
                               (uint32_t*)vo, (uint32_t*)lo, w);
        else
            hipLaunchKernelGGL(k_tile_scatter<int64_t>, dim3(ntiles), dim3(kTileThreads), 0, h->stream, h->parent, h->cap, off,
                               (int64_t*)vo, (int64_t*)lo, w);
        GS_HIP(hipGetLastError());
        if (!dev) {
            GS_HIP(hipMemcpyAsync(vertices, vo, w * esz, hipMemcpyDeviceToHost, h->stream));
            GS_HIP(hipMemcpyAsync(labels, lo, w * esz, hipMemcpyDeviceToHost, h->stream));
        }
    }
    GS_TRY(sync_and_check(h));
    if (total > cap) return fail(GS_ERR_CAPACITY, "gs_cc_emit_pairs: %llu pairs, capacity %llu",
                                 (unsigned long long)total, (unsigned long long)cap);
    return GS_OK;
}

// ---- delta emission ----
static int delta_begin(gs_cc_t* h, const char* who, void* vertices, void* labels, uint64_t cap, uint64_t* n_out) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));                      // a pending multi-GPU window first (comm.hip)
    if (!n_out) return fail(GS_ERR_INVALID, "%s: null n_out", who);
    if (cap && (!vertices || !labels)) return fail(GS_ERR_INVALID, "%s: null output", who);
    if (h->sparse) return fail(GS_ERR_UNSUPPORTED, "%s: sparse-id summary (use gs_cc_emit_pairs)", who);
    if (!h->elab) {                      // first call: every vertex dirty, nothing emitted yet
        DeviceGuard g(h->device);
        if (hipMalloc(&h->elab, (size_t)h->cap * 4) != hipSuccess || hipMalloc(&h->dbits, mark_bytes(h->cap)) != hipSuccess) {
            (void)hipGetLastError();
            if (h->elab) (void)hipFree(h->elab);
            h->elab = nullptr;
            return fail(GS_ERR_NOMEM, "%s: state allocation failed", who);
        }
        GS_HIP(hipMemsetAsync(h->elab, 0xFF, (size_t)h->cap * 4, h->stream));
        GS_HIP(hipMemsetAsync(h->dbits, 0xFF, mark_bytes(h->cap), h->stream));
    }
    return GS_OK;
}

// The delta on h->stream in three launches: k_delta_stage (every tile's changed pairs into its own
// region of the tile staging, h->tmp: counts, offsets, ntiles x kTile pairs), k_tile_scan (offsets;
// the size also to *total_host if given), k_delta_pack (the pairs packed to vo/lo — device
// addresses, cap entries — elab and the dirty words updated, only if the delta fits cap). Returns
// the device word holding the size.
static int delta_enqueue(gs_cc_t* h, uint64_t cap, void* vo, void* lo, unsigned long long* total_host,
                         const uint64_t** total, uint64_t* total_out = nullptr) {
    const uint32_t ntiles = (uint32_t)((h->cap + kTile - 1) / kTile);
    const size_t esz = h->cfg.id_bits / 8;
    const size_t cnt_b = ((size_t)ntiles * 4 + 15) & ~(size_t)15;
    const size_t off_b = ((size_t)(ntiles + 1) * 8 + 15) & ~(size_t)15;
    const size_t tile_pairs = (size_t)ntiles * kTile;
    GS_TRY(ensure_buf(&h->tmp, &h->tmp_bytes, cnt_b + off_b + 2 * tile_pairs * esz));
    uint32_t* cnt = static_cast<uint32_t*>(h->tmp);
    uint64_t* off = reinterpret_cast<uint64_t*>(static_cast<char*>(h->tmp) + cnt_b);
    char* sv = static_cast<char*>(h->tmp) + cnt_b + off_b;
    char* sl = sv + tile_pairs * esz;
#define GS_DELTA(IdT)                                                                                                    \
    hipLaunchKernelGGL(k_delta_stage<IdT>, dim3((ntiles + kDeltaTiles - 1) / kDeltaTiles), dim3(kTileThreads), 0,       \
                       h->stream, (const uint32_t*)h->parent, h->cap, (const uint32_t*)h->elab, (const uint32_t*)h->dbits, \
                       ntiles, cnt, (IdT*)sv, (IdT*)sl);                                                                   \
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, h->stream, cnt, off, ntiles, total_host);                      \
    hipLaunchKernelGGL(k_delta_pack<IdT>, dim3(ntiles), dim3(256), 0, h->stream, (const IdT*)sv, (const IdT*)sl,           \
                       (const uint32_t*)cnt, (const uint64_t*)off, ntiles, cap, h->elab, h->dbits, h->cap, (IdT*)vo, (IdT*)lo, \
                       total_out)
    if (h->cfg.id_bits == 32) { GS_DELTA(uint32_t); } else { GS_DELTA(int64_t); }
#undef GS_DELTA
    GS_HIP(hipGetLastError());
    *total = total_out ? total_out : off + ntiles;
    return GS_OK;
}

// The device's view of an output buffer: device memory as is, pinned host memory (hipHostMalloc,
// hipHostRegister) through its device mapping; nullptr for pageable host memory.
static void* device_view(void* p) {
    hipPointerAttribute_t a;
    if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged || a.isManaged) return p;
    if (a.type == hipMemoryTypeHost && a.devicePointer && a.hostPointer)
        return static_cast<char*>(a.devicePointer) + (static_cast<char*>(p) - static_cast<char*>(a.hostPointer));
    return nullptr;
}

// workgroups of the async copy-out kernel (few: its PCIe writes share the CUs with the next fold)
static unsigned emit_copy_blocks() {
    static const unsigned b = [] {
        const char* e = getenv("GSGPU_EMIT_COPY_BLOCKS");
        const unsigned v = (e && *e) ? (unsigned)strtoul(e, nullptr, 0) : 64u;
        return v ? v : 64u;
    }();
    return b;
}

// packed pairs for host outputs: slot si's buffer, 2 x min(cap, capacity) ids
static int delta_slot(gs_cc_t* h, int si, uint64_t cap, char** sv, char** sl) {
    const size_t esz = h->cfg.id_bits / 8;
    const uint64_t scap = std::min<uint64_t>(cap, h->cap);
    gs_cc::EmitSlot& S = h->eslot[si];
    GS_TRY(ensure_buf(&S.mem, &S.bytes, 16 + 2 * scap * esz));     // [size word | vertices | labels]
    *sv = static_cast<char*>(S.mem) + 16;
    *sl = *sv + scap * esz;
    return GS_OK;
}

// Device outputs: packed in place. Host outputs (pinned or pageable): packed in HBM, the size read
// back, then two DMA copies of exactly the delta.
int gs_cc_emit_delta(gs_cc_t* h, void* vertices, void* labels, uint64_t cap, uint64_t* n_out) {
    GS_TRY(delta_begin(h, "gs_cc_emit_delta", vertices, labels, cap, n_out));
    GS_TRY(gs_cc_emit_wait(h, 0));             // async emissions still pending come first
    DeviceGuard g(h->device);
    GS_TRY(compress_impl(h));
    const size_t esz = h->cfg.id_bits / 8;
    const bool dev = cap == 0 || (is_device_pointer(vertices) && is_device_pointer(labels));
    char *sv = nullptr, *sl = nullptr;
    if (!dev) GS_TRY(delta_slot(h, 0, cap, &sv, &sl));
    const uint64_t* total = nullptr;
    GS_TRY(delta_enqueue(h, cap, dev ? vertices : sv, dev ? labels : sl, nullptr, &total));
    GS_HIP(hipMemcpyAsync(h->hscratch, total, 8, hipMemcpyDeviceToHost, h->stream));
    GS_TRY(sync_and_check(h));
    const uint64_t n = h->hscratch[0];
    *n_out = n;
    if (n > cap) return fail(GS_ERR_CAPACITY, "gs_cc_emit_delta: %llu changed pairs, capacity %llu (nothing consumed)",
                             (unsigned long long)n, (unsigned long long)cap);
    if (!dev && n) {
        GS_HIP(hipMemcpyAsync(vertices, sv, n * esz, hipMemcpyDeviceToHost, h->stream));
        GS_HIP(hipMemcpyAsync(labels, sl, n * esz, hipMemcpyDeviceToHost, h->stream));
        return sync_and_check(h);
    }
    return GS_OK;
}

// Enqueued only: the delta is packed into one of two slots on h->stream (the next fold may follow
// at once) and its size lands in a pinned word; device and pinned buffers are written from the slot
// by k_delta_copy on estream while the next fold runs, pageable ones by DMA in gs_cc_emit_wait.
int gs_cc_emit_delta_async(gs_cc_t* h, void* vertices, void* labels, uint64_t cap, uint64_t* n_out) {
    GS_TRY(delta_begin(h, "gs_cc_emit_delta_async", vertices, labels, cap, n_out));
    if (h->n_epend >= 2) return fail(GS_ERR_INVALID, "gs_cc_emit_delta_async: two emissions pending (gs_cc_emit_wait first)");
    DeviceGuard g(h->device);
    if (!h->estream) {
        GS_HIP(hipStreamCreateWithFlags(&h->estream, hipStreamNonBlocking));
        GS_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->ecount), 2 * sizeof(unsigned long long), hipHostMallocDefault));
        for (auto& s : h->eslot) {
            GS_HIP(hipEventCreateWithFlags(&s.staged, hipEventDisableTiming));
            GS_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        }
    }
    GS_TRY(compress_impl(h));
    const int si = (int)(h->enext & 1u);
    char *sv = nullptr, *sl = nullptr;
    GS_TRY(delta_slot(h, si, cap, &sv, &sl));
    unsigned long long* cdev = nullptr;
    GS_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&cdev), h->ecount, 0));
    const uint64_t* total = nullptr;
    // the size goes to the pinned word from the copy kernel (a host store at the end of the scan
    // cost that kernel ~20 us: the release of a kernel that writes host memory) or, for pageable
    // buffers, by a DMA behind the pack
    GS_TRY(delta_enqueue(h, cap, sv, sl, nullptr, &total, static_cast<uint64_t*>(h->eslot[si].mem)));
    // buffers the device can write: copied out right away, on estream, by a few workgroups (their
    // PCIe writes overlap the next fold); pageable ones: by DMA at the wait
    void* dv = cap ? device_view(vertices) : nullptr;
    void* dl = cap ? device_view(labels) : nullptr;
    const bool kcopy = dv && dl;
    if (!kcopy) GS_HIP(hipMemcpyAsync(h->ecount + si, total, 8, hipMemcpyDeviceToHost, h->stream));
    GS_HIP(hipEventRecord(h->eslot[si].staged, h->stream));
    if (kcopy) {
        GS_HIP(hipStreamWaitEvent(h->estream, h->eslot[si].staged, 0));
        if (h->cfg.id_bits == 32)
            hipLaunchKernelGGL(k_delta_copy<uint32_t>, dim3(emit_copy_blocks()), dim3(256), 0, h->estream, (const uint32_t*)sv,
                               (const uint32_t*)sl, total, cap, (uint32_t*)dv, (uint32_t*)dl, cdev + si);
        else
            hipLaunchKernelGGL(k_delta_copy<int64_t>, dim3(emit_copy_blocks()), dim3(256), 0, h->estream, (const int64_t*)sv,
                               (const int64_t*)sl, total, cap, (int64_t*)dv, (int64_t*)dl, cdev + si);
        GS_HIP(hipGetLastError());
        GS_HIP(hipEventRecord(h->eslot[si].done, h->estream));
    }
    h->epend[h->n_epend++] = gs_cc::EmitPend{si, n_out, cap, vertices, labels, kcopy};
    ++h->enext;
    return GS_OK;
}

int gs_cc_emit_wait(gs_cc_t* h, uint32_t keep) {
    GS_TRY(check(h));
    DeviceGuard g(h->device);
    const size_t esz = h->cfg.id_bits / 8;
    uint64_t over = 0, over_cap = 0;
    while (h->n_epend > (int)keep) {
        const gs_cc::EmitPend p = h->epend[0];
        for (int i = 1; i < h->n_epend; ++i) h->epend[i - 1] = h->epend[i];
        --h->n_epend;
        GS_HIP(hipEventSynchronize(p.kcopy ? h->eslot[p.slot].done : h->eslot[p.slot].staged));
        const uint64_t n = h->ecount[p.slot];
        *p.n_out = n;
        if (n > p.cap) { over = n; over_cap = p.cap; continue; }
        if (n && !p.kcopy) {
            const hipMemcpyKind kind = hipMemcpyDeviceToHost;      // pageable host buffers
            char* sv = static_cast<char*>(h->eslot[p.slot].mem) + 16;       // past the size word
            const uint64_t scap = std::min<uint64_t>(p.cap, h->cap);
            GS_HIP(hipMemcpyAsync(p.vertices, sv, n * esz, kind, h->estream));
            GS_HIP(hipMemcpyAsync(p.labels, sv + scap * esz, n * esz, kind, h->estream));
            GS_HIP(hipStreamSynchronize(h->estream));
        }
    }
    if (over) return fail(GS_ERR_CAPACITY, "gs_cc_emit_delta_async: %llu changed pairs, capacity %llu (nothing consumed)",
                          (unsigned long long)over, (unsigned long long)over_cap);
    return GS_OK;
}

int gs_cc_find(gs_cc_t* h, const void* ids, void* roots, uint64_t n) {
    return gs_cc_find_flags(h, ids, roots, nullptr, n);
}

int gs_cc_find_flags(gs_cc_t* h, const void* ids, void* roots, uint8_t* found, uint64_t n) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));                      // a pending multi-GPU window first (comm.hip)
    if (n == 0) return GS_OK;
    if (!ids || !roots) return fail(GS_ERR_INVALID, "gs_cc_find: null buffer");
    DeviceGuard g(h->device);
    if (h->sparse) return find_sparse(h, static_cast<const int64_t*>(ids), static_cast<int64_t*>(roots), found, n);
    const size_t esz = h->cfg.id_bits / 8;
    const bool dev = is_device_pointer(ids) && is_device_pointer(roots);
    const void* di = ids;
    void* dr = roots;
    if (!dev) {
        GS_TRY(ensure_buf(&h->tmp, &h->tmp_bytes, 2 * n * esz));
        di = h->tmp;
        dr = static_cast<char*>(h->tmp) + n * esz;
        GS_HIP(hipMemcpyAsync(const_cast<void*>(di), ids, n * esz, is_device_pointer(ids) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, h->stream));
    }
    const dim3 grid(grid_for(n, 256, 16384));
    if (h->cfg.id_bits == 32)
        hipLaunchKernelGGL(k_find<uint32_t>, grid, dim3(256), 0, h->stream, (const uint32_t*)di, (uint32_t*)dr, n, h->parent, h->cap);
    else
        hipLaunchKernelGGL(k_find<int64_t>, grid, dim3(256), 0, h->stream, (const int64_t*)di, (int64_t*)dr, n, h->parent, h->cap);
    GS_HIP(hipGetLastError());
    if (!dev) GS_TRY(copy_out(h, roots, dr, n * esz));
    GS_TRY(sync_and_check(h));
    if (found) {                           // dense ids: found <=> label != -1 (ids are < 2^32 - 1)
        const bool host_roots = !is_device_pointer(roots);
        if (host_roots && !is_device_pointer(found)) {
            for (uint64_t i = 0; i < n; ++i)
                found[i] = esz == 4 ? (static_cast<const uint32_t*>(roots)[i] != 0xFFFFFFFFu)
                                    : (static_cast<const int64_t*>(roots)[i] >= 0);
        } else {
            return fail(GS_ERR_UNSUPPORTED, "gs_cc_find_flags: found flags for device buffers need a sparse-id summary");
        }
    }
    return GS_OK;
}

int gs_cc_labels_device(gs_cc_t* h, const void** p) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));                      // a pending multi-GPU window first (comm.hip)
    if (!p) return fail(GS_ERR_INVALID, "null out");
    if (h->sparse) return fail(GS_ERR_UNSUPPORTED, "gs_cc_labels_device: sparse-id summary (labels are per slot)");
    *p = h->parent;
    return GS_OK;
}

int gsgpu::export_launch(gs_cc_t* h, void* out, uint64_t cap, unsigned long long* counter, uint64_t expect) {
    // the pending hook-log entries -> (v, root(v)) pairs; the count is on the device, so the grid
    // follows the caller's expectation (the exchange: twice its last delta), strided past it: a
    // steady window's few thousand hooks need a few workgroups, a young one's millions up to 1024.
    // (Every workgroup counts itself once on one word to let the last one advance the cursor:
    // 1024 of them cost ~11 us per export, r03_xchg2.)
    {
        const unsigned grid = expect == ~0ull ? 1024u : (unsigned)std::min<uint64_t>(std::max<uint64_t>((expect + 255) / 256, 8), 1024);
        KTimer t(h, GS_K_EXPORT);
        if (h->sparse)                               // (id, root id) as int64 pairs
            klaunch(k_export_log_sparse, dim3(grid), dim3(256), h->stream, t.start(), t.stop(), (const uint32_t*)h->mark_buf,
                    h->mark_ctr, (const uint32_t*)h->parent, sparse_args(h), (int64_t*)out, cap, counter);
        else
            klaunch(k_export_log, dim3(grid), dim3(256), h->stream, t.start(), t.stop(), (const uint32_t*)h->mark_buf,
                    h->mark_ctr, (const uint32_t*)h->parent, (uint32_t*)out, cap, counter);
    }
    GS_HIP(hipGetLastError());
    return GS_OK;
}

static int export_check(gs_cc_t* h, const char* fn) {
    if (!h->mark_buf) return fail(GS_ERR_UNSUPPORTED, "%s: handle created without GS_CC_TRACK_MARKS", fn);
    return GS_OK;
}
// bytes per exported pair: (uint32 vertex, uint32 root) dense, (int64 id, int64 root id) sparse
static size_t pair_bytes(const gs_cc_t* h) { return h->sparse ? 16 : 8; }

int gs_cc_export_marks(gs_cc_t* h, void* pairs, uint64_t cap, uint64_t* n_out) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));                      // a pending multi-GPU window first (comm.hip)
    if (!n_out) return fail(GS_ERR_INVALID, "gs_cc_export_marks: null n_out");
    GS_TRY(export_check(h, "gs_cc_export_marks"));
    if (cap && !pairs) return fail(GS_ERR_INVALID, "gs_cc_export_marks: null output");
    DeviceGuard g(h->device);
    const bool dev = cap == 0 || is_device_pointer(pairs);
    void* out = pairs;
    if (!dev) {
        GS_TRY(ensure_buf(&h->tmp, &h->tmp_bytes, cap * pair_bytes(h)));
        out = h->tmp;
    }
    GS_TRY(export_launch(h, out, cap, h->dscratch));
    GS_HIP(hipMemcpyAsync(h->hscratch, h->dscratch, 8, hipMemcpyDeviceToHost, h->stream));
    GS_TRY(sync_and_check(h));
    const uint64_t total = h->hscratch[0];
    *n_out = total < cap ? total : cap;
    if (!dev && *n_out) {
        GS_HIP(hipMemcpyAsync(pairs, out, *n_out * pair_bytes(h), hipMemcpyDeviceToHost, h->stream));
        GS_TRY(sync_and_check(h));
    }
    if (total > cap) return fail(GS_ERR_CAPACITY, "gs_cc_export_marks: %llu marked, capacity %llu (rest kept)",
                                 (unsigned long long)total, (unsigned long long)cap);
    return GS_OK;
}

int gs_cc_export_marks_async(gs_cc_t* h, void* pairs, uint64_t cap, void* dev_count) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));                      // a pending multi-GPU window first (comm.hip)
    GS_TRY(export_check(h, "gs_cc_export_marks_async"));
    if (!dev_count || !is_device_pointer(dev_count) || (cap && (!pairs || !is_device_pointer(pairs))))
        return fail(GS_ERR_INVALID, "gs_cc_export_marks_async: pairs and dev_count must be device pointers");
    if (cap < 2ull * h->cap) return fail(GS_ERR_CAPACITY, "gs_cc_export_marks_async: capacity %llu < 2 x vertex capacity %u",
                                         (unsigned long long)cap, h->cap);
    DeviceGuard g(h->device);
    return export_launch(h, pairs, cap, static_cast<unsigned long long*>(dev_count));
}

int gs_cc_filter_edges(gs_cc_t* h, const void* src, const void* dst, uint64_t n, void* pairs, uint64_t cap,
                       uint64_t* n_out) {
    GS_TRY(check(h));
    GS_TRY(cc_settle(h));
    if (!n_out || (n && (!src || !dst || !pairs))) return fail(GS_ERR_INVALID, "gs_cc_filter_edges: null argument");
    if (n && !is_device_pointer(pairs)) return fail(GS_ERR_INVALID, "gs_cc_filter_edges: pairs must be device memory");
    *n_out = 0;
    DeviceGuard g(h->device);
    unsigned long long* dcount = reinterpret_cast<unsigned long long*>(h->dscratch);
    GS_TRY(cc_filter_async(h, src, dst, n, pairs, cap, dcount));
    uint64_t* hc = reinterpret_cast<uint64_t*>(h->hscratch + 5);
    GS_HIP(hipMemcpyAsync(hc, dcount, sizeof(uint64_t), hipMemcpyDeviceToHost, h->stream));
    GS_TRY(sync_and_check(h));
    *n_out = *hc;
    return GS_OK;
}

int gs_cc_set_marking(gs_cc_t* h, int on) {
    GS_TRY(check(h));
    if (!h->mark_buf) return on ? fail(GS_ERR_UNSUPPORTED, "gs_cc_set_marking: handle created without GS_CC_TRACK_MARKS") : GS_OK;
    h->mark = on ? h->mark_buf : nullptr;
    return GS_OK;
}

int gs_cc_timing(gs_cc_t* h, int enable) {
    GS_TRY(check(h));
    DeviceGuard g(h->device);
    GS_TRY(resolve_timing(h));
    h->timing = enable != 0;
    h->timing_mask = (enable & GS_TIMING_MASK) ? ((uint32_t)enable & 0xFFu) : ~0u;
    if (h->timing_mask & (1u << GS_K_FOLD)) h->timing_mask |= (1u << GS_K_RING);   // "fold" = every launch kind
    for (int k = 0; k < GS_K_COUNT; ++k) { h->total_ms[k] = 0; h->launches[k] = 0; h->units[k] = 0; }
    return GS_OK;
}

int gs_cc_kernel_time(gs_cc_t* h, int kernel, double* total_ms, uint64_t* launches) {
    GS_TRY(check(h));
    if (kernel < 0 || kernel >= GS_K_COUNT) return fail(GS_ERR_INVALID, "bad kernel id %d", kernel);
    DeviceGuard g(h->device);
    GS_TRY(resolve_timing(h));
    if (total_ms) *total_ms = h->total_ms[kernel];
    if (launches) *launches = h->launches[kernel];
    return GS_OK;
}

int gs_cc_kernel_units(gs_cc_t* h, int kernel, uint64_t* units) {
    GS_TRY(check(h));
    if (kernel < 0 || kernel >= GS_K_COUNT) return fail(GS_ERR_INVALID, "bad kernel id %d", kernel);
    if (!units) return fail(GS_ERR_INVALID, "null out");
    DeviceGuard g(h->device);
    GS_TRY(resolve_timing(h));
    *units = h->units[kernel];
    return GS_OK;
}

}  // extern "C"
