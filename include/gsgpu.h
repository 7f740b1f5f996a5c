/*
 * gsgpu.h — C ABI of libgsgpu.so: MI355X (gfx950) streaming Connected Components for the
 * Gelly Streaming `ConnectedComponents` SummaryBulkAggregation hot path.
 *
 * Reference interfaces replaced (paths relative to the reference's
 * src/main/java/org/apache/flink/graph/streaming/):
 *
 *   gs_cc_create / gs_cc_reset   new DisjointSet<K>() as the fold's initial value
 *                                (library/ConnectedComponents.java:52-54, summaries/DisjointSet.java:31-34)
 *   gs_cc_fold / gs_cc_fold_pairs  EdgesFold.foldEdges -> UpdateCC: ds.union(u, v) per edge
 *                                (EdgesFold.java:47, library/ConnectedComponents.java:83-85,
 *                                 summaries/DisjointSet.java:92-118, SummaryBulkAggregation.java:121-123)
 *   gs_cc_merge                  DisjointSet.merge(other)  (summaries/DisjointSet.java:127-131)
 *   gs_cc_combine                CombineCC.reduce(s1, s2): merge the smaller summary into the larger
 *                                (library/ConnectedComponents.java:116-125)
 *   gs_cc_close_window           the Merger step that emits the cumulative summary per window
 *                                (SummaryAggregation.java:106-119; transientState=false)
 *   gs_cc_find                   DisjointSet.find (summaries/DisjointSet.java:66-80; -1 = null)
 *   gs_cc_stats                  getMatches().size() and the number of components
 *                                (summaries/DisjointSet.java:44-46)
 *   gs_cc_emit_dense / _pairs    the emitted summary as canonical (vertex, min-id) labels:
 *                                what getMatches()+find() give FlattenSet
 *                                (example/ConnectedComponentsExample.java:143-156) and toString
 *                                groups by (summaries/DisjointSet.java:133-150), canonicalised
 *   gs_cc_export_marks           the partial summary that crosses the windowAll / tree exchange
 *                                (SummaryBulkAggregation.java:81, SummaryTreeReduce.java:95-123)
 *
 * Conventions: every function returns 0 (GS_OK) or a negative GS_ERR_* code; the message of the
 * last failure on the calling thread is gs_last_error(). No C++ exception crosses the ABI.
 * Buffers passed in may be host (pageable or pinned) or device pointers; the caller keeps
 * ownership of them, the library owns all device state of a handle. Input buffers of a fold must
 * stay unchanged until the handle's stream has run it (gs_cc_sync): host edges are copied
 * asynchronously (double-buffered staging, gs_cc_config.staging_edges per chunk). One handle per subtask
 * thread; calls on one handle must be serialised by the caller; different handles may be used
 * concurrently. All work of a handle is ordered on its HIP stream (gs_cc_set_stream).
 */
#ifndef GSGPU_H
#define GSGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSGPU_VERSION 2

enum {
    GS_OK = 0,
    GS_ERR_INVALID = -1,      /* bad argument                                           */
    GS_ERR_HIP = -2,          /* HIP runtime failure                                    */
    GS_ERR_RANGE = -3,        /* a vertex id outside [0, vertex_capacity)               */
    GS_ERR_NOMEM = -4,        /* device allocation failed                               */
    GS_ERR_STATE = -5,        /* call not valid in the handle's current state           */
    GS_ERR_UNSUPPORTED = -6,  /* feature not built / not enabled on this handle         */
    GS_ERR_CAPACITY = -7,     /* output buffer too small                                */
    GS_ERR_COMM = -8          /* collective / communicator failure (RCCL)               */
};

/* gs_cc_config.flags */
enum {
    GS_CC_TRACK_MARKS = 1u << 0, /* keep per-vertex marks of this window's hooks, needed by
                                    gs_cc_export_marks (multi-GPU / multi-handle merge)    */
    GS_CC_SPARSE_IDS = 1u << 1   /* id_bits 64 only: ids are ANY 64-bit values (Java long,
                                    negatives included), hashed to slots on the device;
                                    vertex_capacity = most distinct ids (<= 2^30). Canonical
                                    labels are still the minimum id of each component.
                                    gs_cc_emit_dense, gs_cc_emit_delta and
                                    gs_cc_labels_device are not available in this mode; with
                                    GS_CC_TRACK_MARKS the exchange carries int64 pairs.      */
};

typedef struct gs_cc gs_cc_t;

typedef struct gs_cc_config {
    uint32_t struct_size;       /* sizeof(gs_cc_config)                                    */
    uint32_t id_bits;           /* 32 (int/uint32 ids) or 64 (long ids, the reference's K=Long) */
    uint64_t vertex_capacity;   /* ids must lie in [0, vertex_capacity); <= 2^32 - 1
                                   (GS_CC_SPARSE_IDS: the number of distinct ids, <= 2^30)   */
    int32_t  device;            /* HIP device ordinal                                      */
    uint32_t flags;             /* GS_CC_*                                                 */
    uint64_t staging_edges;     /* staging chunk of host-pointer folds, 2 slots (0 = 2^24) */
} gs_cc_config;

/* ---- lifetime ---- */
int gs_cc_create(gs_cc_t** out, const gs_cc_config* cfg);
int gs_cc_destroy(gs_cc_t* h);
int gs_cc_reset(gs_cc_t* h);                        /* back to an empty DisjointSet          */
/* Orders all later work of the handle on hip_stream (NULL = the HIP null stream). A new handle
 * runs on a non-blocking stream of its own; set the caller's stream before folding device buffers
 * the caller produced on it. */
int gs_cc_set_stream(gs_cc_t* h, void* hip_stream);
int gs_cc_get_stream(gs_cc_t* h, void** hip_stream);
int gs_cc_sync(gs_cc_t* h);                         /* wait for the handle's stream; reports
                                                       deferred device errors (GS_ERR_RANGE) */

/* ---- UpdateCC / DisjointSet.union over a batch ----
 * src/dst: n ids each (id_bits wide). pairs: n interleaved (src, dst) ids. Duplicates and
 * self-loops are allowed: union(u,u) makes u a singleton (DisjointSet.java:94-105). */
int gs_cc_fold(gs_cc_t* h, const void* src, const void* dst, uint64_t n);
int gs_cc_fold_pairs(gs_cc_t* h, const void* pairs, uint64_t n);

/* ---- DisjointSet.merge / CombineCC ---- (both handles on one device) */
int gs_cc_merge(gs_cc_t* into, gs_cc_t* from);
/* CombineCC.reduce(s1, s2): if |s1| <= |s2| then s2.merge(s1), *result = s2; else s1.merge(s2),
 * *result = s1 (sizes = getMatches().size()). */
int gs_cc_combine(gs_cc_t* s1, gs_cc_t* s2, gs_cc_t** result);

/* ---- Merger / emission ----
 * close_window fully compresses the summary: afterwards every seen vertex's label is the
 * minimum vertex id of its component, resident on the device (gs_cc_labels_device). */
int gs_cc_close_window(gs_cc_t* h);
int gs_cc_stats(gs_cc_t* h, uint64_t* n_vertices, uint64_t* n_components);
/* labels[v] for v < n: canonical label of v, or -1 if v is not in the summary.
 * Output element width = id_bits. Implies close_window. */
int gs_cc_emit_dense(gs_cc_t* h, void* labels, uint64_t n);
/* (vertex, label) pairs of every vertex in the summary, sorted by vertex.
 * Writes min(cap, |V|) pairs, *n_out = |V|; GS_ERR_CAPACITY if cap < |V|. Implies close_window. */
int gs_cc_emit_pairs(gs_cc_t* h, void* vertices, void* labels, uint64_t cap, uint64_t* n_out);
/* Per-window DELTA of the emission (what a host-side Merger / FlattenSet consumer needs to keep its
 * copy of the cumulative summary, SummaryAggregation.java:110-111, ConnectedComponentsExample.java:
 * 143-156, at O(changes) PCIe cost): the (vertex, label) pairs, sorted by vertex, of every vertex
 * that is new or whose canonical label changed since the previous gs_cc_emit_delta call (the first
 * call, and the first after gs_cc_reset, returns the whole emission). Writes the pairs if they fit:
 * *n_out = their number; if cap < *n_out, GS_ERR_CAPACITY and NOTHING is consumed (call again with
 * a bigger buffer). Applying every delta in order to a map reproduces gs_cc_emit_pairs. Output
 * element width = id_bits; vertices/labels host or device. Dense ids only. Implies close_window. */
int gs_cc_emit_delta(gs_cc_t* h, void* vertices, void* labels, uint64_t cap, uint64_t* n_out);
/* gs_cc_emit_delta, enqueued only (the per-window Merger emission without a host wait): the delta is
 * computed on the handle's stream into one of two device slots — the next fold can be enqueued at
 * once — and its size into a pinned word. gs_cc_emit_wait copies it to vertices/labels (device or
 * host memory; pinned host memory copies at full PCIe rate) while the GPU runs whatever was enqueued
 * after it; the buffers and *n_out are valid once gs_cc_emit_wait has returned that emission. An
 * emission that did not fit cap consumed nothing (*n_out = its size, gs_cc_emit_wait returns
 * GS_ERR_CAPACITY) and its pairs stay in the next delta. At most two emissions pending per handle;
 * gs_cc_emit_delta waits for pending ones first. */
int gs_cc_emit_delta_async(gs_cc_t* h, void* vertices, void* labels, uint64_t cap, uint64_t* n_out);
/* Waits for async delta emissions, oldest first, until at most `keep` are pending (0: all; also done
 * by gs_cc_sync), writing their *n_out. GS_ERR_CAPACITY if one of them did not fit its cap. */
int gs_cc_emit_wait(gs_cc_t* h, uint32_t keep);
/* Order-independent checksum of the canonical emission (definition shared with oracle/:
 * sum over seen v of splitmix64(v ^ splitmix64(label ^ 0xD1B54A32D192ED03))). Implies close_window. */
int gs_cc_checksum(gs_cc_t* h, uint64_t* checksum, uint64_t* n_vertices, uint64_t* n_components);
/* DisjointSet.find for n ids: roots[i] = current root of ids[i], -1 if unknown (null).
 * The root is the canonical label (roots are always component minima). */
int gs_cc_find(gs_cc_t* h, const void* ids, void* roots, uint64_t n);
/* as gs_cc_find, and found[i] = 1 if ids[i] is in the summary, 0 if not (null) — needed where -1
 * is itself a valid id (GS_CC_SPARSE_IDS). found may be NULL. Implies close_window. */
int gs_cc_find_flags(gs_cc_t* h, const void* ids, void* roots, uint8_t* found, uint64_t n);
/* device pointer to the uint32 label/parent array (length vertex_capacity, 0xFFFFFFFF = unseen). */
int gs_cc_labels_device(gs_cc_t* h, const void** dev_ptr);

/* ---- partial-summary exchange (windowAll / tree merge) ----
 * Requires GS_CC_TRACK_MARKS. Writes the (vertex, root) pairs (uint32, interleaved; with
 * GS_CC_SPARSE_IDS (id, id of the root's component) as int64, interleaved, 16 B per pair) of
 * every vertex whose root status changed in this handle since the last export (roots it hooked,
 * singletons made by self-loops: the handle's hook log, at most 2 x vertex_capacity entries), and
 * consumes them; pairs past cap stay for the next export. Folding these pairs into another
 * summary (gs_cc_fold_pairs, 32-bit ids regardless of id_bits via gs_cc_fold_pairs32) transfers
 * all connectivity this handle gained. */
int gs_cc_export_marks(gs_cc_t* h, void* pairs, uint64_t cap, uint64_t* n_out);
int gs_cc_fold_pairs32(gs_cc_t* h, const void* pairs, uint64_t n);
/* as gs_cc_export_marks, but only enqueued on the handle's stream: the pair count lands in the
 * device uint64 *dev_count (no host synchronisation; a collective can take it from there).
 * pairs and dev_count are device pointers; cap must be >= 2 x vertex_capacity (never overflows). */
int gs_cc_export_marks_async(gs_cc_t* h, void* pairs, uint64_t cap, void* dev_count);
/* The giant pre-filter alone (UpdateCC's read-only half; what a GS_MERGE_PREFILTER sender runs):
 * the edges (src[i], dst[i]), i < n (id_bits wide, host or device), that survive this handle's
 * giant filter — NOT both endpoints in the giant component it last picked — written as uint32
 * (u, v) pairs to the device buffer pairs (cap >= n pairs); *n_out = their number (synchronous).
 * Nothing is folded. Dense ids only. Out-of-range ids are skipped and reported (GS_ERR_RANGE). */
int gs_cc_filter_edges(gs_cc_t* h, const void* src, const void* dst, uint64_t n, void* pairs, uint64_t cap,
                       uint64_t* n_out);
/* Pause (on = 0) / resume (on = 1) marking on a GS_CC_TRACK_MARKS handle: folds while paused leave
 * no marks (a replica folding the other ranks' partial summaries must not re-export them). */
int gs_cc_set_marking(gs_cc_t* h, int on);

/* ---- multi-GPU CombineCC (windowAll / tree reduce of partial summaries), csrc/comm.hip ----
 * One process (or thread) per GPU, one gs_comm_t per rank. Replaces the windowAll gather of the
 * partitions' window results (SummaryBulkAggregation.java:81-83) and ConnectedComponentsTree's
 * pairwise rounds (SummaryTreeReduce.java:95-123) with RCCL collectives over xGMI.
 *   gs_comm_unique_id   rank 0 makes the 128-byte RCCL unique id; the caller hands it to every
 *                       rank (torch.distributed broadcast, the job configuration, ...)
 *   gs_comm_create      every rank, concurrently: ncclCommInitRank(world, id, rank) on `device`
 *   gs_comm_create_local  `world` communicators of ONE process and device, one thread per rank
 *                       (tests of the exchange on a one-GPU box: RCCL refuses two ranks on one device)
 *   gs_cc_merge_window  after folding this rank's slice of a window: exchange this window's
 *                       partial summary (the handle needs GS_CC_TRACK_MARKS) and close the window.
 *     GS_MERGE_ALLGATHER  every rank keeps the GLOBAL summary (all-gather of deltas; every rank's
 *                         emission is the Merger's). From the second window on ONE all-gather of
 *                         slots sized from the last window's deltas (an outgrown slot costs one
 *                         more exact round, decided alike on every rank)
 *     GS_MERGE_GATHER     windowAll: deltas to rank 0, which folds them and emits
 *     GS_MERGE_TREE       log2(P) pairwise rounds to rank 0 (SummaryTreeReduce.enhance)
 *     GS_MERGE_PREFILTER  gs_cc_fold_windows only (the exchange needs the window's edges): ranks
 *                         1..P-1 keep no forest — each filters its slice of a window against the
 *                         giant bitmap rank 0 broadcasts and sends the surviving edges to rank 0,
 *                         which folds its own slice and every survivor, closes and emits (dense
 *                         ids; GS_CC_TRACK_MARKS not needed). Slices may differ in size per rank
 *                         and may be empty. The bitmap goes out after close 0 on the call's stream
 *                         (window 2's filter waits for it), later ones on a side stream over a
 *                         communicator split from this one when a handle is first bound in this
 *                         mode (collective), installed two windows later: a stale bitmap only lets
 *                         more edges through.
 *   Every rank must call it once per window with the same mode. In GATHER / TREE only rank 0's
 *   emission is the job's, and the call waits for the delta sizes. In ALLGATHER it does not wait:
 *   the sizes are checked lazily (an outgrown slot's tail round) by the next merge_window, or first
 *   thing in any call that consumes the emission or folds (stats, checksum, emit_*, find,
 *   labels_device, sync, fold*, merge, combine, reset, destroy) — gs_cc_fold_windows alone folds
 *   the next window without that wait (its merge exports before settling). */
typedef struct gs_comm gs_comm_t;
enum { GS_MERGE_ALLGATHER = 0, GS_MERGE_GATHER = 1, GS_MERGE_TREE = 2, GS_MERGE_PREFILTER = 3 };
int gs_comm_unique_id(void* id, uint64_t id_bytes);
int gs_comm_create(gs_comm_t** out, const void* unique_id, int rank, int world, int device);
int gs_comm_create_local(gs_comm_t** comms, int world, int device);
int gs_comm_destroy(gs_comm_t* comm);
/* rank, world size, payload bytes sent / received, windows merged, and speculative all-gather
 * rounds whose slot a delta outgrew (each then ran one exact round) */
int gs_comm_info(gs_comm_t* comm, int* rank, int* world, uint64_t* bytes_sent, uint64_t* bytes_recv, uint64_t* exchanges,
                 uint64_t* overflows);
int gs_cc_merge_window(gs_cc_t* h, gs_comm_t* comm, int mode);

/* ---- a batch of count windows in one call ----
 * SummaryBulkAggregation.run over a bounded stream (SummaryBulkAggregation.java:68-90, the Merger
 * SummaryAggregation.java:106-119): for each window of window_edges edges of src/dst (the last
 * window may be shorter) gs_cc_fold, then gs_cc_merge_window(h, comm, mode) when comm is not NULL,
 * else gs_cc_close_window — the per-window host loop run inside the library (one ABI call per batch
 * instead of two per window). After it returns, the labels are those of the last window's
 * emission; *windows_out (may be NULL) = windows folded. Stops at the first failure. With
 * GS_MERGE_PREFILTER only rank 0 folds (the others filter their slices for it); the ranks agree on
 * the call's window count (the most any rank passes, n / window_edges rounded up; one collective per
 * call) and a rank with fewer windows, or none (n == 0), runs empty ones; window_edges may differ. */
int gs_cc_fold_windows(gs_cc_t* h, gs_comm_t* comm, int mode, const void* src, const void* dst, uint64_t n,
                       uint64_t window_edges, uint64_t* windows_out);

/* ---- instrumentation ----
 * kernel ids: 0 fold (young-forest / plain k_fold launches), 1 compress (close_window), 2 merge,
 * 3 export, 4 ring (the steady k_fold_ring launches), 5 reserved (a retired steady-fold variant;
 * always 0); fold time = 0 + 4. */
enum { GS_K_FOLD = 0, GS_K_COMPRESS = 1, GS_K_MERGE = 2, GS_K_EXPORT = 3, GS_K_RING = 4, GS_K_ROUTE = 5, GS_K_COUNT = 6 };
/* enable = 0: off; 1: every kernel; GS_TIMING_MASK | (1 << GS_K_x) | ...: only those kernels
 * carry timing events (a timed launch costs ~3 us more dispatch time). Totals reset. */
enum { GS_TIMING_MASK = 0x100 };
int gs_cc_timing(gs_cc_t* h, int enable);
int gs_cc_kernel_time(gs_cc_t* h, int kernel, double* total_ms, uint64_t* launches);
/* units the timed launches of that class processed since gs_cc_timing: edges for folds and merges
 * (what each launch actually folded, after the library's internal cuts), vertex capacity per close */
int gs_cc_kernel_units(gs_cc_t* h, int kernel, uint64_t* units);

/* ---- synthetic streams on the device (definition: oracle/gen.c header) ----
 * Write ids [first, first+n) of the stream into src/dst (device pointers, id_bits wide). */
int gs_gen_rmat(void* src, void* dst, uint32_t id_bits, uint64_t first, uint64_t n, int scale,
                uint64_t seed, uint32_t ta, uint32_t tb, uint32_t tc, int scramble, void* hip_stream);
int gs_gen_er(void* src, void* dst, uint32_t id_bits, uint64_t first, uint64_t n, uint64_t nv,
              uint64_t seed, void* hip_stream);

/* ---- edge-file ingestion (ConnectedComponentsExample.java:108-119) ----
 * Parses n_bytes of text, one edge per line: Long.parseLong of fields 0 and 1 of
 * line.split("\\s") (one whitespace character between fields; trailing whitespace and fields
 * past the second ignored; a last line without '\n' counts). text: host or device; src/dst:
 * host or device, id_bits wide, capacity cap edges. *n_edges = lines parsed. A line the
 * reference would reject -> GS_ERR_INVALID, *n_edges = its 0-based index. */
int gs_parse_edges(const char* text, uint64_t n_bytes, uint32_t id_bits, void* src, void* dst, uint64_t cap,
                   uint64_t* n_edges, int device, void* hip_stream);

/* ---- streaming edge-file ingestion into a summary (ConnectedComponentsExample.java:108-119 ->
 * edges.aggregate(new ConnectedComponents<>(mergeWindowTime)), :61) ----
 * The text (gs_parse_edges' line rules) is consumed in chunks of at most chunk_bytes (0 = 64 MiB),
 * each cut after its last '
' (the partial last line carried to the next chunk), copied to the
 * device through two pinned staging buffers (the host's read / copy of chunk i+1 overlaps the parse
 * of chunk i and the folds of chunk i-1), parsed on the device into an edge ring, and folded into h
 * straight from it in count windows of window_edges edges, every window closed (the Merger's
 * emission; a last partial window is closed too). The ids never return to the host.
 * gs_cc_fold_text: text in host memory (pinned: DMA straight from it; pageable: through the pinned
 * staging) or device memory (one chunk). gs_cc_fold_file: read(2) from path into the staging.
 * h: either id width; GS_CC_SPARSE_IDS summaries take any Long id. *edges_out = edges folded; *windows_out =
 * windows closed. A line the reference rejects: GS_ERR_INVALID, every line before it folded (its
 * window left open), *edges_out = its 0-based line number. A line longer than chunk_bytes:
 * GS_ERR_CAPACITY (a read error: GS_ERR_INVALID), every whole chunk before the one holding it
 * folded (its window left open), *edges_out = the lines folded. Enqueued on h's stream like
 * gs_cc_fold_windows. on_window (may be NULL): called on the calling thread after window w's close is enqueued (w counts from 0 per call): the Merger's
 * per-window emission hook (read it with gs_cc_emit_delta / _pairs / gs_cc_checksum there); with a
 * callback every window is folded and closed by a call of its own (gs_cc_fold + gs_cc_close_window)
 * instead of in gs_cc_fold_windows batches. */
typedef void (*gs_window_fn)(void* ctx, uint64_t window);
int gs_cc_fold_text(gs_cc_t* h, const char* text, uint64_t n_bytes, uint64_t window_edges, uint64_t chunk_bytes,
                    gs_window_fn on_window, void* ctx, uint64_t* edges_out, uint64_t* windows_out);
int gs_cc_fold_file(gs_cc_t* h, const char* path, uint64_t window_edges, uint64_t chunk_bytes,
                    gs_window_fn on_window, void* ctx, uint64_t* edges_out, uint64_t* windows_out);

/* ---- BipartitenessCheck (library/BipartitenessCheck.java:38-133, summaries/Candidates.java) ----
 * A Candidates summary on the device: union-find with a parity bit per vertex. ids in
 * [0, vertex_capacity), vertex_capacity <= 2^31 - 1, id_bits 32 or 64. The emission of a
 * bipartite summary = every vertex with its component key (the component's minimum id) and its
 * sign (true iff on the key vertex's side); a summary that has seen an odd cycle is failed for
 * good (Candidates.fail(): "(false,{})"). Self-loops only add their vertex (edgeToCandidate).
 *   gs_bip_create / _reset     new Candidates(true)                       (Candidates.java:30-33)
 *   gs_bip_fold / _fold_pairs  updateFunction.foldEdges over a batch      (BipartitenessCheck.java:93-95)
 *   gs_bip_merge               combineFunction.reduce: into.merge(from)   (BipartitenessCheck.java:121-124)
 *   gs_bip_close_window        the Merger's per-window emission           (SummaryAggregation.java:106-119)
 *   gs_bip_status / _checksum  getSuccess() (Candidates.java:40-42), sizes, and
 *                              sum over v of splitmix64(v ^ splitmix64(((key << 1) | sign) ^ 0xD1B54A32D192ED03))
 *   gs_bip_emit_pairs          (vertex, key, sign) ordered by vertex      (Candidates.getMap(), :44-46)
 *   gs_bip_restore             restoreState: the summary becomes a snapshot's — getSuccess() and
 *                              the n entries gs_bip_emit_pairs wrote (any order; host or device
 *                              arrays of the handle's id width)           (SummaryAggregation.java:121-135)
 * GS_BIP_REFERENCE_LITERAL (gs_bip_create_ex): the reference's Candidates rule as written
 * (Candidates.java:77-192) instead of its intended semantics, for callers that need the reference's
 * emissions on multi-window / multi-partition streams: a merge writes an input component under
 * min(input key, lowest overlapping key) and removes only the other overlapping components (so a
 * vertex may sit in several components), drops the result of their inner merges (:130), keeps the
 * receiving side's signs, and skips components with an equal vertex set. The rule is sequential:
 * one workgroup applies it edge after edge (csrc/bip_literal.hpp), for parity, not throughput.
 * State: at most entry_capacity component memberships made between resets (0: 16 x
 * vertex_capacity; GS_ERR_CAPACITY past it). Such summaries merge only with each other;
 * gs_bip_status / _checksum count (component, vertex) entries; gs_bip_emit_pairs writes every
 * entry ordered by vertex, then key; close_window is a no-op; a place where the reference's
 * merge would throw (an empty mergeBy list, :156) fails the call with GS_ERR_INVALID; gs_bip_restore
 * loads the entries as they are (components sharing vertices included). An intended-semantics
 * summary is restored from one parity edge per vertex (GS_ERR_INVALID for entries no bipartite
 * summary emits: a key outside its component, a component of one side only). */
typedef struct gs_bip gs_bip_t;
enum { GS_BIP_REFERENCE_LITERAL = 1 };
int gs_bip_create(gs_bip_t** out, uint64_t vertex_capacity, uint32_t id_bits, int device);
int gs_bip_create_ex(gs_bip_t** out, uint64_t vertex_capacity, uint32_t id_bits, int device, uint32_t flags,
                     uint64_t entry_capacity);
int gs_bip_destroy(gs_bip_t* h);
int gs_bip_reset(gs_bip_t* h);
int gs_bip_set_stream(gs_bip_t* h, void* hip_stream);
int gs_bip_sync(gs_bip_t* h);
int gs_bip_fold(gs_bip_t* h, const void* src, const void* dst, uint64_t n);
int gs_bip_fold_pairs(gs_bip_t* h, const void* pairs, uint64_t n);
int gs_bip_merge(gs_bip_t* into, gs_bip_t* from);
int gs_bip_close_window(gs_bip_t* h);
int gs_bip_status(gs_bip_t* h, int* bipartite, uint64_t* n_vertices, uint64_t* n_components);
int gs_bip_checksum(gs_bip_t* h, uint64_t* checksum, int* bipartite, uint64_t* n_vertices, uint64_t* n_components);
int gs_bip_emit_pairs(gs_bip_t* h, void* vertices, void* keys, uint8_t* signs, uint64_t cap, uint64_t* n_out);
int gs_bip_restore(gs_bip_t* h, int bipartite, const void* vertices, const void* keys, const uint8_t* signs, uint64_t n);

const char* gs_last_error(void);
int gs_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GSGPU_H */
