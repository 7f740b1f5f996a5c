/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's streaming Connected Components path, used as the parity
 * checker for the HIP implementation (libgsgpu.so). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this code. The product path never links it.
 *
 * Parity pinning: the reference is Java 8 + Apache Flink 1.8 and cannot be built or run here
 * (no JDK, no Flink jars, no network: SURVEY.md §8c). This restatement is pinned by the
 * reference's own known-answer tests, committed as fixtures under tests/golden/:
 *   - DisjointSetTest          (src/test/.../util/DisjointSetTest.java:37-78)
 *   - ConnectedComponentsTest  (src/test/.../example/test/ConnectedComponentsTest.java:41,54-63)
 *   - ConnectedComponentsExample sample stream (src/main/.../example/ConnectedComponentsExample.java:121-127)
 * and cross-checked against scipy.sparse.csgraph on random streams (tests/golden/make_golden.py).
 *
 * Reference files followed (paths relative to src/main/java/org/apache/flink/graph/streaming/):
 *   summaries/DisjointSet.java:28-150      -> gso_ds_* (hash-map union-find, union by rank,
 *                                              recursive full path compression, merge)
 *   library/ConnectedComponents.java:83-85 -> UpdateCC (gso_ds_union per edge)
 *   library/ConnectedComponents.java:116-125 -> CombineCC (gso_combine: merge smaller into larger)
 *   SummaryBulkAggregation.java:68-130     -> per-partition fold of a fresh summary per window,
 *                                              windowAll reduce (gso_cc_run)
 *   SummaryAggregation.java:106-119        -> Merger: summary = CombineCC(windowResult, summary)
 */
#ifndef GS_ORACLE_H
#define GS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- DisjointSet<Long> restatement ---------------- */
typedef struct gso_ds gso_ds;

gso_ds*  gso_ds_new(void);
void     gso_ds_free(gso_ds* ds);
uint64_t gso_ds_size(const gso_ds* ds);                 /* getMatches().size()          */
void     gso_ds_make_set(gso_ds* ds, int64_t e);        /* DisjointSet.java:53-56       */
int      gso_ds_find(gso_ds* ds, int64_t e, int64_t* root); /* :66-80; 0 => null (unknown) */
void     gso_ds_union(gso_ds* ds, int64_t e1, int64_t e2);  /* :92-118                   */
void     gso_ds_merge(gso_ds* ds, gso_ds* other);       /* :127-131                     */
/* CombineCC.reduce (ConnectedComponents.java:116-125): returns the summary that absorbed the other. */
gso_ds*  gso_combine(gso_ds* s1, gso_ds* s2);
/* Iteration over getMatches() in insertion order: key i in [0, size). */
int64_t  gso_ds_key_at(const gso_ds* ds, uint64_t i);
/* Canonical labels: for every vertex in the summary, the minimum vertex id of its component.
 * Writes dense labels[v] for v < cap (-1 for vertices not in the summary). Returns #vertices. */
uint64_t gso_ds_canonical_dense(gso_ds* ds, int64_t* labels, uint64_t cap);
/* Order-independent checksum of the canonical (vertex,label) set (see gso_pair_mix). */
uint64_t gso_ds_canonical_checksum(gso_ds* ds, uint64_t* n_vertices, uint64_t* n_components);

/* ---------------- emission checksum (shared definition with the GPU) ---------------- */
uint64_t gso_pair_mix(uint64_t v, uint64_t label);
/* checksum over a dense label array (label < 0 == unseen) */
uint64_t gso_dense_checksum(const int64_t* labels, uint64_t n, uint64_t* n_seen, uint64_t* n_comp);

/* ---------------- streaming pipeline (SummaryBulkAggregation + Merger) ---------------- */
enum {
    GSO_EMIT_NONE = 0,       /* fold + combine + merge only                                   */
    GSO_EMIT_FLATTEN = 1,    /* + FlattenSet (find() for every vertex, ConnectedComponentsExample.java:143-156) */
    GSO_EMIT_CHECKSUM = 2,   /* + canonical checksum per window                               */
    GSO_EMIT_DENSE = 3,      /* + canonical dense labels per window into out_labels[w*cap + v] */
    GSO_EMIT_TRACK = 4       /* + canonical checksum per window from the incremental tracker
                                (emission.c; ids < label_cap), cross-checked against the full
                                canonical checksum of the Merger's summary every verify_every
                                windows and after the last (a difference returns -2)           */
};

typedef struct {
    uint64_t window_edges;   /* count-based window length (edges); 0 => one window             */
    int      partitions;     /* P = Flink parallelism of the fold                              */
    int      threads;        /* host threads used for the per-partition folds (<= partitions)  */
    int      emit_mode;      /* GSO_EMIT_*                                                     */
    uint64_t label_cap;      /* for GSO_EMIT_DENSE: dense label array length per window        */
    uint64_t verify_every;   /* for GSO_EMIT_TRACK: full-checksum cross-check period (0 = last only) */
} gso_run_cfg;

typedef struct {
    uint64_t windows;        /* emissions produced                                             */
    uint64_t final_vertices; /* |V_seen| after the last window                                 */
    uint64_t final_components;
    double   seconds;        /* wall time of the whole run                                     */
} gso_run_stats;

/* Runs the pipeline over edges (src[i], dst[i]). Windows are contiguous runs of window_edges
 * edges; inside a window, partition p folds the contiguous slice [p*len/P, (p+1)*len/P).
 * out_checksums (optional, length >= #windows) receives the per-window emission checksum
 * (GSO_EMIT_CHECKSUM / GSO_EMIT_DENSE). out_labels (optional) receives dense canonical labels
 * per window (GSO_EMIT_DENSE). final_labels (optional, label_cap) receives the final emission. */
int gso_cc_run(const int64_t* src, const int64_t* dst, uint64_t n, const gso_run_cfg* cfg,
               uint64_t* out_checksums, int64_t* out_labels, int64_t* final_labels,
               gso_run_stats* stats);
/* As gso_cc_run, with the Merger restored first (untimed) from a snapshot of n_init canonical
 * (vertex, label) pairs (ListCheckpointed restoreState, SummaryAggregation.java:127-135): the run
 * then continues the stream from the middle. */
int gso_cc_run_from(const int64_t* init_v, const int64_t* init_l, uint64_t n_init,
                    const int64_t* src, const int64_t* dst, uint64_t n, const gso_run_cfg* cfg,
                    uint64_t* out_checksums, int64_t* out_labels, int64_t* final_labels,
                    gso_run_stats* stats);

/* As gso_cc_run_from, also writing the per-window emission's (vertices, components) into
 * out_counts[2w], out_counts[2w+1] (GSO_EMIT_CHECKSUM / GSO_EMIT_DENSE; optional). */
int gso_cc_run_counts(const int64_t* init_v, const int64_t* init_l, uint64_t n_init,
                      const int64_t* src, const int64_t* dst, uint64_t n, const gso_run_cfg* cfg,
                      uint64_t* out_checksums, uint64_t* out_counts, int64_t* out_labels, int64_t* final_labels,
                      gso_run_stats* stats);

/* ---------------- BipartitenessCheck (bipartite.c; the semantics the reference's tests pin) ----
 * The dataflow of gso_cc_run over a parity union-find: *ok = the stream is bipartite; the final
 * summary's vertex and component counts. */
int gso_bip_run(const int64_t* src, const int64_t* dst, uint64_t n, uint64_t window_edges, int partitions,
                int threads, int* ok, uint64_t* n_vertices, uint64_t* n_components, double* seconds);

/* ---------------- incremental canonical emission (emission.c) ---------------- */
typedef struct gso_track gso_track;
gso_track* gso_track_new(uint64_t cap);            /* dense ids in [0, cap)                    */
void       gso_track_free(gso_track* t);
void       gso_track_union(gso_track* t, int64_t u, int64_t v);
uint64_t   gso_track_checksum(const gso_track* t, uint64_t* n_vertices, uint64_t* n_components);
int        gso_track_overflow(const gso_track* t);  /* an id outside [0, cap) was seen         */

/* ---------------- deterministic synthetic streams (same definition as the device generators) ---------------- */
uint64_t gso_splitmix64(uint64_t x);
/* RMAT: vertex space 2^scale; a,b,c as 32-bit integer thresholds (probability * 2^32, cumulative
 * handled inside); edge i depends only on (seed, i). ids scrambled by a seeded bijection. */
void gso_gen_rmat(int64_t* src, int64_t* dst, uint64_t first, uint64_t n, int scale,
                  uint64_t seed, uint32_t ta, uint32_t tb, uint32_t tc, int scramble);
/* Erdős–Rényi G(n, m)-style: uniform endpoints in [0, nv). */
void gso_gen_er(int64_t* src, int64_t* dst, uint64_t first, uint64_t n, uint64_t nv, uint64_t seed);

/* Edge-file input (ConnectedComponentsExample.java:108-119, parse.c): lines parsed (<= cap are
 * written), or -(index of the first line the reference rejects) - 1. */
int64_t gso_parse_edges(const char* text, uint64_t n_bytes, int64_t* src, int64_t* dst, uint64_t cap);

#ifdef __cplusplus
}
#endif

#endif
