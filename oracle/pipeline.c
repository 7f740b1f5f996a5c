/*
 * pipeline.c — TEST INFRASTRUCTURE ONLY (parity checker and cpu_baseline; see oracle.h).
 *
 * Restatement of the dataflow SummaryBulkAggregation.run builds for ConnectedComponents
 * (reference src/main/java/org/apache/flink/graph/streaming/):
 *   SummaryBulkAggregation.java:76-83   map(PartitionMapper) -> keyBy(partition) ->
 *                                       timeWindow(fold from a fresh initial value) ->
 *                                       timeWindowAll(reduce CombineCC) -> flatMap(Merger), p=1
 *   SummaryBulkAggregation.java:121-123 PartialAgg.fold -> UpdateCC.foldEdges -> ds.union(u,v)
 *   SummaryAggregation.java:106-119     Merger.flatMap: summary = CombineCC(s, summary); emit
 *                                       (transientState == false for ConnectedComponents,
 *                                       library/ConnectedComponents.java:53)
 * Windows are count-based here (the reference's are wall-clock; SURVEY.md §7 "Hard parts"),
 * and window w's partition p is the contiguous slice [p*len/P, (p+1)*len/P) of the window.
 * The per-partition folds run on `threads` host threads (one Flink task thread per partition in
 * the reference); the windowAll reduce and the Merger run on one thread, as in the reference.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
    const int64_t* src;
    const int64_t* dst;
    uint64_t lo, len;      /* window slice */
    int P, T, tid;
    gso_ds** partials;
} fold_job;

static void* fold_worker(void* arg) {
    fold_job* j = (fold_job*)arg;
    for (int p = j->tid; p < j->P; p += j->T) {
        uint64_t a = j->lo + (j->len * (uint64_t)p) / (uint64_t)j->P;
        uint64_t b = j->lo + (j->len * (uint64_t)(p + 1)) / (uint64_t)j->P;
        if (a == b) { j->partials[p] = NULL; continue; }   /* no element => no window result */
        gso_ds* ds = gso_ds_new();                        /* fresh copy of the initial value */
        for (uint64_t i = a; i < b; ++i) gso_ds_union(ds, j->src[i], j->dst[i]);  /* UpdateCC */
        j->partials[p] = ds;
    }
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* FlattenSet (example/ConnectedComponentsExample.java:143-156): (vertex, find(vertex)) for every
 * vertex of the emitted summary. The tuple stream is consumed into a sink checksum. */
static uint64_t flatten_set(gso_ds* ds) {
    uint64_t h = 0;
    for (uint64_t i = 0; i < gso_ds_size(ds); ++i) {
        int64_t v = gso_ds_key_at(ds, i), r = 0;
        gso_ds_find(ds, v, &r);
        h += (uint64_t)v * 31u + (uint64_t)r;
    }
    return h;
}

int gso_cc_run(const int64_t* src, const int64_t* dst, uint64_t n, const gso_run_cfg* cfg,
               uint64_t* out_checksums, int64_t* out_labels, int64_t* final_labels,
               gso_run_stats* stats) {
    return gso_cc_run_counts(NULL, NULL, 0, src, dst, n, cfg, out_checksums, NULL, out_labels, final_labels, stats);
}

int gso_cc_run_from(const int64_t* init_v, const int64_t* init_l, uint64_t n_init,
                    const int64_t* src, const int64_t* dst, uint64_t n, const gso_run_cfg* cfg,
                    uint64_t* out_checksums, int64_t* out_labels, int64_t* final_labels,
                    gso_run_stats* stats) {
    return gso_cc_run_counts(init_v, init_l, n_init, src, dst, n, cfg, out_checksums, NULL, out_labels, final_labels,
                             stats);
}

int gso_cc_run_counts(const int64_t* init_v, const int64_t* init_l, uint64_t n_init,
                      const int64_t* src, const int64_t* dst, uint64_t n, const gso_run_cfg* cfg,
                      uint64_t* out_checksums, uint64_t* out_counts, int64_t* out_labels, int64_t* final_labels,
                      gso_run_stats* stats) {
    const int P = cfg->partitions > 0 ? cfg->partitions : 1;
    int T = cfg->threads > 0 ? cfg->threads : 1;
    if (T > P) T = P;
    const uint64_t W = cfg->window_edges ? cfg->window_edges : (n ? n : 1);
    gso_ds** partials = (gso_ds**)calloc((size_t)P, sizeof(gso_ds*));
    fold_job* jobs = (fold_job*)calloc((size_t)T, sizeof(fold_job));
    pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
    gso_ds* summary = NULL;            /* Merger.summary = initialVal (empty) */
    gso_track* track = NULL;           /* GSO_EMIT_TRACK: the incremental canonical emission */
    int rc = 0;
    if (cfg->emit_mode == GSO_EMIT_TRACK) {
        track = gso_track_new(cfg->label_cap);
        if (!track) { free(partials); free(jobs); free(th); return -1; }
    }
    if (n_init) {                      /* Merger.restoreState (SummaryAggregation.java:131-135): the
                                          snapshotted summary, rebuilt from its (vertex, label) pairs */
        summary = gso_ds_new();
        for (uint64_t i = 0; i < n_init; ++i) gso_ds_union(summary, init_v[i], init_l[i]);
        if (track) for (uint64_t i = 0; i < n_init; ++i) gso_track_union(track, init_v[i], init_l[i]);
    }
    uint64_t w = 0;
    volatile uint64_t sink = 0;
    double t0 = now_s();                /* the restore is not timed */

    for (uint64_t lo = 0; lo < n; lo += W, ++w) {
        uint64_t len = (n - lo < W) ? (n - lo) : W;
        for (int t = 0; t < T; ++t) {
            jobs[t] = (fold_job){src, dst, lo, len, P, T, t, partials};
            if (T == 1) fold_worker(&jobs[0]);
            else pthread_create(&th[t], NULL, fold_worker, &jobs[t]);
        }
        if (T > 1) for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);

        /* timeWindowAll(...).reduce(CombineCC) over the partials, in partition order */
        gso_ds* acc = NULL;
        for (int p = 0; p < P; ++p) {
            if (!partials[p]) continue;
            if (!acc) { acc = partials[p]; continue; }
            gso_ds* keep = gso_combine(acc, partials[p]);
            gso_ds_free(keep == acc ? partials[p] : acc);
            acc = keep;
        }
        /* Merger: summary = CombineCC.reduce(windowResult, summary); collect(summary) */
        if (!summary) {
            summary = acc;             /* reduce(s, empty) merges nothing and returns s */
        } else {
            gso_ds* keep = gso_combine(acc, summary);
            gso_ds_free(keep == acc ? summary : acc);
            summary = keep;
        }
        /* emission */
        switch (cfg->emit_mode) {
        case GSO_EMIT_FLATTEN: sink += flatten_set(summary); break;
        case GSO_EMIT_CHECKSUM:
            if (out_checksums)
                out_checksums[w] = gso_ds_canonical_checksum(summary, out_counts ? &out_counts[2 * w] : NULL,
                                                             out_counts ? &out_counts[2 * w + 1] : NULL);
            break;
        case GSO_EMIT_DENSE:
            if (out_labels) gso_ds_canonical_dense(summary, out_labels + w * cfg->label_cap, cfg->label_cap);
            if (out_checksums)
                out_checksums[w] = gso_ds_canonical_checksum(summary, out_counts ? &out_counts[2 * w] : NULL,
                                                             out_counts ? &out_counts[2 * w + 1] : NULL);
            break;
        case GSO_EMIT_TRACK: {
            for (uint64_t i = lo; i < lo + len; ++i) gso_track_union(track, src[i], dst[i]);
            uint64_t nv = 0, nc = 0;
            const uint64_t h = gso_track_checksum(track, &nv, &nc);
            if (out_checksums) out_checksums[w] = h;
            if (out_counts) { out_counts[2 * w] = nv; out_counts[2 * w + 1] = nc; }
            const int last = lo + len >= n;
            if (gso_track_overflow(track)) { rc = -3; goto done; }
            if (last || (cfg->verify_every && (w + 1) % cfg->verify_every == 0)) {
                uint64_t fv = 0, fc = 0;
                const uint64_t fh = gso_ds_canonical_checksum(summary, &fv, &fc);
                if (fh != h || fv != nv || fc != nc) { rc = -2; goto done; }
            }
            break;
        }
        default: break;
        }
    }
done:;
    double t1 = now_s();
    (void)sink;
    if (stats) {
        stats->windows = w;
        stats->seconds = t1 - t0;
        stats->final_vertices = 0;
        stats->final_components = 0;
        if (summary) gso_ds_canonical_checksum(summary, &stats->final_vertices, &stats->final_components);
    }
    if (final_labels) {
        if (summary) gso_ds_canonical_dense(summary, final_labels, cfg->label_cap);
        else for (uint64_t v = 0; v < cfg->label_cap; ++v) final_labels[v] = -1;
    }
    gso_ds_free(summary);
    gso_track_free(track);
    free(partials); free(jobs); free(th);
    return rc;
}
