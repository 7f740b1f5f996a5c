/*
 * emission.c — TEST INFRASTRUCTURE ONLY (parity checker; see oracle.h for the pinning).
 *
 * Incremental canonical-emission tracker for long streams of small windows (BASELINE config 5:
 * 4,096 windows of 2^16 edges). The Merger emits the whole cumulative summary after every window
 * (SummaryAggregation.java:106-119, transientState == false: ConnectedComponents.java:53); the
 * oracle's per-window checksum of that emission (gso_ds_canonical_checksum) walks every vertex
 * of the summary, O(|V_seen|) per window, which is 10^10-10^11 hash probes over 4,096 windows.
 *
 * The canonical emission — every vertex with the minimum id of its component — depends only on the
 * partition of the vertices seen so far into components, i.e. on the edge set, not on the union
 * order, rank tie-breaks or partitioning. The tracker keeps that partition
 * itself, driven by the same edges in the same windows: a dense union-find by size whose roots also
 * carry the component's minimum id, its member list and its share of the checksum,
 *     S(C) = sum over v in C of pair_mix(v, min C),   H = sum over components of S(C).
 * A union that changes a component's minimum re-sums that component's members (the one with the
 * larger minimum), so a window costs its edges plus the members of components whose label changed,
 * never |V_seen|. It is NOT trusted on its own: gso_cc_run_counts with GSO_EMIT_TRACK compares it
 * with the reference restatement's full canonical checksum of the Merger's summary every
 * verify_every windows and after the last one, and fails (returns -2) on any difference.
 */
#include "oracle.h"

#include <stdlib.h>

struct gso_track {
    int64_t*  tp;       /* union-find parent, -1 = unseen                     */
    uint32_t* size;     /* component size (roots)                             */
    int64_t*  mn;       /* component minimum id (roots)                       */
    uint64_t* sum;      /* S(C) (roots)                                       */
    int64_t*  head;     /* member list: first member (roots)                  */
    int64_t*  tail;     /* last member (roots)                                */
    int64_t*  next;     /* next member, -1 = end                              */
    uint64_t  cap;
    uint64_t  h, nv, nc;
    int       overflow; /* an id >= cap or < 0 was seen                       */
};

gso_track* gso_track_new(uint64_t cap) {
    gso_track* t = (gso_track*)calloc(1, sizeof(gso_track));
    if (!t) return NULL;
    t->cap = cap;
    t->tp = (int64_t*)malloc(cap * sizeof(int64_t));
    t->size = (uint32_t*)malloc(cap * sizeof(uint32_t));
    t->mn = (int64_t*)malloc(cap * sizeof(int64_t));
    t->sum = (uint64_t*)malloc(cap * sizeof(uint64_t));
    t->head = (int64_t*)malloc(cap * sizeof(int64_t));
    t->tail = (int64_t*)malloc(cap * sizeof(int64_t));
    t->next = (int64_t*)malloc(cap * sizeof(int64_t));
    if (!t->tp || !t->size || !t->mn || !t->sum || !t->head || !t->tail || !t->next) {
        gso_track_free(t);
        return NULL;
    }
    for (uint64_t v = 0; v < cap; ++v) t->tp[v] = -1;
    return t;
}

void gso_track_free(gso_track* t) {
    if (!t) return;
    free(t->tp); free(t->size); free(t->mn); free(t->sum); free(t->head); free(t->tail); free(t->next);
    free(t);
}

static inline int64_t tr_find(gso_track* t, int64_t x) {
    int64_t r = x;
    while (t->tp[r] != r) r = t->tp[r];
    while (t->tp[x] != r) { int64_t nx = t->tp[x]; t->tp[x] = r; x = nx; }
    return r;
}

static inline void tr_touch(gso_track* t, int64_t v) {
    if (t->tp[v] >= 0) return;
    t->tp[v] = v;
    t->size[v] = 1;
    t->mn[v] = v;
    t->sum[v] = gso_pair_mix((uint64_t)v, (uint64_t)v);
    t->head[v] = t->tail[v] = v;
    t->next[v] = -1;
    t->h += t->sum[v];
    t->nv += 1;
    t->nc += 1;
}

/* S(C) with the label m, over C's member list */
static uint64_t tr_resum(const gso_track* t, int64_t root, int64_t m) {
    uint64_t s = 0;
    for (int64_t x = t->head[root]; x >= 0; x = t->next[x]) s += gso_pair_mix((uint64_t)x, (uint64_t)m);
    return s;
}

void gso_track_union(gso_track* t, int64_t u, int64_t v) {
    if (u < 0 || v < 0 || (uint64_t)u >= t->cap || (uint64_t)v >= t->cap) { t->overflow = 1; return; }
    tr_touch(t, u);
    tr_touch(t, v);
    if (u == v) return;
    int64_t a = tr_find(t, u), b = tr_find(t, v);
    if (a == b) return;
    if (t->size[a] < t->size[b]) { int64_t x = a; a = b; b = x; }   /* b joins a */
    const int64_t m = t->mn[a] < t->mn[b] ? t->mn[a] : t->mn[b];
    uint64_t sa = t->sum[a], sb = t->sum[b];
    if (t->mn[a] != m) sa = tr_resum(t, a, m);
    if (t->mn[b] != m) sb = tr_resum(t, b, m);
    t->h += (sa + sb) - (t->sum[a] + t->sum[b]);
    t->tp[b] = a;
    t->size[a] += t->size[b];
    t->mn[a] = m;
    t->sum[a] = sa + sb;
    t->next[t->tail[a]] = t->head[b];
    t->tail[a] = t->tail[b];
    t->nc -= 1;
}

uint64_t gso_track_checksum(const gso_track* t, uint64_t* n_vertices, uint64_t* n_components) {
    if (n_vertices) *n_vertices = t->nv;
    if (n_components) *n_components = t->nc;
    return t->h;
}

int gso_track_overflow(const gso_track* t) { return t->overflow; }
