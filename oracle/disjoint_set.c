/*
 * disjoint_set.c — TEST INFRASTRUCTURE ONLY (parity checker; see oracle.h for the pinning).
 *
 * Restatement of summaries/DisjointSet.java (reference, src/main/java/org/apache/flink/graph/
 * streaming/summaries/DisjointSet.java). The Java class keeps two HashMaps:
 *   matches: vertex -> parent     (DisjointSet.java:28)
 *   ranks:   vertex -> rank       (DisjointSet.java:29)
 * Here both live in insertion-ordered arrays indexed through an open-addressing table, and the
 * parent is held as an array index instead of a key (one hash lookup per hop saved; the
 * union/find decisions, and therefore every tree the Java code builds for a given iteration
 * order, are unchanged). Iteration order of getMatches() is insertion order; Java's HashMap
 * order differs, which can change rank tie-breaks inside merge() but never the partition into
 * components, hence never the canonical (minimum-id) labels this oracle emits.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

struct gso_ds {
    /* insertion-ordered entries */
    int64_t*  key;     /* vertex id                                      */
    uint64_t* par;     /* parent as entry index (matches.get(key))       */
    int32_t*  rank;    /* ranks.get(key)                                 */
    uint64_t  n, cap;
    /* open-addressing index: slot -> entry index + 1 (0 = empty) */
    int64_t*  skey;
    uint64_t* sidx;
    uint64_t  smask;
};

uint64_t gso_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

uint64_t gso_pair_mix(uint64_t v, uint64_t label) {
    return gso_splitmix64(v ^ gso_splitmix64(label ^ 0xD1B54A32D192ED03ULL));
}

static void* xrealloc(void* p, size_t sz) {
    void* q = realloc(p, sz);
    if (!q && sz) abort();
    return q;
}

gso_ds* gso_ds_new(void) {
    gso_ds* ds = (gso_ds*)calloc(1, sizeof(gso_ds));
    ds->cap = 16;
    ds->key = (int64_t*)xrealloc(NULL, ds->cap * sizeof(int64_t));
    ds->par = (uint64_t*)xrealloc(NULL, ds->cap * sizeof(uint64_t));
    ds->rank = (int32_t*)xrealloc(NULL, ds->cap * sizeof(int32_t));
    ds->smask = 31;
    ds->skey = (int64_t*)calloc(ds->smask + 1, sizeof(int64_t));
    ds->sidx = (uint64_t*)calloc(ds->smask + 1, sizeof(uint64_t));
    return ds;
}

void gso_ds_free(gso_ds* ds) {
    if (!ds) return;
    free(ds->key); free(ds->par); free(ds->rank); free(ds->skey); free(ds->sidx);
    free(ds);
}

uint64_t gso_ds_size(const gso_ds* ds) { return ds->n; }
int64_t gso_ds_key_at(const gso_ds* ds, uint64_t i) { return ds->key[i]; }

static inline uint64_t slot_of(const gso_ds* ds, int64_t k) {
    return gso_splitmix64((uint64_t)k) & ds->smask;
}

/* containsKey / get: entry index or UINT64_MAX */
static inline uint64_t lookup(const gso_ds* ds, int64_t k) {
    uint64_t s = slot_of(ds, k);
    for (;;) {
        uint64_t i = ds->sidx[s];
        if (i == 0) return UINT64_MAX;
        if (ds->skey[s] == k) return i - 1;
        s = (s + 1) & ds->smask;
    }
}

static void rehash(gso_ds* ds) {
    uint64_t nslots = (ds->smask + 1) * 2;
    free(ds->skey); free(ds->sidx);
    ds->smask = nslots - 1;
    ds->skey = (int64_t*)calloc(nslots, sizeof(int64_t));
    ds->sidx = (uint64_t*)calloc(nslots, sizeof(uint64_t));
    for (uint64_t i = 0; i < ds->n; ++i) {
        uint64_t s = slot_of(ds, ds->key[i]);
        while (ds->sidx[s]) s = (s + 1) & ds->smask;
        ds->skey[s] = ds->key[i];
        ds->sidx[s] = i + 1;
    }
}

/* makeSet(e): matches.put(e,e); ranks.put(e,0)   (DisjointSet.java:53-56).
 * Only ever called for absent keys on the union path; for a present key the Java put()
 * overwrites parent and rank, which this also does. */
static uint64_t make_set_idx(gso_ds* ds, int64_t e) {
    uint64_t i = lookup(ds, e);
    if (i != UINT64_MAX) { ds->par[i] = i; ds->rank[i] = 0; return i; }
    if (ds->n == ds->cap) {
        ds->cap *= 2;
        ds->key = (int64_t*)xrealloc(ds->key, ds->cap * sizeof(int64_t));
        ds->par = (uint64_t*)xrealloc(ds->par, ds->cap * sizeof(uint64_t));
        ds->rank = (int32_t*)xrealloc(ds->rank, ds->cap * sizeof(int32_t));
    }
    if ((ds->n + 1) * 2 > ds->smask + 1) rehash(ds);
    i = ds->n++;
    ds->key[i] = e; ds->par[i] = i; ds->rank[i] = 0;
    uint64_t s = slot_of(ds, e);
    while (ds->sidx[s]) s = (s + 1) & ds->smask;
    ds->skey[s] = e; ds->sidx[s] = i + 1;
    return i;
}

void gso_ds_make_set(gso_ds* ds, int64_t e) { (void)make_set_idx(ds, e); }

/* find with full path compression (DisjointSet.java:66-80: the recursion rewrites every vertex
 * on the path to the root). Iterative two-pass form, identical final state. */
static inline uint64_t find_idx(gso_ds* ds, uint64_t i) {
    uint64_t r = i;
    while (ds->par[r] != r) r = ds->par[r];
    while (ds->par[i] != r) { uint64_t nx = ds->par[i]; ds->par[i] = r; i = nx; }
    return r;
}

int gso_ds_find(gso_ds* ds, int64_t e, int64_t* root) {
    uint64_t i = lookup(ds, e);
    if (i == UINT64_MAX) return 0;               /* find() returns null for unknown ids (:67-69) */
    *root = ds->key[find_idx(ds, i)];
    return 1;
}

/* union (DisjointSet.java:92-118) */
void gso_ds_union(gso_ds* ds, int64_t e1, int64_t e2) {
    uint64_t i1 = lookup(ds, e1);
    if (i1 == UINT64_MAX) i1 = make_set_idx(ds, e1);        /* :94-96  */
    uint64_t i2 = lookup(ds, e2);
    if (i2 == UINT64_MAX) i2 = make_set_idx(ds, e2);        /* :97-99  */
    uint64_t r1 = find_idx(ds, i1), r2 = find_idx(ds, i2);  /* :101-102 */
    if (r1 == r2) return;                                   /* :104-106 */
    int32_t d1 = ds->rank[r1], d2 = ds->rank[r2];           /* :108-109 */
    if (d1 > d2) {
        ds->par[r2] = r1;                                   /* :110-111 */
    } else if (d1 < d2) {
        ds->par[r1] = r2;                                   /* :112-113 */
    } else {
        ds->par[r2] = r1;                                   /* :114-116 */
        ds->rank[r1] = d1 + 1;
    }
}

/* merge: union every (key, parent) entry of other (DisjointSet.java:127-131) */
void gso_ds_merge(gso_ds* ds, gso_ds* other) {
    for (uint64_t i = 0; i < other->n; ++i)
        gso_ds_union(ds, other->key[i], other->key[other->par[i]]);
}

/* CombineCC.reduce (library/ConnectedComponents.java:116-125) */
gso_ds* gso_combine(gso_ds* s1, gso_ds* s2) {
    uint64_t c1 = s1->n, c2 = s2->n;
    if (c1 <= c2) { gso_ds_merge(s2, s1); return s2; }
    gso_ds_merge(s1, s2);
    return s1;
}

/* per-entry canonical label: minimum key of the entry's component */
static int64_t* canonical_per_entry(gso_ds* ds) {
    int64_t* mn = (int64_t*)malloc((ds->n ? ds->n : 1) * sizeof(int64_t));
    for (uint64_t i = 0; i < ds->n; ++i) mn[i] = INT64_MAX;
    for (uint64_t i = 0; i < ds->n; ++i) {
        uint64_t r = find_idx(ds, i);
        if (ds->key[i] < mn[r]) mn[r] = ds->key[i];
    }
    for (uint64_t i = 0; i < ds->n; ++i) {
        uint64_t r = ds->par[i];            /* fully compressed by the loop above */
        if (r != i) mn[i] = mn[r];
    }
    return mn;
}

uint64_t gso_ds_canonical_dense(gso_ds* ds, int64_t* labels, uint64_t cap) {
    for (uint64_t v = 0; v < cap; ++v) labels[v] = -1;
    int64_t* mn = canonical_per_entry(ds);
    for (uint64_t i = 0; i < ds->n; ++i) {
        int64_t k = ds->key[i];
        if (k >= 0 && (uint64_t)k < cap) labels[k] = mn[i];
    }
    free(mn);
    return ds->n;
}

uint64_t gso_ds_canonical_checksum(gso_ds* ds, uint64_t* n_vertices, uint64_t* n_components) {
    int64_t* mn = canonical_per_entry(ds);
    uint64_t h = 0, nc = 0;
    for (uint64_t i = 0; i < ds->n; ++i) {
        h += gso_pair_mix((uint64_t)ds->key[i], (uint64_t)mn[i]);
        if (mn[i] == ds->key[i]) ++nc;
    }
    free(mn);
    if (n_vertices) *n_vertices = ds->n;
    if (n_components) *n_components = nc;
    return h;
}

uint64_t gso_dense_checksum(const int64_t* labels, uint64_t n, uint64_t* n_seen, uint64_t* n_comp) {
    uint64_t h = 0, ns = 0, nc = 0;
    for (uint64_t v = 0; v < n; ++v) {
        if (labels[v] < 0) continue;
        h += gso_pair_mix(v, (uint64_t)labels[v]);
        ++ns;
        if ((uint64_t)labels[v] == v) ++nc;
    }
    if (n_seen) *n_seen = ns;
    if (n_comp) *n_comp = nc;
    return h;
}
