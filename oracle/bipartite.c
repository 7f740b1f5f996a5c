/*
 * bipartite.c — TEST INFRASTRUCTURE ONLY (parity checker / cpu_baseline of BipartitenessCheck).
 *
 * A C restatement of the semantics the reference's own BipartitenessCheck tests pin
 * (src/test/.../example/test/BipartitenessCheckTest.java:35-90) — oracle/bipartite.py
 * ParityUnionFind / intended_run — run through the reference's dataflow
 * (SummaryBulkAggregation.java:68-130: a fresh summary per partition per window, folded by that
 * partition's task; the window's partials combined in partition order, BipartitenessCheck.java:
 * 121-124; the Merger folding each window result into the cumulative summary,
 * SummaryAggregation.java:106-119). A summary is a union-find with a parity bit per vertex
 * (hash map keyed by the Long id): an edge asks for opposite sides (edgeToCandidate,
 * BipartitenessCheck.java:54-61), a self-loop only adds its vertex, a same-component edge with equal
 * sides fails the summary for good (Candidates.fail()); a merge unions every (vertex, its root,
 * its parity) relation of the other summary. Roots are component minima (the smaller root wins),
 * so a vertex's key is its component's minimum id and its sign is "same side as the key".
 * Where the literal Candidates.merge departs from these semantics: oracle/bipartite.py header.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"

typedef struct {
    int64_t* key;      /* slot -> id (INT64_MIN: empty)             */
    uint32_t* idx;     /* slot -> entry                              */
    uint64_t mask;
    int64_t* id;       /* entry -> id                                */
    uint32_t* parent;  /* entry -> parent entry                      */
    uint8_t* par;      /* entry -> parity relative to its parent     */
    uint64_t n, cap;
    int ok;
} bip_uf;

static void* xalloc(size_t n) {
    void* p = calloc(1, n ? n : 1);
    if (!p) abort();
    return p;
}

static void uf_init(bip_uf* u, uint64_t hint) {
    uint64_t s = 64;
    while (s < 2 * hint) s <<= 1;
    memset(u, 0, sizeof(*u));
    u->mask = s - 1;
    u->key = xalloc(s * sizeof(int64_t));
    for (uint64_t i = 0; i < s; ++i) u->key[i] = INT64_MIN;
    u->idx = xalloc(s * sizeof(uint32_t));
    u->cap = hint > 16 ? hint : 16;
    u->id = xalloc(u->cap * sizeof(int64_t));
    u->parent = xalloc(u->cap * sizeof(uint32_t));
    u->par = xalloc(u->cap);
    u->ok = 1;
}

static void uf_free(bip_uf* u) {
    free(u->key); free(u->idx); free(u->id); free(u->parent); free(u->par);
    memset(u, 0, sizeof(*u));
}

static void uf_rehash(bip_uf* u) {
    const uint64_t s = 2 * (u->mask + 1);
    int64_t* key = xalloc(s * sizeof(int64_t));
    uint32_t* idx = xalloc(s * sizeof(uint32_t));
    for (uint64_t i = 0; i < s; ++i) key[i] = INT64_MIN;
    for (uint64_t e = 0; e < u->n; ++e) {
        uint64_t h = gso_splitmix64((uint64_t)u->id[e]) & (s - 1);
        while (key[h] != INT64_MIN) h = (h + 1) & (s - 1);
        key[h] = u->id[e];
        idx[h] = (uint32_t)e;
    }
    free(u->key); free(u->idx);
    u->key = key; u->idx = idx; u->mask = s - 1;
}

/* entry of id v, made (its own root, parity 0) if absent */
static uint32_t uf_entry(bip_uf* u, int64_t v) {
    uint64_t h = gso_splitmix64((uint64_t)v) & u->mask;
    while (u->key[h] != INT64_MIN) {
        if (u->key[h] == v) return u->idx[h];
        h = (h + 1) & u->mask;
    }
    if (u->n == u->cap) {
        u->cap *= 2;
        u->id = realloc(u->id, u->cap * sizeof(int64_t));
        u->parent = realloc(u->parent, u->cap * sizeof(uint32_t));
        u->par = realloc(u->par, u->cap);
        if (!u->id || !u->parent || !u->par) abort();
    }
    const uint32_t e = (uint32_t)u->n++;
    u->key[h] = v;
    u->idx[h] = e;
    u->id[e] = v;
    u->parent[e] = e;
    u->par[e] = 0;
    if (2 * u->n > u->mask + 1) uf_rehash(u);
    return e;
}

/* root of e (path compression, parity to the root accumulated); *p = parity of e to the root */
static uint32_t uf_find(bip_uf* u, uint32_t e, uint8_t* p) {
    uint32_t r = e;
    uint8_t acc = 0;
    while (u->parent[r] != r) { acc ^= u->par[r]; r = u->parent[r]; }
    /* compress: every entry on the path points at r with its parity to r */
    uint8_t rem = acc;
    uint32_t x = e;
    while (u->parent[x] != x) {
        const uint32_t nx = u->parent[x];
        const uint8_t px = u->par[x];
        u->parent[x] = r;
        u->par[x] = rem;
        rem ^= px;
        x = nx;
    }
    *p = acc;
    return r;
}

/* relation "side(a) xor side(b) == d" (an edge: d = 1) */
static void uf_relate(bip_uf* u, int64_t a, int64_t b, uint8_t d) {
    const uint32_t ea = uf_entry(u, a), eb = uf_entry(u, b);
    if (!u->ok || a == b) return;
    uint8_t pa, pb;
    const uint32_t ra = uf_find(u, ea, &pa), rb = uf_find(u, eb, &pb);
    if (ra == rb) {
        if ((uint8_t)(pa ^ pb) != d) u->ok = 0;
        return;
    }
    const int a_lo = u->id[ra] < u->id[rb];
    const uint32_t lo = a_lo ? ra : rb, hi = a_lo ? rb : ra;
    u->parent[hi] = lo;
    u->par[hi] = (uint8_t)(pa ^ pb ^ d);
}

/* into.merge(from): every (vertex, root, parity) relation of `from` */
static void uf_merge(bip_uf* into, bip_uf* from) {
    if (!from->ok) into->ok = 0;
    for (uint64_t e = 0; e < from->n; ++e) {
        uint8_t p;
        const uint32_t r = uf_find(from, (uint32_t)e, &p);
        if (r == e) (void)uf_entry(into, from->id[e]);
        else uf_relate(into, from->id[e], from->id[r], p);
    }
}

typedef struct {
    const int64_t* src;
    const int64_t* dst;
    uint64_t a, b;
    bip_uf uf;
} part_job;

static void* fold_part(void* arg) {
    part_job* j = (part_job*)arg;
    uf_init(&j->uf, (j->b - j->a) + 16);
    for (uint64_t i = j->a; i < j->b; ++i) uf_relate(&j->uf, j->src[i], j->dst[i], 1);
    return NULL;
}

int gso_bip_run(const int64_t* src, const int64_t* dst, uint64_t n, uint64_t window_edges, int partitions,
                int threads, int* ok, uint64_t* n_vertices, uint64_t* n_components, double* seconds) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    if (partitions < 1) partitions = 1;
    if (threads < 1) threads = 1;
    const uint64_t W = window_edges ? window_edges : (n ? n : 1);
    bip_uf summary;
    uf_init(&summary, 1024);
    part_job* jobs = xalloc((size_t)partitions * sizeof(part_job));
    pthread_t* th = xalloc((size_t)partitions * sizeof(pthread_t));
    for (uint64_t lo = 0; lo < n; lo += W) {
        const uint64_t len = (n - lo < W) ? n - lo : W;
        for (int p0 = 0; p0 < partitions; p0 += threads) {           /* `threads` task threads at a time */
            const int p1 = p0 + threads < partitions ? p0 + threads : partitions;
            for (int p = p0; p < p1; ++p) {
                jobs[p].src = src;
                jobs[p].dst = dst;
                jobs[p].a = lo + len * (uint64_t)p / (uint64_t)partitions;
                jobs[p].b = lo + len * (uint64_t)(p + 1) / (uint64_t)partitions;
                if (pthread_create(&th[p], NULL, fold_part, &jobs[p]) != 0) fold_part(&jobs[p]), th[p] = 0;
            }
            for (int p = p0; p < p1; ++p) if (th[p]) pthread_join(th[p], NULL);
        }
        /* windowAll combine in partition order, then the Merger: window result into the summary */
        bip_uf* win = &jobs[0].uf;
        for (int p = 1; p < partitions; ++p) { uf_merge(win, &jobs[p].uf); uf_free(&jobs[p].uf); }
        uf_merge(&summary, win);
        uf_free(win);
    }
    uint64_t comps = 0;
    for (uint64_t e = 0; e < summary.n; ++e) comps += summary.parent[e] == e;
    *ok = summary.ok;
    *n_vertices = summary.n;
    *n_components = comps;
    uf_free(&summary);
    free(jobs);
    free(th);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    return 0;
}
