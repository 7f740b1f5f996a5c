// bip_literal.hpp — the reference's Candidates summary restated literally (GS_BIP_REFERENCE_LITERAL):
// summaries/Candidates.java:25-197 and library/BipartitenessCheck.java:50-133, including the
// behaviour the intended-semantics union-find of bip.hip does not reproduce on multi-window streams:
//   * Candidates.merge (:77-139) merges an input component into the LOWEST-keyed overlapping
//     candidate component `firstKey`, but writes it under min(inputKey, firstKey) (:176) and removes
//     only the other overlapping components (:126-134): a smaller input key leaves the old firstKey
//     component in place beside the new one, sharing vertices with it;
//   * the result of the inner merge of those other components is dropped (`fail();` at :130);
//   * a reversed merge keeps the receiving side's signs (:155-187), so a key can be signed false;
//   * components whose vertex sets are equal are skipped, whatever their signs (:91-95).
// The state is therefore not a partition: a vertex can belong to several components. It is kept as
//   vhead[v]      -> v's membership nodes (linked; nodes of removed components pruned lazily)
//   node          = (component slot, sign, vertex)
//   component slot= key, alive, member array (node indices) in a bump-allocated arena
//   kslot[key]    -> the live component keyed `key` (keys are vertex ids: Candidates keys a
//                    component by its smallest endpoint, BipartitenessCheck.java:54-61)
// Every operation is the reference's sequential rule; the work inside one step (a component's
// members: overlap counts, the mergeBy minimum, consistency checks, additions) is spread over the
// threads of ONE workgroup. The rule's order only matters through the smallest common vertex
// (`mergeBy.get(0)`, a min-reduction) and the first failing add in TreeMap order (a min-reduction
// over the failing vertices); everything else is order-free. The engine is written against an
// execution context X (tid, nthreads, sync, atomics, a block scan): bip.hip runs it as a HIP
// workgroup; tests/bipl_host_check.cpp runs the same code serially on the host under ASan/UBSan.
#pragma once

#include <cstdint>

#ifdef __HIPCC__
#define GS_HD __host__ __device__
#else
#define GS_HD
#endif

namespace gsgpu {
namespace lit {

constexpr int32_t kNone = -1;
constexpr uint32_t kSign = 0x80000000u;           // node_cs: component slot | sign << 31
constexpr uint32_t kNoVertex = 0xFFFFFFFFu;

// error bits (Ctl::err): the engine stops at the first one, the host maps them to GS_ERR_*
constexpr uint32_t kErrCapacity = 1u;             // nodes / components / arena exhausted
constexpr uint32_t kErrRange = 2u;                // an edge endpoint >= capacity (the edge is skipped)
constexpr uint32_t kErrThrows = 4u;               // the reference would throw (an empty mergeBy, :156)

struct Ctl {
    uint32_t n_nodes, n_comps, n_arena;           // bump allocators
    uint32_t ok;                                  // Candidates.f0 (getSuccess)
    uint32_t err;
    uint32_t live_comps, live_entries;            // live components, live (component, vertex) entries
    uint32_t skipped;                             // kErrRange: an edge was skipped (reported, not fatal)
};

struct State {
    int32_t* vhead;       // [cap]
    int32_t* kslot;       // [cap]
    uint32_t* node_cs;    // [E]
    uint32_t* node_v;     // [E]
    int32_t* node_next;   // [E]
    uint32_t* comp_key;   // [C]
    uint32_t* comp_alive; // [C]
    uint32_t* comp_base;  // [C]
    uint32_t* comp_size;  // [C]
    uint32_t* comp_cap;   // [C]
    int32_t* arena;       // [A]
    uint32_t* cnt;        // [C] overlap counters, zero between uses
    uint32_t* touched;    // [C]
    uint64_t* mw;         // [C] mergeWith: key << 32 | slot
    uint64_t* mws;        // [C] mergeWith sorted by key
    uint32_t* sv;         // [cap] an input component's vertices
    uint8_t* ss;          // [cap] ... and signs
    uint32_t* keys;       // [cap] an input summary's live keys, ascending
    Ctl* ctl;
    uint32_t cap, E, C, A;
};

// values every thread reads after a sync (LDS on the device)
struct Shared {
    uint32_t n_touched, n_mw, minv, minc, flag, rev, cslot, newbase, nkeys, stop;
    uint32_t iv[2];
    uint8_t is[2];
};

GS_HD inline uint32_t slot_of(uint32_t cs) { return cs & ~kSign; }
GS_HD inline uint32_t sign_of(uint32_t cs) { return cs >> 31; }

// v's node in component slot c, or kNone (reads only; a list never holds more than E nodes, the
// bound only keeps a walk finite whatever the memory holds)
GS_HD inline int32_t find_node(const State& S, uint32_t v, uint32_t c) {
    uint32_t guard = 0;
    for (int32_t nd = S.vhead[v]; nd != kNone && guard < S.E; nd = S.node_next[nd], ++guard)
        if (slot_of(S.node_cs[nd]) == c) return nd;
    return kNone;
}

// a sync, then whether an error or a failure ended the operation (read by thread 0, handed to all
// through the shared block: control words are read from global memory by one thread only)
template <class X>
GS_HD inline bool stopped(X& x, const State& S, Shared& sh) {
    x.sync();
    if (x.tid() == 0) sh.stop = (S.ctl->err != 0 || S.ctl->ok == 0) ? 1u : 0u;
    x.sync();
    return sh.stop != 0;
}

// thread 0: a new, empty component keyed k (kslot[k] must be free)
GS_HD inline uint32_t new_comp(State& S, uint32_t k) {
    Ctl& c = *S.ctl;
    if (c.n_comps >= S.C) {
        c.err |= kErrCapacity;
        return 0;
    }
    const uint32_t s = c.n_comps++;
    S.comp_key[s] = k;
    S.comp_alive[s] = 1;
    S.comp_base[s] = 0;
    S.comp_size[s] = 0;
    S.comp_cap[s] = 0;
    S.kslot[k] = (int32_t)s;
    ++c.live_comps;
    return s;
}

// room for `more` members in component c: a bigger array in the arena, the old members copied
template <class X>
GS_HD inline void grow(X& x, State& S, Shared& sh, uint32_t c, uint32_t more) {
    const uint32_t size = S.comp_size[c];
    if (x.tid() == 0) {
        sh.newbase = kNoVertex;
        if (size + more > S.comp_cap[c]) {
            uint32_t nc = S.comp_cap[c] * 2;
            if (nc < size + more) nc = size + more;
            if (nc < 4) nc = 4;
            if ((uint64_t)S.ctl->n_arena + nc > S.A) {
                S.ctl->err |= kErrCapacity;
            } else {
                sh.newbase = S.ctl->n_arena;
                S.ctl->n_arena += nc;
                S.comp_cap[c] = nc;
            }
        }
    }
    x.sync();
    if (sh.newbase == kNoVertex) return;
    const uint32_t ob = S.comp_base[c], nb = sh.newbase;
    for (uint32_t i = x.tid(); i < size; i += x.nt()) S.arena[nb + i] = S.arena[ob + i];
    x.sync();
    if (x.tid() == 0) S.comp_base[c] = nb;
    x.sync();
}

// v joins component c with sign sg (v absent from c; the calling thread owns v's list)
template <class X>
GS_HD inline void add_node(X& x, State& S, uint32_t c, uint32_t v, uint32_t sg) {
    const uint32_t nd = x.atomic_add(&S.ctl->n_nodes, 1u);
    if (nd >= S.E) {
        x.atomic_or(&S.ctl->err, kErrCapacity);
        return;
    }
    S.node_cs[nd] = c | (sg << 31);
    S.node_v[nd] = v;
    S.node_next[nd] = S.vhead[v];
    S.vhead[v] = (int32_t)nd;
    const uint32_t pos = x.atomic_add(&S.comp_size[c], 1u);
    S.arena[S.comp_base[c] + pos] = (int32_t)nd;
    x.atomic_add(&S.ctl->live_entries, 1u);
}

// Candidates.getMap().remove(key) of slot c (thread 0)
GS_HD inline void kill_comp(State& S, uint32_t c) {
    S.comp_alive[c] = 0;
    if (S.kslot[S.comp_key[c]] == (int32_t)c) S.kslot[S.comp_key[c]] = kNone;
    --S.ctl->live_comps;
    S.ctl->live_entries -= S.comp_size[c];
}

// Adds the members (iv[i], is[i] ^ flip) of an input component to component c in TreeMap order,
// stopping at the first refused one (a member already in c with the other sign): the refused
// vertex is the smallest such, every smaller absent member is added. Returns (to every thread)
// whether one was refused.
template <class X>
GS_HD inline bool add_all(X& x, State& S, Shared& sh, uint32_t c, const uint32_t* iv, const uint8_t* is, uint32_t s,
                          uint32_t flip) {
    if (x.tid() == 0) sh.minc = kNoVertex;
    x.sync();
    for (uint32_t i = x.tid(); i < s; i += x.nt()) {
        const int32_t nd = find_node(S, iv[i], c);
        if (nd != kNone && sign_of(S.node_cs[nd]) != ((uint32_t)is[i] ^ flip)) x.atomic_min(&sh.minc, iv[i]);
    }
    x.sync();
    grow(x, S, sh, c, s);
    const uint32_t stop = sh.minc;
    if (stopped(x, S, sh)) return true;
    for (uint32_t i = x.tid(); i < s; i += x.nt()) {
        const uint32_t v = iv[i];
        if (v < stop && find_node(S, v, c) == kNone) add_node(x, S, c, v, (uint32_t)is[i] ^ flip);
    }
    x.sync();
    return stop != kNoVertex;
}

// The private merge(input, candidates, inputKey, selfKey) of Candidates.java:142-192 for an input
// component given as arrays, into component f: 1 = consistent and merged into component `dst`,
// 0 = inconsistent (nothing added: the check precedes the adds), 2 = merged but an add was
// refused (cannot happen after a consistent check; kept for the rule's literal shape), 3 = empty
// mergeBy (the reference throws).
template <class X>
GS_HD inline int merge_into(X& x, State& S, Shared& sh, const uint32_t* iv, const uint8_t* is, uint32_t s, uint32_t f,
                            uint32_t dst) {
    if (x.tid() == 0) { sh.minv = kNoVertex; sh.flag = 0; }
    x.sync();
    for (uint32_t i = x.tid(); i < s; i += x.nt())
        if (find_node(S, iv[i], f) != kNone) x.atomic_min(&sh.minv, iv[i]);          // mergeBy.get(0)
    x.sync();
    if (sh.minv == kNoVertex) return 3;
    for (uint32_t i = x.tid(); i < s; i += x.nt())
        if (iv[i] == sh.minv) sh.rev = ((uint32_t)is[i] != sign_of(S.node_cs[find_node(S, iv[i], f)])) ? 1u : 0u;
    x.sync();
    const uint32_t rev = sh.rev;
    for (uint32_t i = x.tid(); i < s; i += x.nt()) {                                 // :162-173
        const int32_t nd = find_node(S, iv[i], f);
        if (nd != kNone && (((uint32_t)is[i] ^ rev) != sign_of(S.node_cs[nd]))) sh.flag = 1;
    }
    x.sync();
    if (sh.flag) return 0;
    return add_all(x, S, sh, dst, iv, is, s, rev) ? 2 : 1;                           // :176-189
}

// Candidates.merge's body for ONE input component (key inKey; members iv/is, s of them) against
// this summary (:84-135). Returns false when the whole merge fails (fail(): the caller marks the
// summary failed), true otherwise (errors: S.ctl->err).
template <class X>
GS_HD inline bool merge_component(X& x, State& S, Shared& sh, uint32_t inKey, const uint32_t* iv, const uint8_t* is,
                                  uint32_t s) {
    if (x.tid() == 0) { sh.n_touched = 0; sh.n_mw = 0; }
    x.sync();
    // the candidate components that share a vertex with the input component, and how many (:88-106);
    // nodes of removed components are unlinked on the way (each thread owns its vertices' lists)
    for (uint32_t i = x.tid(); i < s; i += x.nt()) {
        const uint32_t v = iv[i];
        int32_t prev = kNone, nd = S.vhead[v];
        for (uint32_t guard = 0; nd != kNone && guard < S.E; ++guard) {
            const int32_t next = S.node_next[nd];
            const uint32_t c = slot_of(S.node_cs[nd]);
            if (!S.comp_alive[c]) {
                if (prev == kNone) S.vhead[v] = next;
                else S.node_next[prev] = next;
            } else {
                if (x.atomic_add(&S.cnt[c], 1u) == 0) S.touched[x.atomic_add(&sh.n_touched, 1u)] = c;
                prev = nd;
            }
            nd = next;
        }
    }
    x.sync();
    // components with exactly the input's vertex set are skipped (:91-95)
    const uint32_t nt = sh.n_touched;
    for (uint32_t t = x.tid(); t < nt; t += x.nt()) {
        const uint32_t c = S.touched[t];
        const uint32_t k = S.cnt[c];
        S.cnt[c] = 0;
        if (!(k == s && S.comp_size[c] == s)) S.mw[x.atomic_add(&sh.n_mw, 1u)] = ((uint64_t)S.comp_key[c] << 32) | c;
    }
    x.sync();
    const uint32_t n = sh.n_mw;
    for (uint32_t i = x.tid(); i < n; i += x.nt()) {                                 // Collections.sort (:114)
        uint32_t r = 0;
        for (uint32_t j = 0; j < n; ++j) r += S.mw[j] < S.mw[i];
        S.mws[r] = S.mw[i];
    }
    x.sync();
    if (n == 0) {                                      // disjoint from every component: add it (:108-111)
        if (x.tid() == 0) {
            int32_t c = S.kslot[inKey];
            if (c == kNone) c = (int32_t)new_comp(S, inKey);
            sh.cslot = (uint32_t)c;
        }
        if (stopped(x, S, sh)) return true;
        (void)add_all(x, S, sh, sh.cslot, iv, is, s, 0u);      // (the refusal is ignored, :111)
        return true;
    }
    const uint32_t f = (uint32_t)(S.mws[0] & 0xFFFFFFFFu), kf = (uint32_t)(S.mws[0] >> 32);
    const uint32_t common = inKey < kf ? inKey : kf;           // :123, :176
    if (x.tid() == 0) {
        int32_t c = (common == kf) ? (int32_t)f : S.kslot[common];
        if (c == kNone) c = (int32_t)new_comp(S, common);
        sh.cslot = (uint32_t)c;
    }
    if (stopped(x, S, sh)) return true;
    const uint32_t cs = sh.cslot;
    const int r1 = merge_into(x, S, sh, iv, is, s, f, cs);    // :118-121
    if (r1 == 3) {
        if (x.tid() == 0) S.ctl->err |= kErrThrows;
        x.sync();
        return true;
    }
    if (r1 != 1) return false;                                 // return fail()
    if (stopped(x, S, sh)) return true;
    for (uint32_t j = 1; j < n; ++j) {                         // :126-134
        const uint32_t ck = (uint32_t)(S.mws[j] & 0xFFFFFFFFu);
        const uint32_t sk = S.comp_size[ck], bk = S.comp_base[ck];
        // component ck as an input component (its own arrays in the scratch)
        for (uint32_t i = x.tid(); i < sk; i += x.nt()) {
            const int32_t nd = S.arena[bk + i];
            S.sv[i] = S.node_v[nd];
            S.ss[i] = (uint8_t)sign_of(S.node_cs[nd]);
        }
        x.sync();
        const int r2 = merge_into(x, S, sh, S.sv, S.ss, sk, cs, cs);
        if (r2 == 3) {
            if (x.tid() == 0) S.ctl->err |= kErrThrows;
            x.sync();
            return true;
        }
        // r2 == 0: `fail();` is called and its result dropped (:129-131): nothing was added
        if (x.tid() == 0) kill_comp(S, ck);                    // this.getMap().remove(...) (:133)
        if (stopped(x, S, sh)) return true;
    }
    return true;
}

// updateFunction.foldEdges: candidates.merge(edgeToCandidate(v1, v2)) (BipartitenessCheck.java:54-61,
// :93-95) for edges [0, n); returns after the first error
template <class X, class IdT>
GS_HD inline void fold_edges(X& x, State& S, Shared& sh, const IdT* a, const IdT* b, uint64_t n, bool aos) {
    for (uint64_t e = 0; e < n; ++e) {
        if (stopped(x, S, sh)) return;
        const IdT ra = aos ? a[2 * e] : a[e];
        const IdT rb = aos ? a[2 * e + 1] : b[e];
        if ((uint64_t)ra >= S.cap || (uint64_t)rb >= S.cap) {   // (negative int64: huge) skipped, GS_ERR_RANGE later
            if (x.tid() == 0) S.ctl->skipped |= kErrRange;
            continue;
        }
        const uint32_t u = (uint32_t)ra, v = (uint32_t)rb;
        const uint32_t lo = u < v ? u : v, hi = u < v ? v : u;
        if (x.tid() == 0) {
            // edgeToCandidate: {lo: true, hi: false}; a self-loop's (v, false) is refused and the
            // refusal ignored (Candidates.add, :61-74): {v: true}
            sh.iv[0] = lo;
            sh.is[0] = 1;
            sh.iv[1] = hi;
            sh.is[1] = 0;
        }
        x.sync();
        const uint32_t iv[2] = {sh.iv[0], sh.iv[1]};
        const uint8_t is[2] = {sh.is[0], sh.is[1]};
        if (!merge_component(x, S, sh, lo, iv, is, lo == hi ? 1u : 2u)) {
            if (x.tid() == 0) S.ctl->ok = 0;                  // Candidates.fail(): empty, f0 = false
        }
    }
    x.sync();
}

// into.merge(from) (Candidates.java:77-139): every component of `from` in key order (TreeMap)
template <class X>
GS_HD inline void merge_summaries(X& x, State& S, Shared& sh, const State& F) {
    if (x.tid() == 0 && F.ctl->ok == 0) S.ctl->ok = 0;      // :79-81
    if (stopped(x, S, sh)) return;
    // the live keys of `from`, ascending: block scans over kslot in chunks of nthreads
    if (x.tid() == 0) sh.nkeys = 0;
    x.sync();
    for (uint32_t base = 0; base < F.cap; base += x.nt()) {
        const uint32_t k = base + x.tid();
        const uint32_t live = (k < F.cap && F.kslot[k] != kNone && F.comp_alive[F.kslot[k]]) ? 1u : 0u;
        uint32_t total = 0;
        const uint32_t pos = x.scan_excl(live, &total);
        if (live) S.keys[sh.nkeys + pos] = k;
        x.sync();
        if (x.tid() == 0) sh.nkeys += total;
        x.sync();
    }
    const uint32_t nk = sh.nkeys;
    for (uint32_t q = 0; q < nk; ++q) {
        if (stopped(x, S, sh)) return;
        const uint32_t key = S.keys[q];
        const uint32_t c = (uint32_t)F.kslot[key];
        const uint32_t s = F.comp_size[c], b = F.comp_base[c];
        for (uint32_t i = x.tid(); i < s; i += x.nt()) {
            const int32_t nd = F.arena[b + i];
            S.sv[i] = F.node_v[nd];
            S.ss[i] = (uint8_t)sign_of(F.node_cs[nd]);
        }
        x.sync();
        // (merge_component's second phase reuses sv / ss for the components it folds into the
        // first, after this component's own merge is done with them)
        if (!merge_component(x, S, sh, key, S.sv, S.ss, s)) {
            if (x.tid() == 0) S.ctl->ok = 0;
            x.sync();
            return;
        }
    }
    x.sync();
}

// restoreState (SummaryAggregation.java:121-135 for this summary): on a reset state, the snapshot's
// components one after another — run r is component key rk[r] with the members (rv[i], rs[i]),
// i in [ro[r], ro[r + 1]) (distinct vertices within a run; the host groups and checks them); the
// memberships go in as the rule made them, so components may share vertices again
template <class X>
GS_HD inline void load_components(X& x, State& S, Shared& sh, const uint32_t* rk, const uint64_t* ro, uint32_t runs,
                                  const uint32_t* rv, const uint8_t* rs) {
    for (uint32_t r = 0; r < runs; ++r) {
        if (stopped(x, S, sh)) return;
        const uint64_t lo = ro[r], s = ro[r + 1] - ro[r];
        if (x.tid() == 0) sh.cslot = new_comp(S, rk[r]);
        if (stopped(x, S, sh)) return;
        const uint32_t c = sh.cslot;
        grow(x, S, sh, c, (uint32_t)s);
        if (stopped(x, S, sh)) return;
        for (uint64_t i = x.tid(); i < s; i += x.nt()) add_node(x, S, c, rv[lo + i], (uint32_t)rs[lo + i]);
        x.sync();
    }
    x.sync();
}

}  // namespace lit
}  // namespace gsgpu
