// cc_internal.hpp — what comm.hip needs of a summary handle (defined in cc_api.hip), declared once.
#pragma once

#include "common.hpp"

namespace gsgpu {
struct CcInfo {
    uint32_t cap;
    int device;
    hipStream_t stream;
    bool marks;              // created with GS_CC_TRACK_MARKS
    bool sparse;
    bool marking;            // marking currently on (gs_cc_set_marking)
    uint64_t reset_gen;      // gs_cc_reset calls so far: a new stream starts when it changes
    uint32_t id_bits;        // the handle's id width (gs_cc_config.id_bits)
};
int cc_info(gs_cc_t* h, CcInfo* out);
int cc_export_async(gs_cc_t* h, void* pairs, uint64_t cap, unsigned long long* dcount, uint64_t expect = ~0ull);
// caps (host array, nslots entries, or null = every slot holds cap pairs): slot q's own capacity
int cc_fold_slots(gs_cc_t* h, const uint32_t* slots, uint64_t slot_words, int nslots, int skip, uint64_t cap,
                  const uint64_t* caps = nullptr);
void cc_count_folded(gs_cc_t* h, uint64_t n);
// folds n exported partial-summary pairs (device buffer) as CombineCC does: uint32 (vertex, root)
// pairs for dense handles, int64 (id, root id) pairs for sparse-id handles; timed as a merge
int cc_fold_pairs_any(gs_cc_t* h, const void* pairs, uint64_t n);
// partition pre-filter (GS_MERGE_PREFILTER senders): survivors of n SoA edges against the handle's
// giant filter as (u, v) uint32 pairs behind the u64 count word *dcount (zeroed first)
int cc_filter_async(gs_cc_t* h, const void* a, const void* b, uint64_t n, void* out, uint64_t cap,
                    unsigned long long* dcount);
// the giant filter state a Merger broadcasts: gbits (words, bytes) and the 2-word giant slot the
// next fold reads; cc_install_giant puts broadcast slot words (device) in place on a sending rank
int cc_filter_state(gs_cc_t* h, uint32_t** gbits, uint64_t* gbits_bytes, uint32_t** giant_words);
int cc_install_giant(gs_cc_t* h, const uint32_t* words);
// the exchange of one window whose own edges the exchange needs (comm.hip: GS_MERGE_PREFILTER);
// the rank of a communicator
int cc_merge_edges(gs_cc_t* h, gs_comm_t* c, int mode, const void* a, const void* b, uint64_t m);
int cc_comm_rank(const gs_comm_t* c);
int cc_agree_windows(gs_cc_t* h, gs_comm_t* c, uint64_t mine, uint64_t* most);
// a pending exchange verification of the handle's last window (comm.hip): cc_settle runs it once
void cc_set_settle(gs_cc_t* h, int (*fn)(void*), void* ctx);
int cc_settle(gs_cc_t* h);
// per-handle state of the streaming text ingestion (parse.hip gs_cc_fold_text / _file): made on
// first use, kept for the next call, freed by gs_cc_destroy through free_fn
void* cc_ingest_get(gs_cc_t* h);
void cc_ingest_set(gs_cc_t* h, void* p, void (*free_fn)(void*));
}  // namespace gsgpu
