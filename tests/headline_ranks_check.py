"""BASELINE config 3's multi-GPU layout at full scale, on one GPU: the RMAT-26 EF16 stream (seed 1,
int32 ids), 2^24-edge GLOBAL windows split over P ranks (rank r folds slice r of every window: the
PartitionMapper split, SummaryBulkAggregation.java:76-80,93-106; bench.py --scaling strong), every
window exchanged and closed through the C ABI (gs_cc_merge_window) in the chosen mode:
  allgather  every rank keeps the global summary (replicated Merger): every rank is checked;
  gather     the windowAll gather to rank 0 (SummaryBulkAggregation.java:81-83): rank 0 is checked;
  tree       ConnectedComponentsTree's pairwise rounds (SummaryTreeReduce.java:95-123): rank 0;
  prefilter  ranks 1..P-1 filter their slices against rank 0's broadcast giant bitmap (with their own
             hot / warm sets at these ids) and send the survivors; rank 0 takes bench.py's default
             share of each window, folds everything and emits (gs_cc_fold_windows per window): rank 0.
RCCL cannot put several ranks on one GPU, so the ranks are threads over the in-process transport
(gs_comm_create_local): the same exchange code, collectives as device copies.

Checks, printed as one JSON line:
  * the Merger's emission after EVERY window (checksum, vertices, components) equals the C
    oracle's, committed as tests/golden/headline_rmat26.json (canonical labels do not depend on the
    partitioning, SURVEY.md section 4, so the single-summary fixture pins every layout);
  * after the last window the checked ranks' dense labels are identical and equal an independent
    torch CC of the same edges (bench.py torch_min_labels);
  * no speculative slot overflow after the first steady windows is required (reported only).
Run in a subprocess with no GSGPU_* variable (production selection) by tests/test_gpu_variants.py.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "gelly-streaming_amd")):
    sys.path.insert(0, p)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--windows", type=int, default=64, help="global windows folded (a prefix of the fixture)")
    ap.add_argument("--mode", default="allgather", choices=["allgather", "gather", "tree", "prefilter"])
    ap.add_argument("--no-torch", action="store_true")
    a = ap.parse_args()
    import torch
    import gsgpu
    from gsgpu import Comm, gen
    from bench import torch_min_labels
    from headline_check import first_bad, load_fixture
    assert torch.cuda.is_available()
    assert not any(k.startswith("GSGPU_") and k != "GSGPU_LIB" for k in os.environ), "production defaults"
    want = load_fixture(a.scale, 16, 24)[:a.windows]
    t0 = time.time()
    P, V, W, N = a.ranks, 1 << a.scale, 1 << 24, a.windows
    src = torch.empty(N * W, dtype=torch.int32, device="cuda")
    dst = torch.empty(N * W, dtype=torch.int32, device="cuda")
    for w in range(N):
        gen.rmat(src[w * W:(w + 1) * W], dst[w * W:(w + 1) * W], w * W, a.scale, 1)
    torch.cuda.synchronize()
    comms = Comm.local_group(P, 0)
    checked = list(range(P)) if a.mode == "allgather" else [0]
    sums = [[] for _ in range(P)]
    finals = [None] * P
    errors = []
    Wr = W // P
    pre = a.mode == "prefilter"
    if pre:                                   # bench.py's prefilter layout (its default share for rank 0:
        import bench                          # none at P = 8, rank 0 then only merges)

        class _L:
            edge_factor, scale, window_log2, scaling, share0, merge = 16, a.scale, 24, "strong", None, "prefilter"
        sl = []
        for q in range(P):
            lay = bench.layout(_L, P, q)      # (edges, slice, global window, windows, stream, offset)
            sl.append((lay[5], lay[1]))
    else:
        sl = [(q * Wr, Wr) for q in range(P)]

    def rank(r):
        try:
            ds = gsgpu.DisjointSet(V, id_bits=32, track_marks=not pre)
            off, ln = sl[r]
            for w in range(N):
                lo = w * W + off
                if pre:
                    ds.fold_windows(src[lo:lo + ln], dst[lo:lo + ln], max(ln, 1), comm=comms[r], mode="prefilter")
                else:
                    ds.fold(src[lo:lo + ln], dst[lo:lo + ln])
                    ds.merge_window(comms[r], a.mode)
                if r in checked:
                    sums[r].append(ds.checksum())
            if r in checked:
                lab = torch.empty(V, dtype=torch.int32, device="cuda")
                ds.dense(out=lab)
                torch.cuda.synchronize()
                finals[r] = lab
            ds.close()
        except Exception as e:            # reported below
            errors.append((r, repr(e)))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=900)
    hung = any(t.is_alive() for t in th)
    info = [c.info() for c in comms] if not hung else []
    if not hung:
        for c in comms:
            c.close()
    t_gpu = time.time() - t0
    out = {"ranks": P, "scale": a.scale, "global_window": W, "windows": N, "mode": a.mode, "checked_ranks": checked,
           "hung": hung, "errors": errors}
    if hung or errors:
        out["ok"] = False
        print(json.dumps(out), flush=True)
        return
    bad = {r: first_bad(sums[r], want) for r in checked}
    fixture_ok = all(len(sums[r]) == N and bad[r] is None for r in checked)
    replicas_equal = all(torch.equal(finals[checked[0]], finals[r]) for r in checked[1:])
    torch_ok = None
    if not a.no_torch:
        ref = torch_min_labels(src, dst, V)
        torch_ok = bool(torch.equal(finals[0].long(), ref))
    out.update({"fixture_windows_equal": fixture_ok, "first_bad": bad, "replicas_equal": replicas_equal,
                "final_equals_torch_cc": torch_ok,
                "overflow_rounds": [i[5] for i in info],
                "bytes_sent_rank0": info[0][2],
                "seconds": {"gpu": round(t_gpu, 1), "total": round(time.time() - t0, 1)}})
    out["ok"] = fixture_ok and replicas_equal and torch_ok is not False
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
