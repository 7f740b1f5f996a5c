"""BASELINE config 3's multi-GPU layout at full scale, on one GPU: the RMAT-26 EF16 stream (seed 1,
int32 ids), 2^24-edge GLOBAL windows split over P ranks (rank r folds slice r of every window: the
PartitionMapper split, SummaryBulkAggregation.java:76-80,93-106; bench.py --scaling strong), every
window exchanged and closed through the C ABI (gs_cc_merge_window) in allgather mode. RCCL cannot
put several ranks on one GPU, so the ranks are threads over the in-process transport
(gs_comm_create_local): the same exchange code, collectives as device copies.

Checks, printed as one JSON line:
  * every rank's emission checksum of windows 1..K equals the C oracle's with P partitions
    (oracle/, the restatement of DisjointSet.java:53-131 / SummaryAggregation.java:106-119);
  * after N windows every rank's dense labels are identical (replicated Merger) and equal an
    independent torch CC of the same N x 2^24 edges (bench.py torch_min_labels).
Run in a subprocess with no GSGPU_* variable (production selection: young split, ring fold, warm
set) by tests/test_gpu_variants.py.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--windows", type=int, default=12, help="global windows folded (N)")
    ap.add_argument("--oracle-windows", type=int, default=3, help="windows checked against the oracle (K)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import gsgpu
    from gsgpu import Comm, gen
    from pyoracle import EMIT_CHECKSUM, coracle
    from bench import torch_min_labels
    assert torch.cuda.is_available()
    assert not any(k.startswith("GSGPU_") and k != "GSGPU_LIB" for k in os.environ), "production defaults"
    t0 = time.time()
    P, V, W, N, K = a.ranks, 1 << a.scale, 1 << 24, a.windows, a.oracle_windows
    src = torch.empty(N * W, dtype=torch.int32, device="cuda")
    dst = torch.empty(N * W, dtype=torch.int32, device="cuda")
    for w in range(N):
        gen.rmat(src[w * W:(w + 1) * W], dst[w * W:(w + 1) * W], w * W, a.scale, 1)
    torch.cuda.synchronize()
    comms = Comm.local_group(P, 0)
    sums = [[] for _ in range(P)]
    finals = [None] * P
    errors = []
    Wr = W // P

    def rank(r):
        try:
            ds = gsgpu.DisjointSet(V, id_bits=32, track_marks=True)
            for w in range(N):
                lo = w * W + r * Wr
                ds.fold(src[lo:lo + Wr], dst[lo:lo + Wr])
                ds.merge_window(comms[r], "allgather")
                if w < K:
                    sums[r].append(ds.checksum()[0])
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
        t.join(timeout=600)
    hung = any(t.is_alive() for t in th)
    info = [c.info() for c in comms] if not hung else []
    if not hung:
        for c in comms:
            c.close()
    t_gpu = time.time() - t0
    out = {"ranks": P, "scale": a.scale, "global_window": W, "windows": N, "oracle_windows": K,
           "hung": hung, "errors": errors}
    if hung or errors:
        out["ok"] = False
        print(json.dumps(out), flush=True)
        return
    hs = src[:K * W].cpu().numpy().astype(np.int64)
    hd = dst[:K * W].cpu().numpy().astype(np.int64)
    threads = min(os.cpu_count() or 8, 16)
    want = coracle().run(hs, hd, W, partitions=P, threads=min(threads, P), emit=EMIT_CHECKSUM, label_cap=V)
    del hs, hd
    wsum = [int(x) for x in want["checksums"]]
    oracle_ok = all(sums[r] == wsum for r in range(P))
    replicas_equal = all(torch.equal(finals[0], finals[r]) for r in range(1, P))
    ref = torch_min_labels(src, dst, V)
    torch_ok = bool(torch.equal(finals[0].long(), ref))
    out.update({"oracle_checksums_equal": oracle_ok, "replicas_equal": replicas_equal, "final_equals_torch_cc": torch_ok,
                "first_bad": next(([r, i] for r in range(P) for i, (g, x) in enumerate(zip(sums[r], wsum)) if g != x), None),
                "overflow_rounds": [i[5] for i in info],
                "bytes_sent_rank0": info[0][2],
                "seconds": {"gpu": round(t_gpu, 1), "total": round(time.time() - t0, 1)}})
    out["ok"] = oracle_ok and replicas_equal and torch_ok
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
