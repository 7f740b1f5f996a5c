"""Parity of the headline configuration, run as a SUBPROCESS with a clean environment (no GSGPU_*
variable), so the production selection runs exactly as in bench.py: RMAT scale 26, edge factor
16 (2^30 edges, seed 1), int32 ids, 64 windows of 2^24 edges. That covers window 1's young split
(an internal close at capacity/16 edges), the auto choice of the ring fold with its LDS hot set,
the warm set's count-and-build in window 5, and the incremental closes.

Checks (BASELINE.json configs[2] on one GPU; tests/test_gpu_variants.py runs this):
  * the emission checksum of windows 1..K equals the C oracle's (oracle/, the restatement of
    DisjointSet.java:53-131 / SummaryAggregation.java:106-119) on the same edges, P partitions;
  * after all 64 windows the dense canonical labels equal an independent torch CC of the whole
    stream (hook-to-min + pointer jumping: bench.py torch_min_labels) and are minimal/idempotent;
  * the final vertex and component counts.
Prints one JSON line.
"""
from __future__ import annotations

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--window-log2", type=int, default=24)
    ap.add_argument("--oracle-windows", type=int, default=6)
    ap.add_argument("--id-bits", type=int, default=32)
    a = ap.parse_args()
    import numpy as np
    import torch
    import gsgpu
    from gsgpu import gen
    from pyoracle import EMIT_CHECKSUM, coracle
    from bench import torch_min_labels
    assert torch.cuda.is_available()
    assert not any(k.startswith("GSGPU_") and k != "GSGPU_LIB" for k in os.environ), "headline_check runs with production defaults"
    t0 = time.time()
    V, E, W = 1 << a.scale, a.edge_factor << a.scale, 1 << a.window_log2
    dt = torch.int32 if a.id_bits == 32 else torch.int64
    src = torch.empty(E, dtype=dt, device="cuda")
    dst = torch.empty(E, dtype=dt, device="cuda")
    for lo in range(0, E, W):
        gen.rmat(src[lo:lo + W], dst[lo:lo + W], lo, a.scale, 1)
    torch.cuda.synchronize()
    ds = gsgpu.DisjointSet(V, id_bits=a.id_bits, stream=torch.cuda.current_stream())
    sums = []
    for lo in range(0, E, W):
        ds.fold(src[lo:lo + W], dst[lo:lo + W])
        ds.close_window()
        sums.append(ds.checksum())
    t_gpu = time.time() - t0
    K = a.oracle_windows
    hs = src[:K * W].cpu().numpy().astype(np.int64)
    hd = dst[:K * W].cpu().numpy().astype(np.int64)
    threads = min(os.cpu_count() or 8, 16)
    want = coracle().run(hs, hd, W, partitions=threads, threads=threads, emit=EMIT_CHECKSUM, label_cap=V)
    del hs, hd
    t_oracle = time.time() - t0 - t_gpu
    got = [s[0] for s in sums[:K]]
    oracle_ok = got == [int(x) for x in want["checksums"]]
    lab = torch.empty(V, dtype=dt, device="cuda")
    ds.dense(out=lab)
    lab = lab.long()
    seen = lab >= 0
    v = torch.arange(V, device="cuda")
    minimal = bool((lab[seen] <= v[seen]).all()) and bool((lab[lab[seen]] == lab[seen]).all())
    ref = torch_min_labels(src, dst, V)
    torch_ok = bool(torch.equal(lab, ref))
    nv, nc = ds.stats()
    out = {"scale": a.scale, "edges": E, "window_edges": W, "windows": len(sums), "id_bits": a.id_bits,
           "oracle_windows": K, "oracle_checksums_equal": oracle_ok,
           "first_bad_window": next((i for i, (g, w) in enumerate(zip(got, want["checksums"])) if g != int(w)), None),
           "final_equals_torch_cc": torch_ok, "labels_minimal_idempotent": minimal,
           "final_vertices": nv, "final_components": nc,
           "torch_vertices": int((ref >= 0).sum().item()), "torch_components": int((ref[ref >= 0] == v[ref >= 0]).sum().item()),
           "seconds": {"gpu": round(t_gpu, 1), "oracle": round(t_oracle, 1), "total": round(time.time() - t0, 1)}}
    out["ok"] = oracle_ok and torch_ok and minimal and nv == out["torch_vertices"] and nc == out["torch_components"]
    ds.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
