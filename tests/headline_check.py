"""Parity of the headline configuration, run as a SUBPROCESS with a clean environment (no GSGPU_*
variable), so the production selection runs exactly as in bench.py: RMAT scale 26, edge factor
16 (2^30 edges, seed 1), 64 windows of 2^24 edges. That covers window 1's young split (an internal
close at capacity/16 edges), the auto choice of the steady fold with its LDS hot set, the warm
set's count-and-build, the incremental closes with their claim bitmap, giant re-picks every 16th
close, warm-set re-checks and periodic hot-set admission (all of which only run past window 6).

With --fixture c5 the same checks run on BASELINE.json configs[4] (RMAT scale 24, edge factor 16,
seed 3, 4,096 windows of 2^16 edges: tests/golden/c5_rmat24.json, minted by tests/golden/make_c5.py),
which exercises the small-window regime: small plain folds, incremental closes over the whole
stream, giant re-picks every 16th close and the sampled-giant closes.

Checks (BASELINE.json configs[2] on one GPU; tests/test_gpu_variants.py runs this):
  * EVERY window's emission (checksum of the canonical (vertex, min-id label) pairs, vertex count,
    component count) equals the C oracle's, committed as tests/golden/headline_rmat26.json by
    tests/golden/make_headline.py (oracle/: the restatement of DisjointSet.java:53-131 and the
    Merger, SummaryAggregation.java:106-119, which emits after every window);
  * --steps K: K back-to-back passes over the stream with gs_cc_reset between them, every window
    of every pass against the fixture (reset must leave nothing behind);
  * --id-bits 64: the reference's Long ids (ConnectedComponentsExample.java:61);
  * after the last window the dense canonical labels equal an independent torch CC of the whole
    stream (hook-to-min + pointer jumping: bench.py torch_min_labels) and are minimal/idempotent;
  * --label-windows (default 1, 2, 5, 16): the WHOLE emission of those windows — every vertex's
    canonical label, not only the checksum — equals the torch CC of the stream up to them (window 1
    the young forest, 5 the giant-root change, 16 past the warm-set build);
  * --fold-windows: bench.py's timed call itself, gs_cc_fold_windows (the per-window loop inside the
    library), from a reset over the whole stream in one call, then the last window's emission
    checksum against the fixture; again in calls of --chunk windows, each call's last window
    against the fixture; and the whole stream once more from a reset (the same result again).
Prints one JSON line.
"""
from __future__ import annotations

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "gelly-streaming_amd")):
    sys.path.insert(0, p)

FIXTURES = {"headline": (os.path.join(HERE, "golden", "headline_rmat26.json"), 26, 16, 24, 1),
            "c5": (os.path.join(HERE, "golden", "c5_rmat24.json"), 24, 16, 16, 3)}
FIXTURE = FIXTURES["headline"][0]


def load_fixture(scale, edge_factor, window_log2, seed=1, path=FIXTURE):
    fx = json.load(open(path))
    assert (fx["scale"], fx["edge_factor"], fx["window_edges"], fx["seed"]) == (scale, edge_factor, 1 << window_log2, seed), \
        "the fixture was minted for another stream"
    return [(int(s), int(v), int(c)) for s, v, c in zip(fx["checksums"], fx["vertices"], fx["components"])]


def first_bad(got, want):
    return next((i for i, (g, w) in enumerate(zip(got, want)) if tuple(g) != tuple(w)), None)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="headline", choices=sorted(FIXTURES))
    ap.add_argument("--id-bits", type=int, default=32)
    ap.add_argument("--steps", type=int, default=1, help="passes over the stream, gs_cc_reset between them")
    ap.add_argument("--no-torch", action="store_true", help="skip the final torch CC comparison")
    ap.add_argument("--variant", action="store_true", help="allow GSGPU_* variables (a named fold variant)")
    ap.add_argument("--fold-windows", action="store_true", help="also the gs_cc_fold_windows path (bench.py's timed call)")
    ap.add_argument("--chunk", type=int, default=8, help="windows per gs_cc_fold_windows call in the chunked pass")
    ap.add_argument("--label-windows", default="1,2,5,16",
                    help="windows (1-based) whose whole label array is compared with an independent torch CC of "
                         "the stream up to them (first pass; '' = none; skipped with --no-torch)")
    a = ap.parse_args()
    path, a.scale, a.edge_factor, a.window_log2, a.seed = FIXTURES[a.fixture]
    import torch
    import gsgpu
    from gsgpu import gen
    from bench import torch_min_labels
    assert torch.cuda.is_available()
    assert a.variant or not any(k.startswith("GSGPU_") and k != "GSGPU_LIB" for k in os.environ), \
        "headline_check runs with production defaults (--variant for a named fold variant)"
    want = load_fixture(a.scale, a.edge_factor, a.window_log2, a.seed, path)
    t0 = time.time()
    V, E, W = 1 << a.scale, a.edge_factor << a.scale, 1 << a.window_log2
    dt = torch.int32 if a.id_bits == 32 else torch.int64
    src = torch.empty(E, dtype=dt, device="cuda")
    dst = torch.empty(E, dtype=dt, device="cuda")
    for lo in range(0, E, W):
        gen.rmat(src[lo:lo + W], dst[lo:lo + W], lo, a.scale, a.seed)
    torch.cuda.synchronize()
    ds = gsgpu.DisjointSet(V, id_bits=a.id_bits, stream=torch.cuda.current_stream())
    passes = []
    label_windows = [] if a.no_torch else [int(x) for x in a.label_windows.split(",") if x.strip()]
    saved = {}                             # window -> its emission's dense labels (first pass)
    for step in range(a.steps):
        if step:
            ds.reset()
        got = []
        for lo in range(0, E, W):
            ds.fold(src[lo:lo + W], dst[lo:lo + W])
            ds.close_window()
            got.append(ds.checksum())
            if step == 0 and len(got) in label_windows:
                saved[len(got)] = torch.empty(V, dtype=dt, device="cuda")
                ds.dense(out=saved[len(got)])
        passes.append(got)
        print("pass %d: %d windows, first bad %s (%.1f s)" % (step, len(got), first_bad(got, want), time.time() - t0),
              file=sys.stderr, flush=True)
    ok_windows = all(len(g) == len(want) and first_bad(g, want) is None for g in passes)
    fw = None
    if a.fold_windows:                     # bench.py's timed call: the whole stream in one call ...
        ds.reset()
        nw = ds.fold_windows(src, dst, W)
        whole = ds.checksum()
        ds.reset()                         # ... and in calls of --chunk windows
        chunked = []
        for w0 in range(0, len(want), a.chunk):
            hi = min(len(want), w0 + a.chunk)
            ds.fold_windows(src[w0 * W:hi * W], dst[w0 * W:hi * W], W)
            chunked.append((hi - 1, ds.checksum()))
        bad = [w for w, g in chunked if tuple(g) != tuple(want[w])]
        ds.reset()                         # ... and the whole stream again from a reset
        nw2 = ds.fold_windows(src, dst, W)
        again = ds.checksum()
        fw = {"windows": nw, "whole_ok": nw == len(want) and tuple(whole) == tuple(want[-1]) and
              nw2 == nw and tuple(again) == tuple(whole),
              "chunked_ok": not bad, "chunked_first_bad": bad[0] if bad else None, "chunks": len(chunked),
              "final_checksum": str(whole[0])}
        print("fold_windows: %s (%.1f s)" % (fw, time.time() - t0), file=sys.stderr, flush=True)
    t_gpu = time.time() - t0
    lab = torch.empty(V, dtype=dt, device="cuda")
    ds.dense(out=lab)
    lab = lab.long()
    seen = lab >= 0
    v = torch.arange(V, device="cuda")
    minimal = bool((lab[seen] <= v[seen]).all()) and bool((lab[lab[seen]] == lab[seen]).all())
    torch_ok = None
    if not a.no_torch:
        ref = torch_min_labels(src, dst, V)
        torch_ok = bool(torch.equal(lab, ref))
        del ref
    # whole emissions of chosen windows (not only their checksums) vs torch CC of the stream prefix
    window_labels = {}
    for w, got_lab in sorted(saved.items()):
        ref = torch_min_labels(src[:w * W], dst[:w * W], V)
        window_labels[w] = bool(torch.equal(got_lab.long(), ref))
        del ref
    nv, nc = ds.stats()
    out = {"fixture": a.fixture, "scale": a.scale, "edges": E, "window_edges": W, "windows": len(want), "id_bits": a.id_bits,
           "steps": a.steps, "fixture_windows_equal": ok_windows,
           "first_bad": [first_bad(g, want) for g in passes],
           "fold_windows": fw, "final_equals_torch_cc": torch_ok, "labels_minimal_idempotent": minimal,
           "window_labels_equal_torch_cc": window_labels,
           "final_vertices": nv, "final_components": nc,
           "fixture_final": list(want[-1][1:]),
           "seconds": {"gpu": round(t_gpu, 1), "total": round(time.time() - t0, 1)}}
    out["ok"] = ok_windows and torch_ok is not False and minimal and (nv, nc) == tuple(want[-1][1:]) and \
        all(window_labels.values()) and \
        (fw is None or (fw["whole_ok"] and fw["chunked_ok"]))
    ds.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
