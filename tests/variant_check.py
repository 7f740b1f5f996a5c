"""Per-window parity of one fold configuration against the C oracle (run as a SUBPROCESS).

The library reads its debug variables (GSGPU_FOLD_MODE, GSGPU_RING_MIN_BITS, GSGPU_YOUNG_SPLIT,
GSGPU_FOLD_STATS; csrc/cc_api.hip) once per process, so every fold variant is checked in a process
of its own: tests/test_gpu_variants.py starts this script with one named environment and reads the
JSON line it prints. With no variable set this is the production configuration.

Streams (every one compared window by window, bit-exact, against oracle/ run with P partitions
= the reference's SummaryBulkAggregation dataflow, SummaryBulkAggregation.java:68-90):
  golden        the committed golden streams (tests/golden), dense labels per window
  rmat21        RMAT scale 21, 2^24 edges, 2^20-edge windows (checksum per window + final labels)
  er21          Erdos-Renyi n = 2^21, m = 2^22, 2^19-edge windows
  giant_switch  two vertex blocks: a giant grows in the small block first, then a bigger one in
                the other block takes over at a re-pick (the hot set and warm set must be
                dropped), then both are joined — the ring path's stale-entry hazards
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def giant_switch_stream(seed: int = 11):
    """Block A = [0, 2^19), block B = [2^20, 2^21) (ids in a 2^21 space). Windows of 2^19 edges:
    1-8 inside A (A's giant forms and is picked), 9-24 inside B (B's giant grows to twice A's and
    wins a re-pick), 25-28 both blocks, 29-32 both blocks plus a few A-B edges (the two giants
    join). Self-loops and duplicates included."""
    rng = np.random.default_rng(seed)
    W = 1 << 19
    A0, A1, B0, B1 = 0, 1 << 19, 1 << 20, 1 << 21
    src, dst = [], []

    def block(lo, hi, n):
        return rng.integers(lo, hi, n), rng.integers(lo, hi, n)

    for _ in range(8):
        s, d = block(A0, A1, W); src.append(s); dst.append(d)
    for _ in range(16):
        s, d = block(B0, B1, W); src.append(s); dst.append(d)
    for w in range(8):
        sa, da = block(A0, A1, W // 2)
        sb, db = block(B0, B1, W // 2)
        s, d = np.concatenate([sa, sb]), np.concatenate([da, db])
        if w >= 4:                                     # a few A-B edges
            k = rng.integers(0, W, 16)
            d[k] = rng.integers(B0, B1, 16)
        s[:64] = d[:64]                                # self-loops
        perm = rng.permutation(W)
        src.append(s[perm]); dst.append(d[perm])
    return np.concatenate(src).astype(np.int64), np.concatenate(dst).astype(np.int64), W, B1


def run_case(torch, oracle, name, s, d, W, cap, partitions=4):
    import gsgpu
    from pyoracle import EMIT_CHECKSUM
    want = oracle.run(s, d, W, partitions=partitions, threads=8, emit=EMIT_CHECKSUM, label_cap=cap,
                      want_final=True)
    ds = gsgpu.DisjointSet(cap, id_bits=32, stream=torch.cuda.current_stream())
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    bad = None
    for w, lo in enumerate(range(0, s.size, W)):
        ds.fold(ts[lo:lo + W], td[lo:lo + W])
        ds.close_window()
        if ds.checksum()[0] != int(want["checksums"][w]) and bad is None:
            bad = w
    final_ok = bool(np.array_equal(ds.dense().astype(np.int64), want["final"]))
    fw_bad = run_fold_windows(ds, ts, td, W, want)
    ds.close()
    return {"case": name, "windows": int(len(want["checksums"])), "first_bad_window": bad, "final_equal": final_ok,
            "fold_windows_first_bad": fw_bad, "ok": bad is None and final_ok and fw_bad is None}


def run_fold_windows(ds, ts, td, W, want):
    """gs_cc_fold_windows (bench.py's timed call; with the ring fold on, the run-ahead filter
    pipeline of cc_api.hip fold_windows_loop) in calls of 1, 2, 3, 5, 8, ... windows, each call's
    last window vs the oracle; then the whole stream in one call. Returns the first bad window."""
    nwin = len(want["checksums"])
    sizes = [1, 2, 3, 5, 8, 13]
    ds.reset()
    w0, i = 0, 0
    while w0 < nwin:
        k = min(sizes[i % len(sizes)], nwin - w0)
        lo, hi = w0 * W, min(ts.numel(), (w0 + k) * W)
        assert ds.fold_windows(ts[lo:hi], td[lo:hi], W) == k
        w0 += k
        i += 1
        if ds.checksum()[0] != int(want["checksums"][w0 - 1]):
            return w0 - 1
    ds.reset()
    assert ds.fold_windows(ts, td, W) == nwin
    if ds.checksum()[0] != int(want["checksums"][nwin - 1]) or \
            not np.array_equal(ds.dense().astype(np.int64), want["final"]):
        return nwin - 1
    return None


def rank_slices(n, W, world, share0=None):
    """Rank r's part of every window of a stream of n edges in windows of W: [(lo, hi) per window]
    per rank. share0 (GS_MERGE_PREFILTER's Merger): rank 0's fraction of each window, the rest split
    evenly; None: even slices."""
    out = [[] for _ in range(world)]
    for lo in range(0, n, W):
        ln = min(W, n - lo)
        if share0 is None or world == 1:
            cut = [lo + (ln * r) // world for r in range(world + 1)]
        else:
            c0 = max(1, int(ln * share0))
            cut = [lo] + [lo + c0 + ((ln - c0) * r) // (world - 1) for r in range(world)]
        for r in range(world):
            out[r].append((cut[r], cut[r + 1]))
    return out


def run_prefilter(torch, oracle, name, s, d, W, cap, world=4, share0=0.125, per_window=True, id_bits=32, want=None):
    """GS_MERGE_PREFILTER over an in-process group of `world` ranks on this GPU (rank 0 the Merger
    with share0 of every window, the others filtering theirs): one gs_cc_fold_windows call per
    window (rank 0's emission after each checked) or one call for the whole stream (per_window
    False: rank r's slices laid out contiguously, every window the same size per rank, final
    emission checked)."""
    import threading
    import gsgpu
    from gsgpu import Comm
    from pyoracle import EMIT_CHECKSUM
    if want is None:
        want = oracle.run(s, d, W, partitions=world, threads=8, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    nwin = len(want["checksums"])
    sl = rank_slices(s.size, W, world, share0)
    dt = np.int32 if id_bits == 32 else np.int64
    comms = Comm.local_group(world, 0)
    got, finals, errors = [], [None], []

    def rank(r):
        try:
            ds = gsgpu.DisjointSet(cap, id_bits=id_bits)
            if per_window:
                ts = torch.from_numpy(s.astype(dt)).cuda()
                td = torch.from_numpy(d.astype(dt)).cuda()
                for w, (lo, hi) in enumerate(sl[r]):
                    assert ds.fold_windows(ts[lo:hi], td[lo:hi], max(hi - lo, 1), comm=comms[r], mode="prefilter") == 1
                    if r == 0:
                        got.append(ds.checksum()[0])
            else:
                idx = np.concatenate([np.arange(lo, hi) for lo, hi in sl[r]])
                ts = torch.from_numpy(s[idx].astype(dt)).cuda()
                td = torch.from_numpy(d[idx].astype(dt)).cuda()
                Wr = sl[r][0][1] - sl[r][0][0]
                assert ds.fold_windows(ts, td, Wr, comm=comms[r], mode="prefilter") == nwin
                if r == 0:
                    got.append(ds.checksum()[0])
            if r == 0:
                finals[0] = ds.dense().astype(np.int64)
            ds.close()
        except Exception as e:                             # noqa: BLE001
            errors.append((r, repr(e)))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    hung = any(t.is_alive() for t in th)
    info = [] if hung else [c.info() for c in comms]
    if not hung:
        for c in comms:
            c.close()
    ws = [int(x) for x in want["checksums"]]
    bad = None
    if per_window:
        for w in range(min(len(got), nwin)):
            if got[w] != ws[w]:
                bad = w
                break
    ok = (not hung and not errors and bad is None and len(got) == (nwin if per_window else 1)
          and (per_window or got[0] == ws[-1]) and finals[0] is not None
          and bool(np.array_equal(finals[0], want["final"])))
    return {"case": name, "windows": nwin, "world": world, "first_bad_window": bad, "errors": errors, "hung": hung,
            "overflows": [i[5] for i in info], "ok": ok}


def main():
    import torch
    import gsgpu
    from gsgpu import ConnectedComponents, SimpleEdgeStream
    from pyoracle import coracle
    assert torch.cuda.is_available()
    oracle = coracle()
    res = []
    # golden streams (tests/golden, minted by the Python twin of DisjointSet.java, scipy-checked)
    idx = json.load(open(os.path.join(HERE, "golden", "streams_index.json")))
    z = np.load(os.path.join(HERE, "golden", "streams.npz"))
    for c in idx:
        n = c["name"]
        cc = ConnectedComponents(1000, window_edges=c["window_edges"], id_bits=32, vertex_capacity=c["cap"])
        ok = True
        for w, ds in enumerate(SimpleEdgeStream(z[n + "__src"], z[n + "__dst"]).aggregate(cc)):
            ok &= bool(np.array_equal(ds.dense().astype(np.int64), z[n + "__labels"][w]))
        res.append({"case": "golden/" + n, "ok": ok})
    s, d = oracle.gen_rmat(0, 1 << 24, 21, 5)
    res.append(run_case(torch, oracle, "rmat21", s, d, 1 << 20, 1 << 21))
    res.append(run_prefilter(torch, oracle, "rmat21_prefilter_4ranks", s, d, 1 << 20, 1 << 21, world=4))
    s, d = oracle.gen_er(0, 1 << 22, 1 << 21, 6)
    res.append(run_case(torch, oracle, "er21", s, d, 1 << 19, 1 << 21))
    res.append(run_prefilter(torch, oracle, "er21_prefilter_4ranks", s, d, 1 << 19, 1 << 21, world=4))
    s, d, W, cap = giant_switch_stream()
    res.append(run_case(torch, oracle, "giant_switch", s, d, W, cap))
    res.append(run_prefilter(torch, oracle, "giant_switch_prefilter_3ranks", s, d, W, cap, world=3))
    env = {k: v for k, v in os.environ.items() if k.startswith("GSGPU_")}
    print(json.dumps({"env": env, "ok": all(r["ok"] for r in res), "cases": res}), flush=True)


if __name__ == "__main__":
    main()
