"""TEST INFRASTRUCTURE: mints tests/golden/c5_rmat24.json, the per-window emission of BASELINE.json
configs[4] ("power-law Twitter-like stream with small windows (64K edges)"; SURVEY.md section 8(d)
C5) computed by the C oracle (oracle/: the restatement of DisjointSet.java:53-131,
ConnectedComponents.java:83-85,116-125 and the Merger, SummaryAggregation.java:106-119).

Stream: RMAT scale 24, edge factor 16 (2^28 edges), seed 3, Graph500 (a,b,c,d) = (.57,.19,.19,.05),
ids scrambled (oracle/gen.c, bit-identical to the device generator gs_gen_rmat); 4,096 count windows
of 2^16 edges, P = 8 partitions per window. For every window the fixture holds the emission
checksum (sum of pair_mix(v, min-id label) over the cumulative summary's vertices), its vertex
count and its component count.

The per-window checksums come from the oracle's incremental emission tracker (oracle/emission.c,
GSO_EMIT_TRACK): a full canonical checksum of the Merger's summary costs O(|V_seen|) per window,
which 4,096 windows cannot afford. The tracker is cross-checked against that full checksum of the
reference restatement's summary every `--verify-every` windows and after the last window of every
span (the run fails on any difference). The oracle runs in spans of `--span` windows; a span that
starts at window s restores the Merger (and the tracker) from the canonical emission of window s-1
(ListCheckpointed.restoreState, SummaryAggregation.java:127-135). Run time on 8 cores: a few minutes.

    python tests/golden/make_c5.py            # writes tests/golden/c5_rmat24.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)

from make_headline import gen_span  # noqa: E402
from pyoracle import EMIT_TRACK, coracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--window-log2", type=int, default=16)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--span", type=int, default=512, help="windows per oracle run")
    ap.add_argument("--verify-every", type=int, default=128)
    ap.add_argument("--out", default=os.path.join(HERE, "c5_rmat24.json"))
    a = ap.parse_args()
    o = coracle()
    V, E, W = 1 << a.scale, a.edge_factor << a.scale, 1 << a.window_log2
    nwin = E // W
    threads = min(os.cpu_count() or 8, 16)
    sums, nvs, ncs = [], [], []
    init = None
    t0 = time.time()
    for w0 in range(0, nwin, a.span):
        ln = min(a.span, nwin - w0)
        src, dst = gen_span(o, w0 * W, ln * W, a.scale, a.seed, threads)
        r = o.run(src, dst, W, partitions=a.partitions, threads=min(a.partitions, threads), emit=EMIT_TRACK,
                  label_cap=V, want_final=True, init=init, verify_every=a.verify_every)
        del src, dst
        sums += [int(x) for x in r["checksums"]]
        nvs += [int(x) for x in r["counts"][:, 0]]
        ncs += [int(x) for x in r["counts"][:, 1]]
        lab = r["final"]
        seen = np.nonzero(lab >= 0)[0]
        init = (seen.astype(np.int64), lab[seen])
        print("windows %d-%d: %d vertices, %d components (%.0f s)" % (w0 + 1, w0 + ln, nvs[-1], ncs[-1], time.time() - t0),
              flush=True)
    out = {"generator": "rmat", "scale": a.scale, "edge_factor": a.edge_factor, "seed": a.seed,
           "window_edges": W, "windows": nwin, "partitions": a.partitions,
           "checksum": "sum over emitted (v, label) of pair_mix(v, label) mod 2^64 (oracle/disjoint_set.c gso_pair_mix)",
           "made_by": "tests/golden/make_c5.py (C oracle, incremental emission tracker cross-checked against the "
                      "summary's full canonical checksum every %d windows; spans of %d windows)" % (a.verify_every, a.span),
           "checksums": [str(x) for x in sums], "vertices": nvs, "components": ncs}
    with open(a.out, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote %s (%.0f s)" % (a.out, time.time() - t0))


if __name__ == "__main__":
    main()
