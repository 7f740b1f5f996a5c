"""TEST INFRASTRUCTURE: mints tests/golden/headline_rmat26.json, the per-window emission of the
headline stream (BASELINE.json configs[2]) computed by the C oracle (oracle/, the restatement of
DisjointSet.java:53-131, ConnectedComponents.java:83-85,116-125 and the Merger,
SummaryAggregation.java:106-119).

Stream: RMAT scale 26, edge factor 16 (2^30 edges), seed 1, Graph500 (a,b,c,d) = (.57,.19,.19,.05),
ids scrambled (oracle/gen.c, bit-identical to the device generator gs_gen_rmat); 64 count windows
of 2^24 edges, P = 8 partitions per window (canonical labels do not depend on P: SURVEY.md section 4).
For every window w the fixture holds the emission checksum (sum of pair_mix(v, min-id label) over
the cumulative summary's vertices), its vertex count and its component count.

The oracle runs in spans of `--span` windows; a span that starts at window s restores the Merger
from the oracle's own canonical emission of window s-1 (ListCheckpointed.restoreState,
SummaryAggregation.java:127-135: union(v, label) for every emitted pair), so the whole 2^30-edge
stream never sits in host memory at once. Run time on 8 cores: a few minutes.

    python tests/golden/make_headline.py            # writes tests/golden/headline_rmat26.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from pyoracle import EMIT_CHECKSUM, _p, coracle, rmat_thresholds  # noqa: E402


def gen_span(o, first: int, n: int, scale: int, seed: int, threads: int):
    src = np.empty(n, dtype=np.int64)
    dst = np.empty(n, dtype=np.int64)
    ta, tb, tc = rmat_thresholds()
    step = (n + threads - 1) // threads

    def work(t):
        lo, hi = t * step, min(n, (t + 1) * step)
        if lo < hi:
            o.L.gso_gen_rmat(_p(src[lo:hi]), _p(dst[lo:hi]), first + lo, hi - lo, scale, seed, ta, tb, tc, 1)

    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return src, dst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--window-log2", type=int, default=24)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--span", type=int, default=8, help="windows per oracle run")
    ap.add_argument("--out", default=os.path.join(HERE, "headline_rmat26.json"))
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
        r = o.run(src, dst, W, partitions=a.partitions, threads=min(a.partitions, threads), emit=EMIT_CHECKSUM,
                  label_cap=V, want_final=True, init=init)
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
           "made_by": "tests/golden/make_headline.py (C oracle, spans of %d windows)" % a.span,
           "checksums": [str(x) for x in sums], "vertices": nvs, "components": ncs}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote %s (%.0f s)" % (a.out, time.time() - t0))


if __name__ == "__main__":
    main()
