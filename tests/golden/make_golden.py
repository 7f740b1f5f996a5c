"""Mint the golden fixtures under tests/golden/ (run in the build container; committed outputs).

Sources of truth, in order:
1. The reference's own known-answer tests (transcribed as data, not code):
   - src/test/java/org/apache/flink/graph/streaming/util/DisjointSetTest.java:37-78
   - src/test/java/org/apache/flink/graph/streaming/example/test/ConnectedComponentsTest.java:41,54-63
   - src/main/java/org/apache/flink/graph/streaming/example/ConnectedComponentsExample.java:121-127
     (built-in sample stream (k, k+2), timestamps k*100, merge window 1000 ms)
2. Seeded random streams: expected per-window canonical emissions computed with the Python twin
   of DisjointSet (oracle/pyoracle.py: py_cc_stream) AND independently with
   scipy.sparse.csgraph.connected_components on every window prefix; the script asserts both
   agree before writing anything.
3. Generator vectors: the first edges of the counter-based RMAT / ER streams from oracle/gen.c.

Usage: python tests/golden/make_golden.py   (writes tests/golden/*.json, *.npz)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
from scipy.sparse import coo_matrix
from scipy.sparse.csgraph import connected_components

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from pyoracle import (PyDisjointSet, canonical_to_dense, coracle, dense_checksum,  # noqa: E402
                      py_cc_stream)


def scipy_canonical(src, dst, cap):
    """dense min-id labels of the graph (src,dst) over [0,cap), -1 for vertices with no edge."""
    out = np.full(cap, -1, dtype=np.int64)
    if len(src) == 0:
        return out
    m = coo_matrix((np.ones(len(src)), (src, dst)), shape=(cap, cap))
    k, lab = connected_components(m, directed=False)
    mins = np.full(k, cap, dtype=np.int64)
    np.minimum.at(mins, lab, np.arange(cap))
    seen = np.zeros(cap, dtype=bool)
    seen[src] = True
    seen[dst] = True
    out[seen] = mins[lab[seen]]
    return out


def kat_fixtures():
    # DisjointSetTest
    ds = PyDisjointSet()
    for i in range(8):
        ds.union(i, i + 2)
    assert len(ds.getMatches()) == 10
    r0, r1 = ds.find(0), ds.find(1)
    assert r0 != r1 and all(ds.find(i) == (r0 if i % 2 == 0 else r1) for i in range(10))
    ds2 = PyDisjointSet()
    for i in range(8):
        ds2.union(i, i + 100)
    ds2.merge(ds)
    assert len(ds2.getMatches()) == 18
    assert len({ds2.find(e) for e in ds2.getMatches()}) == 2
    dstest = {
        "source": "src/test/java/org/apache/flink/graph/streaming/util/DisjointSetTest.java:37-78",
        "setup_unions": [[i, i + 2] for i in range(8)],
        "expect_matches_size": 10,
        "expect_even_odd_roots_distinct": True,
        "merge_unions": [[i, i + 100] for i in range(8)],
        "expect_merged_size": 18,
        "expect_merged_roots": 2,
    }
    # ConnectedComponentsTest
    edges = [[1, 2], [1, 3], [2, 3], [1, 5], [6, 7], [8, 9]]
    canon = py_cc_stream([e[0] for e in edges], [e[1] for e in edges], 0, 1)[-1]
    comps = {}
    for v, l in canon.items():
        comps.setdefault(l, []).append(v)
    parsed = sorted(", ".join(str(x) for x in sorted(m)) for m in comps.values())
    assert parsed == ["1, 2, 3, 5", "6, 7", "8, 9"], parsed
    cctest = {
        "source": "src/test/java/org/apache/flink/graph/streaming/example/test/ConnectedComponentsTest.java:41,54-63",
        "edges": edges,
        "expect_final_components": ["1, 2, 3, 5", "6, 7", "8, 9"],
    }
    # ConnectedComponentsExample built-in sample stream
    ks = list(range(1, 101))
    src = ks
    dst = [k + 2 for k in ks]
    ts = [k * 100 for k in ks]
    final = py_cc_stream(src, dst, 0, 1)[-1]
    assert len(final) == 102
    assert all(l == (1 if v % 2 else 2) for v, l in final.items())
    # event-time tumbling windows of 1000 ms (window id = ts // 1000): 11 windows
    wid = [t // 1000 for t in ts]
    bounds = [0] + [i for i in range(1, len(wid)) if wid[i] != wid[i - 1]] + [len(wid)]
    per_window = []
    ds = PyDisjointSet()
    for a, b in zip(bounds[:-1], bounds[1:]):
        for i in range(a, b):
            ds.union(src[i], dst[i])
        per_window.append({"edges": [a, b], "n_vertices": len(ds.getMatches()),
                           "max_vertex": max(ds.getMatches())})
    example = {
        "source": "src/main/java/org/apache/flink/graph/streaming/example/ConnectedComponentsExample.java:121-127",
        "src": src, "dst": dst, "timestamps": ts, "merge_window_ms": 1000,
        "expect_final_vertices": 102,
        "expect_final_labels": "odd -> 1, even -> 2",
        "event_time_windows": per_window,
        "note": "Only the final emission is pinned by the reference (its windows are ingestion-time); "
                "the 11 event-time windows are this build's deterministic windowing.",
    }
    # BipartitenessCheckTest: edges and the expected emission strings, as the test holds them
    bip = {
        "source": "src/test/java/org/apache/flink/graph/streaming/example/test/BipartitenessCheckTest.java:35-90",
        "bipartite_edges": [[1, 2], [1, 3], [1, 4], [4, 5], [4, 7], [4, 9]],
        "bipartite_expect": ["(true,{1={1=(1,true), 2=(2,false), 3=(3,false), 4=(4,false), 5=(5,true), "
                             "7=(7,true), 9=(9,true)}})"],
        "non_bipartite_edges": [[1, 2], [2, 3], [3, 1], [4, 5], [5, 7], [4, 1]],
        "non_bipartite_expect": ["(false,{})"],
        "merge_window_ms": 500,
        "note": "env.setParallelism(1); one 500 ms ingestion-time window holds the whole collection, "
                "so each test pins exactly one emission.",
    }
    return {"DisjointSetTest": dstest, "ConnectedComponentsTest": cctest, "ConnectedComponentsExample": example,
            "BipartitenessCheckTest": bip}


def random_cases():
    rng = np.random.default_rng(20240611)
    cases = []

    def add(name, src, dst, cap, window_edges, partitions):
        src = np.asarray(src, dtype=np.int64)
        dst = np.asarray(dst, dtype=np.int64)
        emis = py_cc_stream(src.tolist(), dst.tolist(), window_edges, partitions)
        W = window_edges if window_edges > 0 else max(len(src), 1)
        labels = np.full((max(len(emis), 1), cap), -1, dtype=np.int64)
        for w, c in enumerate(emis):
            labels[w] = canonical_to_dense(c, cap)
            hi = min((w + 1) * W, len(src))
            ref = scipy_canonical(src[:hi], dst[:hi], cap)
            assert (ref == labels[w]).all(), (name, w)
        cases.append(dict(name=name, src=src, dst=dst, cap=cap, window_edges=window_edges,
                          partitions=partitions, labels=labels[: len(emis)],
                          checksums=np.array([dense_checksum(labels[w])[0] for w in range(len(emis))],
                                             dtype=np.uint64)))

    add("er_small", rng.integers(0, 64, 200), rng.integers(0, 64, 200), 64, 32, 3)
    add("er_sparse_many_components", rng.integers(0, 500, 300), rng.integers(0, 500, 300), 512, 50, 4)
    o = coracle()
    s, d = o.gen_rmat(0, 3000, 9, 7)
    add("rmat9", s, d, 512, 256, 4)
    loops = rng.integers(0, 40, 120)
    add("self_loops_and_dups", np.concatenate([loops, loops[:30], [5, 5, 7]]),
        np.concatenate([loops, loops[:30] ^ 1, [5, 5, 7]]), 64, 17, 2)
    add("max_id", [0, 1023, 1022, 1023, 511], [1023, 1022, 1022, 1023, 0], 1024, 2, 2)
    add("single_edge", [3], [4], 8, 1, 1)
    add("chain_long_paths", np.arange(0, 255), np.arange(1, 256), 256, 64, 3)
    add("reverse_chain", np.arange(255, 0, -1), np.arange(254, -1, -1), 256, 100, 1)
    add("star_hub", np.zeros(200, dtype=np.int64), rng.integers(1, 300, 200), 300, 40, 5)
    return cases


def main():
    kats = kat_fixtures()
    with open(os.path.join(HERE, "reference_kats.json"), "w") as f:
        json.dump(kats, f, indent=1)
    cases = random_cases()
    arrays = {}
    index = []
    for c in cases:
        n = c["name"]
        for k in ("src", "dst", "labels", "checksums"):
            arrays["%s__%s" % (n, k)] = c[k]
        index.append({k: c[k] for k in ("name", "cap", "window_edges", "partitions")})
    np.savez_compressed(os.path.join(HERE, "streams.npz"), **arrays)
    with open(os.path.join(HERE, "streams_index.json"), "w") as f:
        json.dump(index, f, indent=1)
    o = coracle()
    s, d = o.gen_rmat(0, 64, 20, 1)
    s2, d2 = o.gen_rmat(1 << 20, 64, 26, 1)
    e, f_ = o.gen_er(0, 64, 1 << 24, 2)
    s3, d3 = o.gen_rmat(5, 64, 12, 9, scramble=False)
    gen = {"rmat_s20_seed1_first0": [s.tolist(), d.tolist()],
           "rmat_s26_seed1_first1M": [s2.tolist(), d2.tolist()],
           "er_n2^24_seed2_first0": [e.tolist(), f_.tolist()],
           "rmat_s12_seed9_first5_noscramble": [s3.tolist(), d3.tolist()]}
    with open(os.path.join(HERE, "generators.json"), "w") as f:
        json.dump(gen, f)
    print("wrote", len(cases), "stream cases")


if __name__ == "__main__":
    main()
