"""CPU: the BipartitenessCheck oracle (oracle/bipartite.py) pinned by the reference's known answers
(BipartitenessCheckTest.java:35-90) and cross-checked: literal restatement of Candidates vs the
intended semantics vs an independent BFS 2-colouring."""
import json
import os

import numpy as np
import pytest

from bipartite import (LiteralCandidates, bfs_bipartition, emission_string, intended_run, literal_run)

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _kat():
    return json.load(open(os.path.join(GOLD, "reference_kats.json")))["BipartitenessCheckTest"]


@pytest.mark.parametrize("which", ["bipartite", "non_bipartite"])
def test_reference_kats_literal_and_intended(which):
    k = _kat()
    e = np.array(k[which + "_edges"])
    assert literal_run(e[:, 0], e[:, 1], 0) == k[which + "_expect"]
    assert [emission_string(*x) for x in intended_run(e[:, 0], e[:, 1], 0)] == k[which + "_expect"]


def _bfs_ordered_tree_stream(nv: int, extra: int, seed: int, odd_chord: bool):
    """Edges in an order that never reaches Candidates.merge's split branch: every edge's smaller
    endpoint is already in a component keyed no higher (BFS from vertex 0 over increasing ids)."""
    rng = np.random.default_rng(seed)
    parent = [0] + [int(rng.integers(0, v)) for v in range(1, nv)]       # parent < child
    depth = [0] * nv
    for v in range(1, nv):
        depth[v] = depth[parent[v]] + 1
    src, dst = [], []
    for v in range(1, nv):
        src.append(parent[v]); dst.append(v)
    for _ in range(extra):                                               # even chords keep it bipartite
        a, b = sorted(int(x) for x in rng.integers(0, nv, 2))
        if a != b and (depth[a] + depth[b]) % 2 == 1:
            src.append(a); dst.append(b)
    if odd_chord:
        a, b = [(x, y) for x in range(nv) for y in range(x + 1, nv) if (depth[x] + depth[y]) % 2 == 0][0]
        src.append(a); dst.append(b)
    return np.array(src), np.array(dst)


@pytest.mark.parametrize("seed,odd", [(1, False), (2, False), (3, True), (4, False)])
def test_literal_equals_intended_where_the_reference_is_consistent(seed, odd):
    """One window, one partition (the reference tests' setting): every fold merges a one-edge
    candidate whose key is >= the key of the component it joins."""
    s, d = _bfs_ordered_tree_stream(60, 40, seed, odd)
    assert literal_run(s, d, 0) == [emission_string(*x) for x in intended_run(s, d, 0)]


def test_literal_windows_diverge():
    """Across windows the reference's Merger merges the cumulative summary INTO the window's
    candidates (summary = window.merge(summary), SummaryAggregation.java:110): the older
    component arrives as the input with the smaller key, so its signs are flipped to the
    window's orientation and the window's component survives beside it (Candidates.java:117-126).
    The intended emission keys each component once with its minimum vertex signed true."""
    s, d = _bfs_ordered_tree_stream(15, 0, 1, False)
    lit = literal_run(s, d, 7)
    ref = [emission_string(*x) for x in intended_run(s, d, 7)]
    assert lit[0] == ref[0] and lit[1] != ref[1]
    assert "0=(0,false)" in lit[1] and "0=(0,true)" in ref[1]


@pytest.mark.parametrize("seed", range(6))
def test_intended_equals_bfs_colouring(seed):
    rng = np.random.default_rng(100 + seed)
    nv = 300
    # random bipartite graph (sides by a hidden colouring), sometimes with one odd edge
    col = rng.integers(0, 2, nv)
    s, d = [], []
    while len(s) < 500:
        a, b = (int(x) for x in rng.integers(0, nv, 2))
        if col[a] != col[b]:
            s.append(a); d.append(b)
    if seed % 2:
        same = [(a, b) for a in range(nv) for b in range(a + 1, nv) if col[a] == col[b]][seed]
        s.append(same[0]); d.append(same[1])
    got = intended_run(np.array(s), np.array(d), 0)[-1]
    assert got == bfs_bipartition(s, d)


def test_literal_split_branch_is_reachable():
    """Documented divergence (oracle/bipartite.py header): edges (5,7), (3,7), (3,5) form a
    triangle; the literal Candidates keeps {3,7} and {5,7} apart after (3,7) and then loses the
    odd cycle, the intended semantics report non-bipartite."""
    lit = literal_run(np.array([5, 3, 3]), np.array([7, 7, 5]), 0)
    assert lit == ["(true,{3={3=(3,true), 5=(5,false), 7=(7,false)}})"]
    assert emission_string(*intended_run(np.array([5, 3, 3]), np.array([7, 7, 5]), 0)[-1]) == "(false,{})"
    c = LiteralCandidates(True)
    assert c.to_string() == "(true,{})"


def test_self_loops_only_add_vertices():
    assert literal_run(np.array([3, 1]), np.array([3, 2]), 0) == ["(true,{1={1=(1,true), 2=(2,false)}, 3={3=(3,true)}})"]
    assert [emission_string(*x) for x in intended_run(np.array([3, 1]), np.array([3, 2]), 0)] == \
        ["(true,{1={1=(1,true), 2=(2,false)}, 3={3=(3,true)}})"]
    assert bfs_bipartition([3, 1], [3, 2])[0]


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_c_restatement_equals_intended_semantics(seed):
    """oracle/bipartite.c (bench.py's BipartitenessCheck cpu_baseline) = intended_run on random
    bipartite and odd-cycle streams, any partition count."""
    from pyoracle import coracle
    rng = np.random.default_rng(seed)
    n, nv = 3000, 400
    side = rng.integers(0, 2, nv)
    a = rng.integers(0, nv, n)
    b = rng.integers(0, nv, n)
    keep = (side[a] != side[b]) | (a == b)
    s, d = a[keep], b[keep]
    if seed % 2 == 0:                                     # one odd edge somewhere
        i = int(rng.integers(0, s.size))
        same = np.nonzero(side == side[s[i]])[0]
        d[i] = same[same != s[i]][0]
    s = s * 1000003 - 7                                   # Long ids, negatives included
    d = d * 1000003 - 7
    W = 700
    want = intended_run(s.tolist(), d.tolist(), W)[-1]
    for P in (1, 3):
        ok, nvert, ncomp, _ = coracle().bip_run(s, d, W, partitions=P, threads=P)
        assert ok == want[0]
        if ok:
            assert nvert == len(want[1]) and ncomp == len(set(want[1].values()))


def _literal_streams(count: int):
    """Random multi-window, multi-partition streams: bipartite ones (cross edges and self-loops),
    random ones (odd cycles: failures), small id ranges (shared vertices across components)."""
    for seed in range(count):
        rng = np.random.default_rng(seed)
        nv = int(rng.integers(5, 60))
        n = int(rng.integers(1, 200))
        if seed % 3 == 0:
            col = rng.integers(0, 2, nv)
            s, d = [], []
            while len(s) < n:
                a, b = (int(x) for x in rng.integers(0, nv, 2))
                if col[a] != col[b] or a == b:
                    s.append(a)
                    d.append(b)
        else:
            s, d = rng.integers(0, nv, n).tolist(), rng.integers(0, nv, n).tolist()
        yield seed, nv, np.array(s), np.array(d), int(rng.integers(0, 40)), int(rng.integers(1, 4))


def test_literal_engine_on_the_host_equals_literal_oracle(tmp_path):
    """csrc/bip_literal.hpp (the engine libgsgpu.so runs as one HIP workgroup) run serially on the
    host under ASan/UBSan (tests/bipl_host_check.cpp) = oracle/bipartite.py literal_run, every
    window's emission, on 240 random streams: windows of 0-39 edges, 1-3 partitions, failures,
    components sharing vertices and keys signed false among them; on half of them again with the
    Merger's summary snapshotted and restored (load_components) after every window."""
    import shutil
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "bipl_host")
    subprocess.run([gxx, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I", os.path.join(here, "..", "gelly-streaming_amd", "csrc"), os.path.join(here, "bipl_host_check.cpp"),
                    "-o", exe], check=True)
    shared = false_key = failed = 0
    for seed, nv, s, d, W, P in _literal_streams(240):
        want = literal_run(s, d, W, partitions=P)
        inp = "%d %d %d %d\n" % (nv, W, P, len(s)) + "".join("%d %d\n" % (a, b) for a, b in zip(s.tolist(), d.tolist()))
        out = subprocess.run([exe], input=inp, capture_output=True, text=True, timeout=60)
        assert out.returncode == 0, (seed, out.stderr[-2000:])
        assert out.stdout.splitlines() == want, seed
        if seed % 2 == 0:
            # restoreState after every window (gs_bip_restore's engine, load_components): the stream
            # continues from the restored summary with the same emissions
            out = subprocess.run([exe, "restore"], input=inp, capture_output=True, text=True, timeout=60)
            assert out.returncode == 0, (seed, out.stdout[-500:], out.stderr[-2000:])
            assert out.stdout.splitlines() == want, seed
        failed += want[-1] == "(false,{})"
        false_key += any("={%d=(%d,false)" % (k, k) in want[-1] for k in range(nv))
        import re
        ids = re.findall(r"(\d+)=\(\1,", want[-1])
        shared += len(ids) != len(set(ids))
    assert failed > 20 and shared > 10 and false_key > 5, (failed, shared, false_key)
