"""GPU parity of BipartitenessCheck (gs_bip_*): the reference's known answers
(BipartitenessCheckTest.java:35-90) exactly, and every window's emission of random streams equal
to the oracle's intended semantics (oracle/bipartite.py: union-find with parity, cross-checked
with a BFS 2-colouring). Integer path: bit-exact."""
import json
import os

import numpy as np
import pytest

from gsgpu import BipartitenessCheck, Candidates, GsError, SimpleEdgeStream
from gsgpu import _abi
from bipartite import ParityUnionFind, bfs_bipartition, emission_string, intended_run
from pyoracle import _np_splitmix64

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _kat():
    return json.load(open(os.path.join(GOLD, "reference_kats.json")))["BipartitenessCheckTest"]


@pytest.mark.parametrize("mode", ["fused", "reference"])
@pytest.mark.parametrize("which", ["bipartite", "non_bipartite"])
def test_reference_kats(which, mode):
    k = _kat()
    e = np.array(k[which + "_edges"])
    out = [c.toString() for c in SimpleEdgeStream(e[:, 0], e[:, 1]).aggregate(
        BipartitenessCheck(k["merge_window_ms"], mode=mode, parallelism=1))]
    assert out == k[which + "_expect"]


def _bipartite_stream(nv: int, n: int, seed: int, odd_at: int = -1):
    rng = np.random.default_rng(seed)
    col = rng.integers(0, 2, nv)
    s = rng.integers(0, nv, 4 * n)
    d = rng.integers(0, nv, 4 * n)
    keep = (col[s] != col[d]) | (s == d)                 # cross edges and self-loops
    s, d = s[keep][:n], d[keep][:n]
    if odd_at >= 0:                                     # one same-side edge at position odd_at
        a = int(rng.integers(0, nv))
        b = int(np.nonzero((col == col[a]) & (np.arange(nv) != a))[0][0])
        s[odd_at], d[odd_at] = a, b
    return s.astype(np.int64), d.astype(np.int64)


@pytest.mark.parametrize("mode", ["fused", "reference"])
@pytest.mark.parametrize("nv,n,W,odd_at", [(200, 600, 100, -1), (200, 600, 100, 350), (5000, 20000, 3000, -1),
                                           (5000, 20000, 3000, 17000)])
def test_windows_vs_oracle(mode, nv, n, W, odd_at):
    s, d = _bipartite_stream(nv, n, seed=nv + n + odd_at, odd_at=odd_at)
    want = [emission_string(*x) for x in intended_run(s, d, W)]
    got = [c.toString() for c in SimpleEdgeStream(s, d).aggregate(
        BipartitenessCheck(1000, window_edges=W, mode=mode, parallelism=3))]
    assert got == want
    if odd_at >= 0:
        assert got[-1] == "(false,{})" and got[odd_at // W - 1].startswith("(true,")


def _checksum(key, sign):
    v = np.array(sorted(key), dtype=np.uint64)
    lab = np.array([(key[x] << 1) | (1 if sign[x] else 0) for x in sorted(key)], dtype=np.uint64)
    mix = _np_splitmix64(v ^ _np_splitmix64(lab ^ np.uint64(0xD1B54A32D192ED03)))
    with np.errstate(over="ignore"):
        return int(np.sum(mix, dtype=np.uint64))


@pytest.mark.parametrize("bits", [32, 64])
def test_large_stream_checksum_and_bfs(bits):
    import torch
    nv, n = 1 << 17, 1 << 20
    s, d = _bipartite_stream(nv, n, seed=5)
    uf = ParityUnionFind()
    for a, b in zip(s.tolist(), d.tolist()):
        uf.union(a, b)
    ok, key, sign = uf.emission()
    assert (ok, key, sign) == bfs_bipartition(s, d)
    c = Candidates(nv, id_bits=bits, stream=torch.cuda.current_stream())
    dt = torch.int32 if bits == 32 else torch.int64
    c.fold(torch.from_numpy(s).to(dt).cuda(), torch.from_numpy(d).to(dt).cuda())
    h, good, nverts, ncomp = c.checksum()
    assert good and nverts == len(key) and ncomp == len(set(key.values()))
    assert h == _checksum(key, sign)


def test_merge_of_partials_equals_whole():
    s, d = _bipartite_stream(3000, 12000, seed=9)
    a, b, whole = Candidates(3000), Candidates(3000), Candidates(3000)
    a.fold(s[:6000], d[:6000])
    b.fold(s[6000:], d[6000:])
    whole.fold(s, d)
    assert a.merge(b).toString() == whole.toString()
    bad = Candidates(3000)
    bad.fold(np.array([1, 2, 3]), np.array([2, 3, 1]))
    assert not bad.getSuccess()
    assert a.merge(bad).toString() == "(false,{})"          # a failed input fails the result


def test_self_loops_range_and_reset():
    c = Candidates(16, id_bits=32)
    c.fold(np.array([3, 1, 5]), np.array([3, 2, 5]))
    assert c.toString() == "(true,{1={1=(1,true), 2=(2,false)}, 3={3=(3,true)}, 5={5=(5,true)}})"
    with pytest.raises(GsError) as e:
        c.fold(np.array([1]), np.array([99]))
        c.sync()
    assert e.value.code == _abi.GS_ERR_RANGE
    c.fold(np.array([1, 2]), np.array([4, 4]))              # 1 and 2 on opposite sides: odd cycle
    assert c.toString() == "(false,{})"
    c.reset()
    assert c.toString() == "(true,{})"


@pytest.mark.parametrize("mode", ["fused", "reference"])
@pytest.mark.parametrize("odd_at", [-1, 1500, 4200])
def test_checkpoint_resume(mode, odd_at):
    """snapshotState after k windows, restoreState into a NEW operator, run the rest: every later
    emission equals the uninterrupted run's (the Merger is ListCheckpointed, SummaryAggregation.java:127-135).
    odd_at 1500: the snapshot itself is failed; 4200: the failure comes after the restore."""
    s, d = _bipartite_stream(2000, 6000, seed=21, odd_at=odd_at)
    W, k = 1000, 3
    want = [c.toString() for c in SimpleEdgeStream(s, d).aggregate(
        BipartitenessCheck(1000, window_edges=W, mode=mode, parallelism=3, vertex_capacity=2000))]
    op = BipartitenessCheck(1000, window_edges=W, mode=mode, parallelism=3, vertex_capacity=2000)
    state = None
    for w, c in enumerate(SimpleEdgeStream(s[:k * W], d[:k * W]).aggregate(op)):
        assert c.toString() == want[w]
        if w == k - 1:
            state = op.snapshotState(1, 0)
    assert state is not None and len(state) == 1
    op2 = BipartitenessCheck(1000, window_edges=W, mode=mode, parallelism=3, vertex_capacity=2000)
    op2.restoreState(state)
    got = [c.toString() for c in SimpleEdgeStream(s[k * W:], d[k * W:]).aggregate(op2)]
    assert got == want[k:]


def test_restore_with_key_signed_false():
    """A snapshot whose component key is signed false (reversed Candidates.merge can leave it so,
    Candidates.java:155-182): the restore reads each vertex's side relative to the key's own sign
    (ADVICE r02). 1 and 3 share a side, 2 is on the other."""
    c = Candidates(16, id_bits=32)
    c.restore(True, np.array([1, 2, 3]), np.array([1, 1, 1]), np.array([False, True, False]))
    assert c.toString() == "(true,{1={1=(1,true), 2=(2,false), 3=(3,true)}})"
    c.fold(np.array([2]), np.array([5]))                     # 5 joins on 1's side: still bipartite
    assert c.toString() == "(true,{1={1=(1,true), 2=(2,false), 3=(3,true), 5=(5,true)}})"
    c.fold(np.array([1]), np.array([3]))                     # same side: an odd cycle
    assert c.toString() == "(false,{})"


# ---- GS_BIP_REFERENCE_LITERAL: the reference's Candidates rule as written (csrc/bip_literal.hpp) ----
from bipartite import literal_run  # noqa: E402


def _literal_emissions(s, d, W, P, id_bits=64, entry_capacity=0):
    return [c.toString() for c in SimpleEdgeStream(np.asarray(s), np.asarray(d)).aggregate(
        BipartitenessCheck(1000, window_edges=W, mode="literal", parallelism=P, id_bits=id_bits,
                           entry_capacity=entry_capacity))]


@pytest.mark.parametrize("which", ["bipartite", "non_bipartite"])
def test_literal_reference_kats(which):
    k = _kat()
    e = np.array(k[which + "_edges"])
    out = [c.toString() for c in SimpleEdgeStream(e[:, 0], e[:, 1]).aggregate(
        BipartitenessCheck(k["merge_window_ms"], mode="literal", parallelism=1))]
    assert out == k[which + "_expect"]


def test_literal_split_branch_and_self_loops():
    """The triangle the literal rule loses (Candidates.java:117-134) and self-loops (edgeToCandidate)."""
    assert _literal_emissions([5, 3, 3], [7, 7, 5], 0, 1) == ["(true,{3={3=(3,true), 5=(5,false), 7=(7,false)}})"]
    assert _literal_emissions([3, 1], [3, 2], 0, 1) == ["(true,{1={1=(1,true), 2=(2,false)}, 3={3=(3,true)}})"]


def _random_literal_cases(count: int, base: int):
    for seed in range(base, base + count):
        rng = np.random.default_rng(seed)
        nv = int(rng.integers(5, 80))
        n = int(rng.integers(1, 260))
        if seed % 3 == 0:                                       # bipartite: cross edges and self-loops
            col = rng.integers(0, 2, nv)
            s, d = [], []
            while len(s) < n:
                a, b = (int(x) for x in rng.integers(0, nv, 2))
                if col[a] != col[b] or a == b:
                    s.append(a)
                    d.append(b)
        else:                                                   # random: odd cycles
            s, d = rng.integers(0, nv, n).tolist(), rng.integers(0, nv, n).tolist()
        yield seed, np.array(s), np.array(d), int(rng.integers(0, 50)), int(rng.integers(1, 4))


@pytest.mark.parametrize("id_bits", [32, 64])
def test_literal_every_window_vs_literal_oracle(id_bits):
    """Every window's emission on 40 random multi-window streams (windows of 0-49 edges, 1-3
    partitions: fresh partials combined in partition order, the Merger's windowResult.merge(summary))
    equals oracle/bipartite.py's literal_run — including components that share vertices, keys
    signed false and the sticky failure."""
    seen_shared = seen_false = 0
    for seed, s, d, W, P in _random_literal_cases(40, 1000 + id_bits):
        want = literal_run(s, d, W, partitions=P)
        got = _literal_emissions(s, d, W, P, id_bits=id_bits)
        assert got == want, (seed, W, P)
        seen_false += want[-1] == "(false,{})"
        seen_shared += any(w.count("=(%d," % v) > 1 for w in want for v in range(80))
    assert seen_false > 5 and seen_shared > 3, (seen_false, seen_shared)


@pytest.mark.parametrize("odd_at", [-1, 2100])
def test_literal_larger_stream(odd_at):
    """A 3000-edge bipartite stream (and one with an odd edge late) over 8 windows and 3 partitions."""
    s, d = _bipartite_stream(400, 3000, seed=7 + odd_at, odd_at=odd_at)
    want = literal_run(s, d, 375, partitions=3)
    assert _literal_emissions(s, d, 375, 3) == want


def test_literal_errors():
    # entry capacity: 2 edges need 4 memberships; 3 fit no window
    with pytest.raises(GsError) as ei:
        _literal_emissions([1, 3], [2, 4], 0, 1, entry_capacity=3)
    assert ei.value.code == _abi.GS_ERR_CAPACITY
    # literal and intended summaries do not merge
    a = Candidates(16, literal=True)
    b = Candidates(16)
    with pytest.raises(GsError) as ei:
        a.merge(b)
    assert ei.value.code == _abi.GS_ERR_UNSUPPORTED
    # an id past the capacity: that edge is skipped and reported, the rest folded
    a.fold(np.array([1, 40, 2]), np.array([2, 3, 5]))
    with pytest.raises(GsError) as ei:
        a.sync()
    assert ei.value.code == _abi.GS_ERR_RANGE
    assert a.toString() == "(true,{1={1=(1,true), 2=(2,false), 5=(5,true)}})"
    a.restore(*a.snapshot())                           # loaded as it is (gs_bip_restore)
    assert a.toString() == "(true,{1={1=(1,true), 2=(2,false), 5=(5,true)}})"
    # a snapshot larger than the entry capacity
    c = Candidates(16, literal=True, entry_capacity=3)
    with pytest.raises(GsError) as ei:
        c.restore(True, np.array([1, 2, 3, 4]), np.array([1, 1, 3, 3]), np.array([True, False, True, False]))
    assert ei.value.code == _abi.GS_ERR_CAPACITY
    # an entry twice in one component
    with pytest.raises(GsError) as ei:
        a.restore(True, np.array([1, 1]), np.array([1, 1]), np.array([True, True]))
    assert ei.value.code == _abi.GS_ERR_INVALID
    a.close()
    b.close()
    c.close()


def test_literal_restore_overlapping_components_then_fold():
    """gs_bip_restore of a literal snapshot whose components share a vertex (key 1 = {1, 2}, key 2 =
    {2, 3}, 2 signed false in one and true in the other) and a key signed false, then more edges:
    every emission equals the literal oracle started from the same map (Candidates.add, :55-67)."""
    from bipartite import LiteralCandidates, edge_to_candidate
    comps = {1: {1: True, 2: False}, 2: {2: True, 3: False}, 5: {5: False, 6: True}}
    v, k, sg = [], [], []
    for key, m in comps.items():
        for vert, sign in m.items():
            v.append(vert); k.append(key); sg.append(sign)
    for id_bits in (32, 64):
        c = Candidates(32, id_bits=id_bits, literal=True)
        c.restore(True, np.array(v), np.array(k), np.array(sg))
        o = LiteralCandidates(True)
        for key in sorted(comps):
            o.add_component(key, dict(comps[key]))
        assert c.toString() == o.to_string()
        for a_, b_ in [(3, 7), (6, 8), (2, 9), (1, 3), (7, 5), (4, 4)]:
            c.fold(np.array([a_]), np.array([b_]))
            o = o.merge(edge_to_candidate(a_, b_))
            assert c.toString() == o.to_string(), (id_bits, a_, b_)
        c.restore(False, np.array([], dtype=np.int64), np.array([], dtype=np.int64), np.array([], dtype=bool))
        assert c.toString() == "(false,{})"
        c.fold(np.array([1]), np.array([2]))
        assert c.toString() == "(false,{})"               # Candidates.fail() is sticky
        c.close()


def test_literal_checkpoint_resume():
    """snapshotState after k windows, restoreState into a NEW literal operator, run the rest: every
    later emission equals the literal oracle's uninterrupted run (ListCheckpointed Merger,
    SummaryAggregation.java:121-135), on random multi-window streams with components that share
    vertices, keys signed false and failures."""
    tried = shared = 0
    for seed, s, d, W, P in _random_literal_cases(40, 3000):
        if W == 0 or len(s) < 3 * W:
            continue
        want = literal_run(s, d, W, partitions=P)
        k = len(want) // 2
        op = BipartitenessCheck(1000, window_edges=W, mode="literal", parallelism=P, vertex_capacity=128)
        state = None
        for w, c in enumerate(SimpleEdgeStream(s[:k * W], d[:k * W]).aggregate(op)):
            assert c.toString() == want[w], (seed, w)
            if w == k - 1:
                state = op.snapshotState(1, 0)
        op2 = BipartitenessCheck(1000, window_edges=W, mode="literal", parallelism=P, vertex_capacity=128)
        op2.restoreState(state)
        got = [c.toString() for c in SimpleEdgeStream(s[k * W:], d[k * W:]).aggregate(op2)]
        assert got == want[k:], seed
        tried += 1
        shared += any(want[k - 1].count("=(%d," % v) > 1 for v in range(128))
    assert tried >= 10 and shared >= 2, (tried, shared)
