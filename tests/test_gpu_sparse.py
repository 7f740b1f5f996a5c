"""GPU parity of the sparse-id mode (GS_CC_SPARSE_IDS): DisjointSet<Long> over arbitrary 64-bit
ids — the reference keys its HashMaps by the Long itself (summaries/DisjointSet.java:28-34), so any
long, negative ones included, is a vertex. Bar: bit-exact canonical (min-id) emissions against the
oracle (C restatement, hash-map DisjointSet over int64) and the pure-Python twin."""
import json
import os

import numpy as np
import pytest

from gsgpu import DisjointSet, GsError
from gsgpu import _abi
from pyoracle import EMIT_CHECKSUM, PyDisjointSet

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
SPECIAL = np.array([np.iinfo(np.int64).min, np.iinfo(np.int64).max, -1, 0, 1, -2], dtype=np.int64)


def _sparse_map(nv: int, seed: int) -> np.ndarray:
    """nv distinct int64 ids, spread over the whole long range, with the edge cases in front."""
    rng = np.random.default_rng(seed)
    ids = np.unique(rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, size=2 * nv, dtype=np.int64))
    ids = np.setdiff1d(ids, SPECIAL)
    rng.shuffle(ids)
    return np.concatenate([SPECIAL, ids])[:nv]


def _dense_stream(n: int, nv: int, seed: int):
    rng = np.random.default_rng(seed)
    # power-law-ish endpoints: a few hubs and a long tail, plus self-loops and duplicates
    w = 1.0 / np.arange(1, nv + 1) ** 0.8
    w /= w.sum()
    s = rng.choice(nv, size=n, p=w)
    d = rng.choice(nv, size=n, p=w)
    d[::17] = s[::17]
    return s, d


def test_disjointset_kat_sparse():
    k = json.load(open(os.path.join(GOLD, "reference_kats.json")))["DisjointSetTest"]
    ds = DisjointSet(64, id_bits=64, sparse=True)
    for a, b in k["setup_unions"]:
        ds.union(a, b)
    assert ds.size() == k["expect_matches_size"]
    r0, r1 = ds.find(0), ds.find(1)
    assert (r0, r1) == (0, 1)
    for i in range(10):
        assert ds.find(i) == (r0 if i % 2 == 0 else r1)
    assert ds.find(77) is None
    ds2 = DisjointSet(64, id_bits=64, sparse=True)
    for a, b in k["merge_unions"]:
        ds2.union(a, b)
    ds2.merge(ds)
    assert ds2.size() == k["expect_merged_size"]
    v, l = ds2.pairs()
    assert len(set(l.tolist())) == k["expect_merged_roots"]


@pytest.mark.parametrize("n,nv,W", [(20000, 3000, 2500), (300000, 60000, 50000)])
def test_sparse_windows_vs_oracle(oracle, n, nv, W):
    s, d = _dense_stream(n, nv, seed=n)
    m = _sparse_map(nv, seed=nv)
    hs, hd = m[s], m[d]
    ds = DisjointSet(nv, id_bits=64, sparse=True)
    got = []
    for lo in range(0, n, W):
        ds.fold(hs[lo:lo + W], hd[lo:lo + W])
        ds.close_window()
        got.append(ds.checksum())
    want = oracle.run(hs, hd, W, partitions=3, threads=3, emit=EMIT_CHECKSUM)
    assert [g[0] for g in got] == [int(x) for x in want["checksums"]]
    assert got[-1][1] == want["final_vertices"] and got[-1][2] == want["final_components"]


def test_sparse_pairs_and_find_vs_python_twin():
    s, d = _dense_stream(5000, 900, seed=7)
    m = _sparse_map(900, seed=9)
    hs, hd = m[s], m[d]
    ds = DisjointSet(900, id_bits=64, sparse=True)
    ds.fold(hs, hd)
    py = PyDisjointSet()
    for a, b in zip(hs.tolist(), hd.tolist()):
        py.union(a, b)
    canon = py.canonical()
    v, l = ds.pairs()
    assert v.tolist() == sorted(canon)                      # sorted by (signed) id
    assert l.tolist() == [canon[x] for x in v.tolist()]
    # find: labels for members, None (found=False) for ids never folded, -1 included
    probe = np.concatenate([v[:50], np.setdiff1d(m, v)[:20]])
    lab, found = ds.find_batch_flags(probe)
    for x, y, f in zip(probe.tolist(), lab.tolist(), found.tolist()):
        if x in canon:
            assert f and y == canon[x]
        else:
            assert not f
    assert ds.find(int(np.setdiff1d(m, v)[0])) is None if len(np.setdiff1d(m, v)) else True


def test_sparse_special_ids():
    mn, mx = int(np.iinfo(np.int64).min), int(np.iinfo(np.int64).max)
    ds = DisjointSet(16, id_bits=64, sparse=True)
    ds.fold(np.array([mx, -1, 5, mn]), np.array([-1, 7, 5, 12]))
    assert ds.find(mx) == -1 and ds.find(7) == -1        # component {mx, -1, 7}: min id -1
    assert ds.find(mn) == mn and ds.find(12) == mn       # INT64_MIN lives in the reserved slot
    assert ds.find(5) == 5                               # self-loop singleton
    assert ds.find(6) is None
    assert ds.stats() == (6, 3)
    v, l = ds.pairs()
    assert v.tolist() == [mn, -1, 5, 7, 12, mx]
    assert l.tolist() == [mn, -1, 5, -1, mn, -1]


def test_sparse_merge_and_combine():
    s, d = _dense_stream(8000, 1500, seed=11)
    m = _sparse_map(1500, seed=12)
    hs, hd = m[s], m[d]
    a = DisjointSet(1500, id_bits=64, sparse=True)
    b = DisjointSet(1500, id_bits=64, sparse=True)
    a.fold(hs[:4000], hd[:4000])
    b.fold(hs[4000:], hd[4000:])
    a.merge(b)
    whole = DisjointSet(1500, id_bits=64, sparse=True)
    whole.fold(hs, hd)
    assert a.checksum() == whole.checksum()
    dense = DisjointSet(4096, id_bits=64)
    with pytest.raises(GsError) as e:
        a.merge(dense)
    assert e.value.code == _abi.GS_ERR_UNSUPPORTED


def test_sparse_capacity_and_unsupported_calls():
    ds = DisjointSet(8, id_bits=64, sparse=True)
    with pytest.raises(GsError) as e:
        ds.fold(np.arange(0, 40, dtype=np.int64) * 1000003, np.arange(1, 41, dtype=np.int64) * 999983)
        ds.sync()
    assert e.value.code == _abi.GS_ERR_CAPACITY
    ds2 = DisjointSet(8, id_bits=64, sparse=True)
    ds2.union(3, 4)
    for fn in (lambda: ds2.dense(8), lambda: ds2.labels_device_ptr()):
        with pytest.raises(GsError) as e:
            fn()
        assert e.value.code == _abi.GS_ERR_UNSUPPORTED
    with pytest.raises(GsError):
        DisjointSet(8, id_bits=32, sparse=True)


def test_sparse_device_buffers_and_reset(oracle):
    import torch
    s, d = _dense_stream(100000, 20000, seed=21)
    m = _sparse_map(20000, seed=22)
    hs, hd = m[s], m[d]
    ds = DisjointSet(20000, id_bits=64, sparse=True, stream=torch.cuda.current_stream())
    ds.fold(torch.from_numpy(hs).cuda(), torch.from_numpy(hd).cuda())
    c1 = ds.checksum()
    want = oracle.run(hs, hd, 0, partitions=1, threads=1, emit=EMIT_CHECKSUM)
    assert c1[0] == int(want["checksums"][-1])
    ds.reset()
    assert ds.stats() == (0, 0)
    ds.fold(hs, hd)
    assert ds.checksum() == c1


@pytest.mark.parametrize("mode", ["fused", "reference"])
def test_aggregation_selects_sparse_ids(mode):
    """ConnectedComponents over Long ids outside [0, 2^32): the operator switches to sparse ids
    and every window's emission equals the Python twin's cumulative summary."""
    from gsgpu import ConnectedComponents, SimpleEdgeStream
    s, d = _dense_stream(3000, 500, seed=31)
    m = _sparse_map(500, seed=32)
    hs, hd = m[s], m[d]
    W = 600
    py = PyDisjointSet()
    nwin = 0
    for w, ds in enumerate(SimpleEdgeStream(hs, hd).aggregate(ConnectedComponents(1000, window_edges=W, mode=mode,
                                                                                 parallelism=3))):
        for a, b in zip(hs[w * W:(w + 1) * W].tolist(), hd[w * W:(w + 1) * W].tolist()):
            py.union(a, b)
        assert ds.sparse
        v, l = ds.pairs()
        assert dict(zip(v.tolist(), l.tolist())) == py.canonical()
        nwin += 1
    assert nwin == (len(hs) + W - 1) // W
