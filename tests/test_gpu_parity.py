"""GPU parity: the HIP path (libgsgpu.so via its C ABI) against the oracle and golden fixtures.

Bar: bit-exact canonical (min-id) labels for every window emission (integer path, no tolerance).
"""
import json
import os

import numpy as np
import pytest

import gsgpu
from gsgpu import DisjointSet, SimpleEdgeStream, ConnectedComponents, GsError, combine_cc
from gsgpu import _abi
from pyoracle import EMIT_CHECKSUM, EMIT_DENSE, dense_checksum

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _kats():
    with open(os.path.join(GOLD, "reference_kats.json")) as f:
        return json.load(f)


def _streams():
    with open(os.path.join(GOLD, "streams_index.json")) as f:
        idx = json.load(f)
    z = np.load(os.path.join(GOLD, "streams.npz"))
    return [dict(c, **{k: z["%s__%s" % (c["name"], k)] for k in ("src", "dst", "labels", "checksums")})
            for c in idx]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def _parse(ds: DisjointSet):
    """ConnectedComponentsTest.parser (example/test/ConnectedComponentsTest.java:65-81)."""
    r = ds.toString()
    out = []
    for g in r.split("="):
        if "[" in g:
            out.append(g.split("]")[0][1:])
    return sorted(out)


# ---------------- reference known-answer tests ----------------
@pytest.mark.parametrize("bits", [32, 64])
def test_disjointset_kat(bits):
    k = _kats()["DisjointSetTest"]
    ds = DisjointSet(256, id_bits=bits)
    for a, b in k["setup_unions"]:
        ds.union(a, b)
    assert ds.size() == k["expect_matches_size"]
    r0, r1 = ds.find(0), ds.find(1)
    assert r0 != r1
    for i in range(10):
        assert ds.find(i) == (r0 if i % 2 == 0 else r1)
    assert ds.find(77) is None
    ds2 = DisjointSet(256, id_bits=bits)
    for a, b in k["merge_unions"]:
        ds2.union(a, b)
    ds2.merge(ds)
    assert ds2.size() == k["expect_merged_size"]
    v, l = ds2.pairs()
    assert len(set(l.tolist())) == k["expect_merged_roots"]


@pytest.mark.parametrize("mode", ["fused", "reference"])
def test_connected_components_kat(mode):
    k = _kats()["ConnectedComponentsTest"]
    e = np.array(k["edges"])
    stream = SimpleEdgeStream(e[:, 0], e[:, 1])
    last = None
    for ds in stream.aggregate(ConnectedComponents(5, window_edges=2, mode=mode, parallelism=2)):
        last = _parse(ds)
    assert last == k["expect_final_components"]


def test_example_sample_stream_event_time():
    k = _kats()["ConnectedComponentsExample"]
    stream = SimpleEdgeStream(k["src"], k["dst"], k["timestamps"])
    emissions = []
    for ds in stream.aggregate(ConnectedComponents(k["merge_window_ms"])):
        emissions.append(ds.getMatches())
    assert len(emissions) == len(k["event_time_windows"])
    for em, w in zip(emissions, k["event_time_windows"]):
        assert len(em) == w["n_vertices"]
        assert all(lab == (1 if v % 2 else 2) for v, lab in em.items())
    assert len(emissions[-1]) == k["expect_final_vertices"]


# ---------------- golden seeded streams, per-window emissions ----------------
@pytest.mark.parametrize("bits", [32, 64])
@pytest.mark.parametrize("mode", ["fused", "reference"])
@pytest.mark.parametrize("case", _streams(), ids=lambda c: c["name"])
def test_streams_golden(case, mode, bits):
    stream = SimpleEdgeStream(case["src"], case["dst"])
    cc = ConnectedComponents(1000, window_edges=case["window_edges"], parallelism=case["partitions"],
                             mode=mode, id_bits=bits, vertex_capacity=case["cap"])
    w = 0
    for ds in stream.aggregate(cc):
        lab = ds.dense().astype(np.int64)
        np.testing.assert_array_equal(lab, case["labels"][w], err_msg="window %d" % w)
        assert ds.checksum()[0] == int(case["checksums"][w])
        w += 1
    assert w == case["labels"].shape[0]


# ---------------- Merger checkpoint / resume (ListCheckpointed, SummaryAggregation.java:127-135) ----------------
@pytest.mark.parametrize("bits", [32, 64])
@pytest.mark.parametrize("mode", ["fused", "reference", "tree"])
@pytest.mark.parametrize("case", _streams()[:3], ids=lambda c: c["name"])
def test_merger_checkpoint_resume(case, mode, bits):
    """Run k windows, snapshotState, restore into a NEW operator and run the rest of the stream:
    every later emission equals the uninterrupted pipeline's (the golden labels). mode "tree":
    ConnectedComponentsTree, whose output also goes through the ListCheckpointed Merger
    (SummaryTreeReduce.java:87-90 -> SummaryAggregation.java:127-135)."""
    from gsgpu import ConnectedComponentsTree
    W = case["window_edges"]
    nwin = case["labels"].shape[0]
    k = max(1, nwin // 2)
    kw = dict(window_edges=W, id_bits=bits, vertex_capacity=case["cap"])
    if mode == "tree":
        make = lambda: ConnectedComponentsTree(1000, max(case["partitions"], 3), **kw)
    else:
        make = lambda: ConnectedComponents(1000, parallelism=case["partitions"], mode=mode, **kw)
    cc = make()
    state = None
    for w, ds in enumerate(SimpleEdgeStream(case["src"][:k * W], case["dst"][:k * W]).aggregate(cc)):
        if w == k - 1:
            state = cc.snapshotState(1, 0)
    assert state is not None and len(state) == 1
    cc2 = make()
    cc2.restoreState(state)
    w = k
    for ds in SimpleEdgeStream(case["src"][k * W:], case["dst"][k * W:]).aggregate(cc2):
        np.testing.assert_array_equal(ds.dense().astype(np.int64), case["labels"][w], err_msg="window %d" % w)
        w += 1
    assert w == nwin


def test_snapshot_restore_sparse_ids(oracle):
    """DisjointSet.snapshot / restore with ids across the whole long range (GS_CC_SPARSE_IDS)."""
    rng = np.random.default_rng(7)
    ids = rng.integers(-(1 << 62), 1 << 62, size=3000, dtype=np.int64)
    ids[:3] = [-1, np.iinfo(np.int64).min, np.iinfo(np.int64).max]
    src = ids[rng.integers(0, ids.size, 8000)]
    dst = ids[rng.integers(0, ids.size, 8000)]
    a = DisjointSet(ids.size, id_bits=64, sparse=True)
    a.fold(src[:5000], dst[:5000])
    a.close_window()
    snap = a.snapshot()
    b = DisjointSet(ids.size, id_bits=64, sparse=True)
    b.restore(*snap)
    assert b.toString() == a.toString()
    a.fold(src[5000:], dst[5000:]); b.fold(src[5000:], dst[5000:])
    va, la = a.pairs(); vb, lb = b.pairs()
    np.testing.assert_array_equal(va, vb)
    np.testing.assert_array_equal(la, lb)
    a.close(); b.close()


# ---------------- larger random streams vs the C oracle ----------------
@pytest.mark.parametrize("gen,scale,n,W", [("rmat", 16, 1 << 20, 1 << 16), ("er", 17, 1 << 19, 100003),
                                           ("rmat", 12, 300000, 4096)])
def test_random_streams_vs_oracle(oracle, torch_cuda, gen, scale, n, W):
    torch = torch_cuda
    cap = 1 << scale
    if gen == "rmat":
        s, d = oracle.gen_rmat(0, n, scale, 17)
    else:
        s, d = oracle.gen_er(0, n, cap, 5)
    want = oracle.run(s, d, W, partitions=4, threads=4, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    ds = DisjointSet(cap, id_bits=32)
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    for w, lo in enumerate(range(0, n, W)):
        ds.fold(ts[lo:lo + W], td[lo:lo + W])
        ds.close_window()
        h, nv, nc = ds.checksum()
        assert h == int(want["checksums"][w]), "window %d" % w
    np.testing.assert_array_equal(ds.dense().astype(np.int64), want["final"])
    assert ds.stats() == (want["final_vertices"], want["final_components"])


def test_host_and_device_buffers_agree(oracle, torch_cuda):
    torch = torch_cuda
    s, d = oracle.gen_rmat(0, 200000, 14, 4)
    a = DisjointSet(1 << 14, id_bits=64, staging_edges=4096)   # host int64, staged in chunks
    a.fold(s, d)
    b = DisjointSet(1 << 14, id_bits=64)
    b.fold(torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda())
    np.testing.assert_array_equal(a.dense(), b.dense())
    out = torch.empty(1 << 14, dtype=torch.int64, device="cuda")
    b.dense(out=out)
    np.testing.assert_array_equal(out.cpu().numpy(), a.dense())


def test_combine_cc_semantics():
    a = DisjointSet(64, id_bits=32)
    b = DisjointSet(64, id_bits=32)
    a.union(1, 2)
    for i in range(5):
        b.union(10 + i, 11 + i)
    r = combine_cc(a, b)
    assert r is b and b.size() == 8
    c = DisjointSet(64, id_bits=32)
    c.union(2, 10)
    r = combine_cc(b, c)
    assert r is b
    assert b.find(15) == 1 and b.find(11) == 1 and b.find(2) == 1


# ---------------- edge cases ----------------
def test_empty_and_noop_calls():
    ds = DisjointSet(16, id_bits=32)
    ds.fold(np.array([], dtype=np.int32), np.array([], dtype=np.int32))
    ds.close_window()
    assert ds.stats() == (0, 0)
    assert ds.pairs()[0].size == 0
    assert (ds.dense() == -1).all()
    assert ds.checksum() == (0, 0, 0)


def test_out_of_range_ids_raise_and_are_skipped():
    ds = DisjointSet(100, id_bits=64)
    ds.fold(np.array([1, 5, -3]), np.array([2, 100, 4]))
    with pytest.raises(GsError) as ei:
        ds.sync()
    assert ei.value.code == _abi.GS_ERR_RANGE
    assert ds.getMatches() == {1: 1, 2: 1}
    ds32 = DisjointSet(100, id_bits=32)
    with pytest.raises(GsError):
        ds32.fold(np.array([0xFFFFFFFF], dtype=np.uint32), np.array([1], dtype=np.uint32))
        ds32.sync()


def test_self_loops_and_duplicates():
    ds = DisjointSet(32, id_bits=32)
    ds.fold(np.array([3, 3, 4, 4, 9]), np.array([3, 3, 9, 9, 4]))
    assert ds.getMatches() == {3: 3, 4: 4, 9: 4}
    assert ds.stats() == (3, 2)


def test_max_capacity_id_and_find_batch():
    cap = (1 << 20) + 3
    ds = DisjointSet(cap, id_bits=64)
    ds.fold(np.array([cap - 1, 7]), np.array([0, cap - 2]))
    r = ds.find_batch(np.array([cap - 1, cap - 2, 0, 7, 5, cap, -1]))
    assert r.tolist() == [0, 7, 0, 7, -1, -1, -1]


def test_emit_pairs_sorted_and_capacity_error(torch_cuda):
    ds = DisjointSet(5000, id_bits=32)
    rng = np.random.default_rng(1)
    s, d = rng.integers(0, 5000, 3000), rng.integers(0, 5000, 3000)
    ds.fold(s, d)
    v, l = ds.pairs()
    assert (np.diff(v) > 0).all()
    dense = ds.dense()
    np.testing.assert_array_equal(dense[v], l)
    assert (dense >= 0).sum() == v.size
    import ctypes
    n = ctypes.c_uint64()
    small = np.empty(4, dtype=np.int32)
    rc = _abi.lib().gs_cc_emit_pairs(ds.handle, small.ctypes.data_as(ctypes.c_void_p),
                                     small.ctypes.data_as(ctypes.c_void_p), 2, ctypes.byref(n))
    assert rc == _abi.GS_ERR_CAPACITY and n.value == v.size


@pytest.mark.parametrize("bits", [32, 64])
def test_emit_delta_rebuilds_every_emission(oracle, torch_cuda, bits):
    """gs_cc_emit_delta: applying each window's delta to a host map reproduces that window's whole
    emission (gs_cc_emit_pairs, and the oracle's checksum), a too-small buffer consumes nothing,
    and after reset the first delta is the whole emission again (SummaryAggregation.java:110-111)."""
    from pyoracle import dense_checksum
    s, d = oracle.gen_rmat(0, 1 << 18, 15, 4)
    cap, W = 1 << 15, 1 << 15
    want = oracle.run(s, d, W, partitions=2, emit=EMIT_CHECKSUM, label_cap=cap)
    ds = DisjointSet(cap, id_bits=bits)
    for step in range(2):
        ds.reset()
        mirror = np.full(cap, -1, dtype=np.int64)
        sizes = []
        for w, lo in enumerate(range(0, s.size, W)):
            ds.fold(s[lo:lo + W], d[lo:lo + W])
            if w == 2:                                   # too small: error, nothing consumed
                small = np.empty(1, dtype=np.int32 if bits == 32 else np.int64)
                with pytest.raises(GsError) as e:
                    ds.delta(small, small.copy())
                assert e.value.code == _abi.GS_ERR_CAPACITY
            v, l = ds.delta()
            assert (np.diff(v) > 0).all()
            sizes.append(v.size)
            mirror[v.astype(np.int64)] = l
            pv, pl = ds.pairs()
            np.testing.assert_array_equal(np.nonzero(mirror >= 0)[0], pv)
            np.testing.assert_array_equal(mirror[pv], pl)
            assert dense_checksum(mirror)[0] == int(want["checksums"][w])
        assert sizes[0] == ds.stats()[0] or len(sizes) > 1
        assert sum(sizes[1:]) < 2 * ds.stats()[0]        # deltas, not whole emissions
        v, l = ds.delta()                                # nothing changed since
        assert v.size == 0


@pytest.mark.parametrize("where", ["pinned", "device"])
@pytest.mark.parametrize("bits", [32, 64])
def test_emit_delta_async_rebuilds_every_emission(oracle, torch_cuda, bits, where):
    """gs_cc_emit_delta_async + gs_cc_emit_wait (the per-window emission without a host wait, two
    slots in flight): the deltas, applied in order, reproduce every window's emission (oracle
    checksums); an emission that does not fit fails at the wait and consumes nothing; pageable host
    buffers are refused (SummaryAggregation.java:110-111)."""
    torch = torch_cuda
    from pyoracle import dense_checksum
    s, d = oracle.gen_rmat(0, 1 << 18, 15, 4)
    cap, W = 1 << 15, 1 << 15
    want = oracle.run(s, d, W, partitions=2, emit=EMIT_CHECKSUM, label_cap=cap)
    ds = DisjointSet(cap, id_bits=bits)
    dt = torch.int32 if bits == 32 else torch.int64

    def mk(n):
        return torch.empty(n, dtype=dt).pin_memory() if where == "pinned" else torch.empty(n, dtype=dt, device="cuda")

    bufs = [(mk(cap), mk(cap)) for _ in range(2)]
    mirror = np.full(cap, -1, dtype=np.int64)
    sums = []

    def apply(done):
        for v, l in done:
            v = v.cpu().numpy().astype(np.int64)
            l = l.cpu().numpy().astype(np.int64)
            assert (np.diff(v) > 0).all()
            mirror[v] = l
            sums.append(dense_checksum(mirror)[0])

    for w, lo in enumerate(range(0, s.size, W)):
        ds.fold(s[lo:lo + W], d[lo:lo + W])
        ds.delta_async(*bufs[w & 1])
        apply(ds.emit_wait(1))
    apply(ds.emit_wait(0))
    assert sums == [int(x) for x in want["checksums"]]
    pv, pl = ds.pairs()
    np.testing.assert_array_equal(np.nonzero(mirror >= 0)[0], pv)
    np.testing.assert_array_equal(mirror[pv], pl)
    # too small: GS_ERR_CAPACITY at the wait, nothing consumed (the next delta is the whole emission)
    ds.reset()
    ds.fold(s[:W], d[:W])
    ds.delta_async(mk(1), mk(1))
    with pytest.raises(GsError) as e:
        ds.emit_wait(0)
    assert e.value.code == _abi.GS_ERR_CAPACITY
    v, l = ds.delta()
    assert v.size == ds.stats()[0]
    ds.delta_async(*bufs[0])                         # nothing changed since
    ((v, l),) = ds.emit_wait(0)
    assert v.numel() == 0
    npdt = np.int32 if bits == 32 else np.int64       # pageable host memory: copied at the wait
    ds.fold(s[W:2 * W], d[W:2 * W])
    ds.delta_async(np.empty(cap, dtype=npdt), np.empty(cap, dtype=npdt))
    ((v, l),) = ds.emit_wait(0)
    mirror = np.full(cap, -1, dtype=np.int64)
    mirror[v.astype(np.int64)] = l                    # (the first delta after reset was the sync one)
    pv, pl = ds.pairs()
    changed = np.isin(pv, v.astype(np.int64))
    np.testing.assert_array_equal(mirror[pv[changed]], pl[changed])
    assert v.size and (np.diff(v.astype(np.int64)) > 0).all()


def test_reset_and_transient_state():
    ds = DisjointSet(64, id_bits=32)
    ds.union(1, 2)
    ds.reset()
    assert ds.stats() == (0, 0)
    ds.union(3, 4)
    assert ds.getMatches() == {3: 3, 4: 3}


# ---------------- device generators vs the host definition ----------------
@pytest.mark.parametrize("bits", [32, 64])
def test_device_generators_match_oracle(oracle, torch_cuda, bits):
    torch = torch_cuda
    from gsgpu import gen
    dt = torch.int32 if bits == 32 else torch.int64
    for first, n, scale, seed, scr in [(0, 100000, 20, 1, True), (1 << 30, 4096, 26, 1, True),
                                       (77, 5000, 12, 9, False)]:
        s = torch.empty(n, dtype=dt, device="cuda")
        d = torch.empty(n, dtype=dt, device="cuda")
        gen.rmat(s, d, first, scale, seed, scramble=scr)
        torch.cuda.synchronize()
        ws, wd = oracle.gen_rmat(first, n, scale, seed, scramble=scr)
        np.testing.assert_array_equal(s.cpu().numpy().astype(np.int64), ws)
        np.testing.assert_array_equal(d.cpu().numpy().astype(np.int64), wd)
    s = torch.empty(50000, dtype=dt, device="cuda")
    d = torch.empty(50000, dtype=dt, device="cuda")
    gen.erdos_renyi(s, d, 123, 1 << 24, 2)
    torch.cuda.synchronize()
    ws, wd = oracle.gen_er(123, 50000, 1 << 24, 2)
    np.testing.assert_array_equal(s.cpu().numpy().astype(np.int64), ws)
    np.testing.assert_array_equal(d.cpu().numpy().astype(np.int64), wd)


# ---------------- partial-summary exchange (multi-GPU tree protocol, one process) ----------------
@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_tree_exchange_single_process(oracle, torch_cuda, world):
    """Every 'rank' is a handle on this GPU; the tree rounds of tests/gloo_tree.py are replayed with
    device buffers handed across directly (what RCCL send/recv does between GPUs)."""
    torch = torch_cuda
    from gloo_tree import tree_schedule
    scale, n, W = 13, 200000, 20000
    cap = 1 << scale
    s, d = oracle.gen_rmat(0, n, scale, 8)
    s = np.concatenate([s, [cap - 1, cap - 2]]); d = np.concatenate([d, [cap - 1, cap - 2]])
    n = s.size
    want = oracle.run(s, d, W, partitions=world, emit=EMIT_DENSE, label_cap=cap)["labels"]
    ranks = [DisjointSet(cap, id_bits=32, track_marks=(r != 0)) for r in range(world)]
    buf = torch.empty(2 * cap, dtype=torch.int32, device="cuda")
    scheds = [tree_schedule(r, world) for r in range(world)]
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    for w, lo in enumerate(range(0, n, W)):
        ln = min(W, n - lo)
        for r in range(world):
            a, b = lo + (ln * r) // world, lo + (ln * (r + 1)) // world
            ranks[r].fold(ts[a:b], td[a:b])
        done = set()
        for i in range(len(scheds[0])):
            for r in range(world):
                if r in done:
                    continue
                role, peer = scheds[r][i]
                if role == "send":
                    m = ranks[r].export_marks(buf)
                    ranks[peer].fold_pairs(buf, m, id_bits=32)
                    ranks[peer].sync()          # buf is reused by the next export (other stream)
                    done.add(r)
        ranks[0].close_window()
        np.testing.assert_array_equal(ranks[0].dense().astype(np.int64), want[w], err_msg="window %d" % w)


@pytest.mark.parametrize("slots", [False, True], ids=["deltas", "padded_slots"])
@pytest.mark.parametrize("world", [2, 3, 4])
def test_replicated_exchange_single_process(oracle, torch_cuda, world, slots):
    """AllgatherMerge's protocol replayed with device handles on this GPU: every rank folds its
    slice, exports its delta asynchronously (count in device memory), folds every other rank's
    delta with marking paused, closes; EVERY replica's emission must equal the oracle's."""
    torch = torch_cuda
    from gloo_tree import fold_deltas, fold_slots
    scale, n, W = 13, 200000, 20000
    cap = 1 << scale
    s, d = oracle.gen_rmat(0, n, scale, 9)
    s = np.concatenate([s, [cap - 1, cap - 2]]); d = np.concatenate([d, [cap - 1, cap - 2]])
    n = s.size
    want = oracle.run(s, d, W, partitions=world, emit=EMIT_DENSE, label_cap=cap)["labels"]
    cur = torch.cuda.current_stream()
    ranks = [DisjointSet(cap, id_bits=32, track_marks=True, stream=cur) for _ in range(world)]
    bufs = [torch.empty(4 * cap, dtype=torch.int32, device="cuda") for _ in range(world)]   # 2 x cap pairs
    cnt = torch.zeros(world, dtype=torch.int64, device="cuda")
    recv = torch.empty(2 * cap * world, dtype=torch.int32, device="cuda")
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    for w, lo in enumerate(range(0, n, W)):
        ln = min(W, n - lo)
        for r in range(world):
            a, b = lo + (ln * r) // world, lo + (ln * (r + 1)) // world
            ranks[r].fold(ts[a:b], td[a:b])
            ranks[r].export_marks_async(bufs[r], cnt[r:r + 1])
        ns = [int(x) for x in cnt.tolist()]
        m = max(ns)
        if slots and m:                 # AllgatherMerge's layout: slots of m pairs, padded
            for q in range(world):
                if 0 < ns[q] < m:
                    bufs[q][2 * ns[q]: 2 * m].view(-1, 2).copy_(bufs[q][0:2].view(1, 2).expand(m - ns[q], 2))
            torch.cat([bufs[q][:2 * m] for q in range(world)], out=recv[:2 * m * world])
        for r in range(world):
            others = [q for q in range(world) if q != r]
            tot = sum(ns[q] for q in others)
            if tot and not slots:
                torch.cat([bufs[q][:2 * ns[q]] for q in others], out=recv[:2 * tot])
            ranks[r].set_marking(False)
            if slots:
                if m:
                    fold_slots(ranks[r], recv, m, [0 if q == r else ns[q] for q in range(world)])
            else:
                fold_deltas(ranks[r], recv, [ns[q] for q in others])
            ranks[r].set_marking(True)
            ranks[r].close_window()
        for r in range(world):
            np.testing.assert_array_equal(ranks[r].dense().astype(np.int64), want[w], err_msg="window %d rank %d" % (w, r))
    # folds while marking is paused leave nothing to export
    ranks[0].reset()
    e = lambda *x: torch.tensor(x, dtype=torch.int32, device="cuda")
    ranks[0].set_marking(False)
    ranks[0].fold(e(1, 7), e(2, 7))              # a join and a self-loop, unmarked
    ranks[0].set_marking(True)
    assert ranks[0].export_marks(bufs[0]) == 0
    ranks[0].fold(e(3, 2), e(4, 9))              # 4 hooked under 3; 9 joins 1's component
    m = ranks[0].export_marks(bufs[0])
    got = sorted(map(tuple, bufs[0][:2 * m].view(-1, 2).cpu().numpy().tolist()))
    assert got == [(4, 3), (9, 1)]
    with pytest.raises(GsError):
        DisjointSet(cap, id_bits=32).set_marking(True)       # no marks tracked


# ---------------- full-size properties (independent torch checker) ----------------
def _torch_min_labels(torch, src, dst, V):
    """Independent min-label CC on the GPU with torch ops (hook-to-min + pointer jumping)."""
    lab = torch.arange(V, dtype=torch.int64, device="cuda")
    s = src.long(); d = dst.long()
    while True:
        ls, ld = lab[s], lab[d]
        m = torch.minimum(ls, ld)
        new = lab.clone()
        new.scatter_reduce_(0, ls, m, reduce="amin")
        new.scatter_reduce_(0, ld, m, reduce="amin")
        while True:                                   # pointer jumping to the fixpoint
            j = new[new]
            if torch.equal(j, new):
                break
            new = j
        if torch.equal(new, lab):
            break
        lab = new
    seen = torch.zeros(V, dtype=torch.bool, device="cuda")
    seen[s] = True
    seen[d] = True
    return torch.where(seen, lab, torch.full_like(lab, -1))


@pytest.mark.parametrize("scale,ef,W", [(22, 16, 1 << 22), (24, 16, 1 << 24)])
def test_full_size_rmat_properties(torch_cuda, scale, ef, W):
    torch = torch_cuda
    from gsgpu import gen
    V, E = 1 << scale, ef << scale
    s = torch.empty(E, dtype=torch.int32, device="cuda")
    d = torch.empty(E, dtype=torch.int32, device="cuda")
    gen.rmat(s, d, 0, scale, 1)
    ds = DisjointSet(V, id_bits=32)
    ds.set_stream(torch.cuda.current_stream())
    sums = []
    for lo in range(0, E, W):
        ds.fold(s[lo:lo + W], d[lo:lo + W])
        ds.close_window()
        sums.append(ds.checksum())
    lab = torch.empty(V, dtype=torch.int32, device="cuda")
    ds.dense(out=lab)
    lab = lab.long()
    seenmask = lab >= 0
    v = torch.arange(V, device="cuda")
    # min-id labels: label <= vertex, label is its own label (idempotent), edges agree
    assert bool((lab[seenmask] <= v[seenmask]).all())
    assert bool((lab[lab[seenmask]] == lab[seenmask]).all())
    assert bool((lab[s.long()] == lab[d.long()]).all())
    want = _torch_min_labels(torch, s, d, V)
    assert torch.equal(lab, want)
    # checksum of the final emission recomputed from the dense labels
    assert sums[-1][0] == dense_checksum(lab.cpu().numpy())[0]
    # number of vertices is monotone over the windows (cumulative summary)
    assert all(a[1] <= b[1] for a, b in zip(sums, sums[1:]))


# ---------------- C++ host mirror: ConnectedComponentsExample port ----------------
def _example_bin():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return os.path.join(root, "gelly-streaming_amd", "gsgpu", "lib", "cc_example")


def _parse_pairs(out: str):
    import re
    return [(int(a), int(b)) for a, b in re.findall(r"^\((-?\d+),(-?\d+)\)$", out, re.M)]


def test_cc_example_builtin_stream():
    import subprocess
    out = subprocess.check_output([_example_bin()], timeout=120).decode()
    pairs = _parse_pairs(out)
    assert pairs, out
    assert all(r == (1 if v % 2 else 2) for v, r in pairs)
    assert {v for v, _ in pairs} == set(range(1, 103))


def test_cc_example_file_input(tmp_path):
    import subprocess
    k = _kats()["ConnectedComponentsTest"]
    f = tmp_path / "edges.txt"
    f.write_text("".join("%d %d\n" % (a, b) for a, b in k["edges"]))
    out = subprocess.check_output([_example_bin(), str(f), "2", "1"], timeout=120).decode()
    last = {}
    for v, r in _parse_pairs(out):
        last[v] = r
    comps = {}
    for v, r in last.items():
        comps.setdefault(r, []).append(v)
    assert sorted(", ".join(map(str, sorted(m))) for m in comps.values()) == k["expect_final_components"]


# ---------------- bench.py multi-rank path (2 ranks on one GPU, gloo-staged exchange) ----------------
@pytest.mark.parametrize("scaling", ["strong", "weak"])
@pytest.mark.parametrize("merge", ["allgather", "gather", "tree"])
def test_bench_two_ranks_one_gpu_verified(merge, scaling):
    import subprocess, sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--scale", "16", "--edge-factor", "16",
           "--window-log2", "16", "--dist-backend", "gloo", "--verify", "--merge", merge, "--scaling", scaling]
    out = subprocess.check_output(cmd, env=env, timeout=240).decode()
    line = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == scaling
    assert line["config"]["edges_total"] == (1 << 20) * (2 if scaling == "weak" else 1)
    assert line["verify"] == {"edges_consistent": True, "labels_minimal_idempotent": True, "equals_torch_cc": True}


@pytest.mark.parametrize("extra", [["--id-bits", "64"], ["--host-input"], ["--host-input", "--id-bits", "64"],
                                   ["--workload", "c3_single"], ["--emit-host"], ["--emit-host", "--emit-sync"],
                                   ["--exchange-world1"]],
                         ids=["int64", "host", "host_int64", "single_window", "emit_host", "emit_host_sync",
                              "exchange_world1"])
def test_bench_lines_verified(extra):
    """The extra bench lines (int64 ids, pinned-host input through the double-buffered staging,
    one window, per-window host emission async and blocking, the C-ABI exchange over RCCL at world
    1), end to end against the independent torch CC, at RMAT-22 / 2^20-edge windows. stdout is the
    one JSON line (RCCL's banner and every other native print go to stderr)."""
    import subprocess, sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--steps", "1", "--warmup", "0", "--scale", "22",
           "--edge-factor", "16", "--no-cpu-baseline", "--verify"] + extra
    if "--workload" not in extra:
        cmd += ["--window-log2", "20"]
    out = subprocess.check_output(cmd, timeout=300).decode()
    assert len(out.strip().splitlines()) == 1, out[:2000]
    line = json.loads(out)
    assert line["verify"] == {"edges_consistent": True, "labels_minimal_idempotent": True, "equals_torch_cc": True}
    if "--emit-host" in extra:
        assert line["emit_host"]["windows"] > 0

# ---------------- BASELINE configs at full size, per-window bit-exact vs the C oracle ----------------
def _device_stream(gen_kind, n, param, seed):
    import torch
    from gsgpu import gen
    s = torch.empty(n, dtype=torch.int32, device="cuda")
    d = torch.empty(n, dtype=torch.int32, device="cuda")
    if gen_kind == "rmat":
        gen.rmat(s, d, 0, param, seed)
    else:
        gen.erdos_renyi(s, d, 0, param, seed)
    torch.cuda.synchronize()
    return s, d


@pytest.mark.parametrize("cfg", [("rmat", 20, 1 << 20, 16 << 20, 1 << 20, 1),       # configs[1] (C2)
                                 ("er", 1 << 24, 1 << 24, 1 << 24, 1 << 20, 2)],    # configs[3] (C4)
                         ids=["C2_rmat20_ef16_w1M", "C4_er_n2^24_m2^24_w1M"])
def test_baseline_config_per_window_vs_oracle(oracle, torch_cuda, cfg):
    kind, param, cap, n, W, seed = cfg
    s, d = _device_stream(kind, n, param, seed)
    ds = DisjointSet(cap, id_bits=32, stream=torch_cuda.cuda.current_stream())
    got = []
    for lo in range(0, n, W):
        ds.fold(s[lo:lo + W], d[lo:lo + W])
        ds.close_window()
        got.append(ds.checksum())
    hs = s.cpu().numpy().astype(np.int64)
    hd = d.cpu().numpy().astype(np.int64)
    want = oracle.run(hs, hd, W, partitions=8, threads=8, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    assert [g[0] for g in got] == [int(x) for x in want["checksums"]]
    np.testing.assert_array_equal(ds.dense().astype(np.int64), want["final"])
    assert got[-1][1:] == (want["final_vertices"], want["final_components"])


def test_c5_small_windows_vs_oracle(oracle, torch_cuda):
    """configs[4] shape (RMAT power-law, 64K-edge windows), first 4M edges of the RMAT-24 stream."""
    n, W, cap = 1 << 22, 1 << 16, 1 << 24
    s, d = _device_stream("rmat", n, 24, 3)
    ds = DisjointSet(cap, id_bits=32, stream=torch_cuda.cuda.current_stream())
    got = []
    for lo in range(0, n, W):
        ds.fold(s[lo:lo + W], d[lo:lo + W])
        ds.close_window()
        got.append(ds.checksum()[0])
    want = oracle.run(s.cpu().numpy().astype(np.int64), d.cpu().numpy().astype(np.int64), W, partitions=4,
                      threads=4, emit=EMIT_CHECKSUM, label_cap=cap)
    assert got == [int(x) for x in want["checksums"]]


@pytest.mark.parametrize("degree", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("case", _streams()[:3], ids=lambda c: c["name"])
def test_connected_components_tree(case, degree):
    """ConnectedComponentsTree(mergeWindowTime, degree): same canonical emissions per window."""
    from gsgpu import ConnectedComponentsTree
    stream = SimpleEdgeStream(case["src"], case["dst"])
    cc = ConnectedComponentsTree(1000, degree, window_edges=case["window_edges"], vertex_capacity=case["cap"],
                                 id_bits=32)
    for w, ds in enumerate(stream.aggregate(cc)):
        np.testing.assert_array_equal(ds.dense().astype(np.int64), case["labels"][w])


def test_cpp_connected_components_tree_matches_bulk(oracle):
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "gelly-streaming_amd", "gsgpu", "lib", "cc_tree_check")
    s, d = oracle.gen_rmat(0, 20000, 11, 13)
    txt = "".join("%d %d\n" % (a, b) for a, b in zip(s.tolist(), d.tolist()))
    for window, degree in ((1000, 4), (777, 3), (5000, 8)):
        out = subprocess.run([exe, str(window), str(degree)], input=txt.encode(), capture_output=True, timeout=120)
        assert out.returncode == 0, out.stdout.decode() + out.stderr.decode()
        assert "DIFF" not in out.stdout.decode()


# ---------------- edge-file ingestion (ConnectedComponentsExample.java:108-119 rules) ----------------
def _java_parse(text: bytes):
    """Reference semantics: per line, fields = line.split("\\\\s") (trailing empties dropped),
    Long.parseLong(fields[0]), Long.parseLong(fields[1]); returns (src, dst) or the bad line index."""
    import re
    lines = text.decode().split("\n")
    if lines and lines[-1] == "":
        lines = lines[:-1]
    src, dst = [], []
    for i, ln in enumerate(lines):
        f = re.split(r"[ \t\n\x0b\f\r]", ln)
        while f and f[-1] == "":
            f.pop()
        ok = len(f) >= 2 and all(re.fullmatch(r"[+-]?[0-9]+", x) for x in f[:2])
        if ok:
            a, b = int(f[0]), int(f[1])
            ok = -(1 << 63) <= a < (1 << 63) and -(1 << 63) <= b < (1 << 63)
        if not ok:
            return i
        src.append(a)
        dst.append(b)
    return np.array(src, dtype=np.int64), np.array(dst, dtype=np.int64)


def test_parse_edges_valid_forms():
    from gsgpu.edgefile import parse_edges
    text = b"1 2\n3\t4\n5 6 extra fields\n+7 -8\r\n9 10  \n" + b"".join(b"%d %d\n" % (i, i * 7 % 1000) for i in range(5000)) + b"11 12"
    want = _java_parse(text)
    got = parse_edges(text, id_bits=64)
    np.testing.assert_array_equal(got[0], want[0])
    np.testing.assert_array_equal(got[1], want[1])


@pytest.mark.parametrize("bad", [b"1  2\n", b"\n", b" 1 2\n", b"1x 2\n", b"1\n", b"1 99999999999999999999\n"])
def test_parse_edges_rejects_what_java_rejects(bad):
    from gsgpu.edgefile import parse_edges
    text = b"5 6\n7 8\n" + bad + b"9 10\n"
    assert _java_parse(text) == 2
    with pytest.raises(GsError) as ei:
        parse_edges(text, id_bits=64)
    assert ei.value.code == _abi.GS_ERR_INVALID and "line 3" in str(ei.value)


def test_parse_edges_large_random_and_fold(oracle):
    from gsgpu.edgefile import parse_edges
    s, d = oracle.gen_rmat(0, 300000, 16, 2)
    text = "".join("%d %d\n" % (a, b) for a, b in zip(s.tolist(), d.tolist())).encode()
    ps, pd = parse_edges(text, id_bits=32)
    np.testing.assert_array_equal(ps, s)
    np.testing.assert_array_equal(pd, d)


def test_parse_edges_long_lines_extremes_and_device_text(torch_cuda):
    """Lines longer than the kernel's 48-byte window (parsed from memory), int64 extremes and
    leading zeros, 4 KiB chunk boundaries at every offset, and device text at a misaligned
    address (copied to aligned scratch) against the Java rules."""
    import ctypes
    from gsgpu._abi import call
    from gsgpu.edgefile import parse_edges
    torch = torch_cuda
    rng = np.random.default_rng(7)
    lines = []
    for i in range(20000):
        k = i % 7
        if k == 0:
            lines.append(b"%d %d" % (rng.integers(0, 1 << 62), -int(rng.integers(0, 1 << 62))))
        elif k == 1:
            lines.append(b"-9223372036854775808 9223372036854775807 trailing fields here")
        elif k == 2:
            lines.append(b"000000000000000000000000000042 +0000000000000000000000000007\t\t")
        elif k == 3:
            lines.append(b"%d\t%d" % (i, i + 1) + b" " * int(rng.integers(0, 40)))
        else:
            lines.append(b"%d %d" % (rng.integers(0, 1000), rng.integers(0, 1000)))
    text = b"\n".join(lines) + b"\n"
    want = _java_parse(text)
    got = parse_edges(text, id_bits=64)
    np.testing.assert_array_equal(got[0], want[0])
    np.testing.assert_array_equal(got[1], want[1])
    buf = torch.zeros(len(text) + 3, dtype=torch.uint8, device="cuda")
    buf[3:] = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
    n = len(want[0])
    ps = torch.empty(n, dtype=torch.int64, device="cuda")
    pd = torch.empty(n, dtype=torch.int64, device="cuda")
    cnt = ctypes.c_uint64()
    torch.cuda.synchronize()
    call("gs_parse_edges", ctypes.c_void_p(buf.data_ptr() + 3), len(text), 64, ctypes.c_void_p(ps.data_ptr()),
         ctypes.c_void_p(pd.data_ptr()), n, ctypes.byref(cnt), 0, None)
    assert cnt.value == n
    np.testing.assert_array_equal(ps.cpu().numpy(), want[0])
    np.testing.assert_array_equal(pd.cpu().numpy(), want[1])
    bad = text + b"1 99999999999999999999\n5 6\n"
    assert _java_parse(bad) == n
    with pytest.raises(GsError):
        parse_edges(bad, id_bits=64)


def _dev_parse(torch, text, id_bits=64, cap=None):
    """gs_parse_edges with device text and device outputs (what bench.py's parse line times)."""
    import ctypes
    from gsgpu._abi import call
    buf = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
    cap = (text.count(b"\n") + 1) if cap is None else cap
    dt = torch.int64 if id_bits == 64 else torch.int32
    ps = torch.full((max(cap, 1),), -7, dtype=dt, device="cuda")
    pd = torch.full((max(cap, 1),), -7, dtype=dt, device="cuda")
    cnt = ctypes.c_uint64()
    torch.cuda.synchronize()
    call("gs_parse_edges", ctypes.c_void_p(buf.data_ptr()), len(text), id_bits, ctypes.c_void_p(ps.data_ptr()),
         ctypes.c_void_p(pd.data_ptr()), cap, ctypes.byref(cnt), 0, None)
    n = cnt.value
    return n, ps[:n].cpu().numpy().astype(np.int64), pd[:n].cpu().numpy().astype(np.int64)


def test_parse_edges_device_outputs(torch_cuda):
    """Device text and device outputs against the Java rules: valid forms, every rejected form past
    the first chunk, texts of 1 B to a few chunks at every length class (no trailing '\\n', exactly
    4096 B, one line per chunk), int32 outputs, the capacity error, and ~20K chunks of random text,
    equal to the host-output path. (Written for the one-pass look-back parse, which was measured
    slower and removed: profiles/r04_parse_onepass_ab.txt.)"""
    from gsgpu.edgefile import parse_edges
    torch = torch_cuda
    text = b"1 2\n3\t4\n5 6 extra fields\n+7 -8\r\n9 10  \n" + b"".join(b"%d %d\n" % (i, i * 7 % 1000) for i in range(5000)) + b"11 12"
    want = _java_parse(text)
    n, s, d = _dev_parse(torch, text)
    assert n == len(want[0])
    np.testing.assert_array_equal(s, want[0])
    np.testing.assert_array_equal(d, want[1])
    for bad in (b"1  2\n", b"\n", b" 1 2\n", b"1x 2\n", b"1\n", b"1 99999999999999999999\n"):
        head = b"".join(b"%d %d\n" % (i, i) for i in range(600))        # the bad line past chunk 0
        t = head + bad + b"9 10\n"
        assert _java_parse(t) == 600
        with pytest.raises(GsError) as ei:
            _dev_parse(torch, t)
        assert ei.value.code == _abi.GS_ERR_INVALID and "line 601" in str(ei.value)
    for t in (b"5 6", b"5 6\n", b"123456789 987654321", b"1 2\n" * 1024, b"1 2\n" * 1023 + b"12 3",
              b"7 8" + b" " * 4093, (b"4 5" + b" " * 4092 + b"\n") * 3, b"1 2\n" * 3000 + b"3 4"):
        want = _java_parse(t)
        n, s, d = _dev_parse(torch, t)
        assert n == len(want[0]), len(t)
        np.testing.assert_array_equal(s, want[0])
        np.testing.assert_array_equal(d, want[1])
    t = b"".join(b"%d %d\n" % (i, 4000000000 - i) for i in range(9000))
    n, s, d = _dev_parse(torch, t, id_bits=32)
    assert n == 9000
    np.testing.assert_array_equal(s, np.arange(9000))
    np.testing.assert_array_equal(d & 0xFFFFFFFF, 4000000000 - np.arange(9000))
    with pytest.raises(GsError) as ei:
        _dev_parse(torch, t, cap=8999)
    assert ei.value.code == _abi.GS_ERR_CAPACITY
    rng = np.random.default_rng(5)
    a = rng.integers(0, 1 << 24, 1 << 22)
    b = rng.integers(0, 1 << 24, 1 << 22)
    big = ("\n".join("%d %d" % (x, y) for x, y in zip(a.tolist(), b.tolist())) + "\n").encode()
    n, s, d = _dev_parse(torch, big)
    assert n == len(a)
    np.testing.assert_array_equal(s, a)
    np.testing.assert_array_equal(d, b)
    part = big[: big.rfind(b"\n", 0, 1 << 20) + 1] + b"77 88"
    hs, hd = parse_edges(part, id_bits=64)
    n2, s2, d2 = _dev_parse(torch, part)
    assert n2 == len(hs)
    np.testing.assert_array_equal(s2, hs)
    np.testing.assert_array_equal(d2, hd)
