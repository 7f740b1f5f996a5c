"""GPU parity of the multi-GPU CombineCC under the C ABI (gs_comm_* / gs_cc_merge_window,
csrc/comm.hip): every emission bit-exact vs the C oracle run with the same number of partitions
(the reference's SummaryBulkAggregation dataflow, SummaryBulkAggregation.java:68-90;
ConnectedComponentsTree, SummaryTreeReduce.java:95-123).

* world 1 through RCCL itself (ncclCommInitRank with one rank: the exchange code path with real
  RCCL collectives; a one-GPU box cannot host two RCCL ranks);
* world 2..8 through the in-process group (gs_comm_create_local): one thread per rank, every
  rank a handle on this GPU — the same exchange code, collectives by device copies;
* sparse-id summaries (GS_CC_SPARSE_IDS: any Java long, the reference's K = Long,
  ConnectedComponentsExample.java:61) through the exchange: (id, root id) int64 pairs.
"""
import threading

import numpy as np
import pytest

import gsgpu
from gsgpu import Comm, DisjointSet
from gsgpu.comm import unique_id
from pyoracle import EMIT_CHECKSUM

pytestmark = pytest.mark.gpu


def _stream(oracle, scale=14, n=300000, seed=8):
    s, d = oracle.gen_rmat(0, n, scale, seed)
    cap = 1 << scale
    # the largest ids, a self-loop and a duplicate at the end
    s = np.concatenate([s, [cap - 1, cap - 2, 5, 5]])
    d = np.concatenate([d, [cap - 2, cap - 1, 5, 5]])
    return s, d, cap


@pytest.mark.parametrize("mode", ["allgather", "gather", "tree"])
def test_rccl_world1(oracle, mode):
    import torch
    s, d, cap = _stream(oracle)
    W = 30000
    want = oracle.run(s, d, W, partitions=1, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    comm = Comm.create(unique_id(), 0, 1, 0)
    ds = DisjointSet(cap, id_bits=32, track_marks=True, stream=torch.cuda.current_stream())
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    got = []
    for lo in range(0, s.size, W):
        ds.fold(ts[lo:lo + W], td[lo:lo + W])
        ds.merge_window(comm, mode)
        got.append(ds.checksum()[0])
    assert got == [int(x) for x in want["checksums"]]
    np.testing.assert_array_equal(ds.dense().astype(np.int64), want["final"])
    r, w, sent, recv, ex, ov = comm.info()
    assert (r, w, ex) == (0, 1, len(got))
    ds.close()
    comm.close()


def _long_ids(x):
    """A bijection of dense ids onto Java longs spread over the whole range (negatives, >= 2^32)."""
    x = np.asarray(x, dtype=np.uint64)
    return ((x * np.uint64(0x9E3779B97F4A7C15)) ^ np.uint64(0x5851F42D4C957F2D)).view(np.int64)


def _run_local(world, mode, s, d, cap, W, sparse=False):
    """One thread per rank: fold slice r of every window, merge_window; returns per-rank checksums.
    sparse: s, d are arbitrary int64 ids folded into GS_CC_SPARSE_IDS summaries (finals None)."""
    import torch
    comms = Comm.local_group(world, 0)
    ts = torch.from_numpy(s.astype(np.int64 if sparse else np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int64 if sparse else np.int32)).cuda()
    torch.cuda.synchronize()
    sums = [[] for _ in range(world)]
    finals = [None] * world
    errors = []

    def rank(r):
        try:
            ds = DisjointSet(cap, id_bits=64 if sparse else 32, track_marks=True, sparse=sparse)
            for lo in range(0, s.size, W):
                ln = min(W, s.size - lo)
                a, b = lo + (ln * r) // world, lo + (ln * (r + 1)) // world
                ds.fold(ts[a:b], td[a:b])
                ds.merge_window(comms[r], mode)
                sums[r].append(ds.checksum()[0])
            finals[r] = None if sparse else ds.dense().astype(np.int64)
            ds.close()
        except Exception as e:          # surfaced by the main thread
            errors.append((r, repr(e)))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank hung"
    info = [c.info() for c in comms]
    for c in comms:
        c.close()
    assert not errors, errors
    return sums, finals, info


@pytest.mark.parametrize("mode", ["allgather", "gather", "tree"])
@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_local_group_vs_oracle(oracle, world, mode):
    s, d, cap = _stream(oracle, seed=world)
    W = 40000
    want = oracle.run(s, d, W, partitions=world, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    sums, finals, info = _run_local(world, mode, s, d, cap, W)
    ranks = range(world) if mode == "allgather" else [0]     # allgather: every replica is the Merger
    for r in ranks:
        assert sums[r] == [int(x) for x in want["checksums"]], "rank %d" % r
        np.testing.assert_array_equal(finals[r], want["final"])
    assert all(i[4] == len(want["checksums"]) for i in info)
    if mode == "allgather":                  # every rank took the same speculative / exact decisions
        assert len({i[5] for i in info}) == 1


def test_local_group_young_windows_big_deltas(oracle):
    """Windows whose deltas exceed the bulk threshold (2^21 pairs): slots folded one per call."""
    s, d = oracle.gen_er(0, 1 << 23, 1 << 23, 3)
    cap = 1 << 23
    W = 1 << 23                                    # one window: ~4M-pair deltas per rank
    want = oracle.run(s, d, W, partitions=2, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    sums, finals, _ = _run_local(2, "allgather", s, d, cap, W)
    for r in range(2):
        assert sums[r] == [int(x) for x in want["checksums"]]
        np.testing.assert_array_equal(finals[r], want["final"])


@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("mode", ["allgather", "gather"])
@pytest.mark.parametrize("world", [2, 4])
def test_local_group_speculative_slot_overflow(oracle, world, mode, sparse):
    """The speculative slots (allgather: one per rank, all-gathered; gather: each sender's own,
    sent to rank 0) are sized from the last window's deltas: a tiny first window (one self-loop)
    then an Erdos-Renyi window whose deltas outgrow the 4K-pair slot — the tail round must carry the
    tails (allgather: overflow counted alike on every rank; gather: on rank 0), and every emission
    stays exact."""
    cap = 1 << 16
    W = 1 << 17
    s1 = np.zeros(W, dtype=np.int64)                 # window 1: the self-loop (0, 0), W times
    s2, d2 = oracle.gen_er(0, 3 * W, cap, 4)        # windows 2-4: 3 x 2^17 uniform edges
    s = np.concatenate([s1, s2]); d = np.concatenate([s1, d2])
    if sparse:                                       # (id, root id) int64 pairs: the tail rounds' offsets in
        s, d = _long_ids(s), _long_ids(d)            # 4-word pairs
    want = oracle.run(s, d, W, partitions=world, emit=EMIT_CHECKSUM, label_cap=0 if sparse else cap,
                      want_final=not sparse)
    sums, finals, info = _run_local(world, mode, s, d, cap, W, sparse=sparse)
    for r in (range(world) if mode == "allgather" else [0]):
        assert sums[r] == [int(x) for x in want["checksums"]], "rank %d" % r
        if not sparse:
            np.testing.assert_array_equal(finals[r], want["final"])
    if mode == "allgather":
        assert all(i[5] >= 1 for i in info) and len({i[5] for i in info}) == 1, info
    else:
        assert info[0][5] >= 1 and all(i[5] >= 1 for i in info[1:]), info


@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("mode", ["allgather", "gather"])
@pytest.mark.parametrize("world", [2, 4])
def test_lazy_verification_overflow_in_a_batch(oracle, world, mode, sparse):
    """The speculative all-gather is verified lazily (comm.hip settle_allgather): with
    gs_cc_fold_windows nothing consumes an emission between windows, so an outgrown slot's tail
    round runs only after the NEXT window's local fold. The final emission must still be exact and
    the overflow counted alike on every rank (the same stream as the per-window overflow test)."""
    import torch
    cap = 1 << 16
    W = 1 << 17
    s1 = np.zeros(W, dtype=np.int64)
    s2, d2 = oracle.gen_er(0, 3 * W, cap, 4)
    s = np.concatenate([s1, s2]); d = np.concatenate([s1, d2])
    if sparse:
        s, d = _long_ids(s), _long_ids(d)
    want = oracle.run(s, d, W, partitions=world, emit=EMIT_CHECKSUM, label_cap=0 if sparse else cap,
                      want_final=not sparse)
    assert W % world == 0
    per = []
    for r in range(world):
        idx = np.concatenate([np.arange(lo + (W * r) // world, lo + (W * (r + 1)) // world) for lo in range(0, s.size, W)])
        per.append((s[idx], d[idx]))
    comms = Comm.local_group(world, 0)
    finals, errors, ov = [None] * world, [], [None] * world

    def rank(r):
        try:
            dt = np.int64 if sparse else np.int32
            ts = torch.from_numpy(per[r][0].astype(dt)).cuda()
            td = torch.from_numpy(per[r][1].astype(dt)).cuda()
            ds = DisjointSet(cap, id_bits=64 if sparse else 32, track_marks=True, sparse=sparse)
            assert ds.fold_windows(ts, td, W // world, comm=comms[r], mode=mode) == s.size // W
            finals[r] = (ds.checksum()[0], None if sparse else ds.dense().astype(np.int64))
            ov[r] = comms[r].info()[5]
            ds.close()
        except Exception as e:
            errors.append((r, repr(e)))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank hung"
    for c in comms:
        c.close()
    assert not errors, errors
    for r in (range(world) if mode == "allgather" else [0]):
        assert finals[r][0] == int(want["checksums"][-1]), "rank %d" % r
        if not sparse:
            np.testing.assert_array_equal(finals[r][1], want["final"])
    assert all(o >= 1 for o in ov) and (mode == "gather" or len(set(ov)) == 1), ov


@pytest.mark.parametrize("mode", ["allgather", "gather", "tree"])
def test_mismatched_capacities_fail_every_rank(mode):
    """Every rank sizes its exchange buffers and speculative slots from its own summary: ranks whose
    capacities differ are refused when the communicator is bound, on every rank alike (ADVICE r04:
    the speculative gather's send and receive sizes would otherwise disagree)."""
    comms = Comm.local_group(2, 0)
    errors = [None, None]

    def rank(r):
        try:
            ds = DisjointSet(1 << (12 + r), id_bits=32, track_marks=True)
            ds.fold(np.array([1, 2]), np.array([2, 3]))
            ds.merge_window(comms[r], mode)
        except gsgpu.GsError as e:
            errors[r] = e.code
    th = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a rank hung"
    for c in comms:
        c.close()
    # (a rank that sees its peer's abort first reports the group failure, GS_ERR_COMM)
    assert set(errors) <= {gsgpu._abi.GS_ERR_INVALID, gsgpu._abi.GS_ERR_COMM} and gsgpu._abi.GS_ERR_INVALID in errors, errors


def test_merge_window_errors():
    """Argument errors fail the call AND the communicator (its peers would otherwise wait forever in
    the next collective): a later call on it returns GS_ERR_COMM."""
    comms = Comm.local_group(1, 0)
    ds = DisjointSet(64, id_bits=32)                  # no marks tracked
    with pytest.raises(gsgpu.GsError) as e:
        ds.merge_window(comms[0])
    assert e.value.code == gsgpu._abi.GS_ERR_UNSUPPORTED
    ds2 = DisjointSet(64, id_bits=32, track_marks=True)
    with pytest.raises(gsgpu.GsError) as e:
        ds2.merge_window(comms[0], "tree")
    assert e.value.code == gsgpu._abi.GS_ERR_COMM     # broken by the first failure
    comms[0].close()
    comms = Comm.local_group(1, 0)
    with pytest.raises(gsgpu.GsError) as e:
        gsgpu._abi.call("gs_cc_merge_window", ds2.handle, comms[0].handle, 7)
    assert e.value.code == gsgpu._abi.GS_ERR_INVALID
    comms[0].close()
    comms = Comm.local_group(1, 0)
    ds2.fold(np.array([1, 2]), np.array([2, 3]))
    ds2.merge_window(comms[0], "tree")                # world 1: a plain close
    assert ds2.getMatches() == {1: 1, 2: 1, 3: 1}
    with pytest.raises(gsgpu.GsError) as e:           # one communicator serves one handle and mode
        ds2.merge_window(comms[0], "gather")
    assert e.value.code == gsgpu._abi.GS_ERR_INVALID
    comms[0].close()


def test_failure_on_one_rank_fails_its_peers():
    """Rank 1 fails before its first collective (its handle tracks no marks); rank 0, already in
    the all-gather, must get an error instead of hanging."""
    comms = Comm.local_group(2, 0)
    errs = [None, None]

    def rank(r):
        try:
            ds = DisjointSet(1 << 10, id_bits=32, track_marks=(r == 0))
            ds.fold(np.array([1, 2]), np.array([2, 3]))
            ds.merge_window(comms[r], "allgather")
        except gsgpu.GsError as e:
            errs[r] = e.code

    th = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in th), "a rank hung"
    assert errs[1] == gsgpu._abi.GS_ERR_UNSUPPORTED and errs[0] == gsgpu._abi.GS_ERR_COMM, errs
    for c in comms:
        c.close()


def test_reset_restarts_the_exact_round(oracle):
    """After gs_cc_reset the first window of the new stream runs the exact round again (ADVICE r02:
    the speculative slot used to survive the reset, so every step's young first window overflowed):
    two identical passes take identical decisions, so the overflow count exactly doubles."""
    import torch
    s, d, cap = _stream(oracle, n=200000, seed=5)
    W = 25000
    world = 2
    comms = Comm.local_group(world, 0)
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    torch.cuda.synchronize()
    ov = [[None, None] for _ in range(world)]
    sums = [[] for _ in range(world)]
    errors = []

    def rank(r):
        try:
            ds = DisjointSet(cap, id_bits=32, track_marks=True)
            for step in range(2):
                ds.reset()
                for lo in range(0, s.size, W):
                    ln = min(W, s.size - lo)
                    a, b = lo + (ln * r) // world, lo + (ln * (r + 1)) // world
                    ds.fold(ts[a:b], td[a:b])
                    ds.merge_window(comms[r], "allgather")
                    sums[r].append(ds.checksum()[0])
                ov[r][step] = comms[r].info()[5]
            ds.close()
        except Exception as e:
            errors.append((r, repr(e)))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th) and not errors, errors
    for c in comms:
        c.close()
    want = oracle.run(s, d, W, partitions=world, emit=EMIT_CHECKSUM, label_cap=cap)
    for r in range(world):
        assert sums[r] == 2 * [int(x) for x in want["checksums"]]
        assert ov[r][1] == 2 * ov[r][0], ov


def test_c5_eight_ranks_small_windows_latency(oracle):
    """BASELINE config 5's layout at 8 ranks (in-process transport, one GPU): the RMAT-24 stream
    (seed 3) in 2^16-edge global windows, 2^13 edges per rank per window, allgather mode — every
    window's emission vs the oracle with 8 partitions; the per-window wall latency (fold + exchange
    + close on every rank, host-observed) is printed."""
    import time
    import torch
    from gsgpu import gen
    P, scale, W, N = 8, 24, 1 << 16, 48
    cap = 1 << scale
    s = torch.empty(N * W, dtype=torch.int32, device="cuda")
    d = torch.empty(N * W, dtype=torch.int32, device="cuda")
    gen.rmat(s, d, 0, scale, 3)
    torch.cuda.synchronize()
    hs, hd = s.cpu().numpy().astype(np.int64), d.cpu().numpy().astype(np.int64)
    want = oracle.run(hs, hd, W, partitions=P, threads=P, emit=EMIT_CHECKSUM, label_cap=cap)
    comms = Comm.local_group(P, 0)
    sums = [[] for _ in range(P)]
    lat = [[] for _ in range(P)]
    errors = []
    Wr = W // P

    def rank(r):
        try:
            ds = DisjointSet(cap, id_bits=32, track_marks=True)
            for w in range(N):
                t0 = time.perf_counter()
                lo = w * W + r * Wr
                ds.fold(s[lo:lo + Wr], d[lo:lo + Wr])
                ds.merge_window(comms[r], "allgather")
                ds.sync()
                lat[r].append((time.perf_counter() - t0) * 1e6)
                sums[r].append(ds.checksum()[0])
            ds.close()
        except Exception as e:
            errors.append((r, repr(e)))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th) and not errors, errors
    for c in comms:
        c.close()
    for r in range(P):
        assert sums[r] == [int(x) for x in want["checksums"]], "rank %d" % r
    steady = sorted(max(lat[r][w] for r in range(P)) for w in range(8, N))
    print("C5 8 ranks (in-process, one GPU): per-window latency p50 %.0f us, p99 %.0f us (max over ranks)"
          % (steady[len(steady) // 2], steady[min(len(steady) - 1, int(len(steady) * 0.99))]))


@pytest.mark.parametrize("world,mode", [(1, None), (1, "allgather"), (3, "allgather"), (3, "gather"), (4, "tree")])
def test_fold_windows_batch(oracle, world, mode):
    """gs_cc_fold_windows (the per-window fold + close / merge loop inside the library) ends in the
    same emission as the oracle's last window; every window is folded, and merged over the comm
    (RCCL at world 1, the in-process group beyond) — exchanges counted per window."""
    import torch
    s, d, cap = _stream(oracle, n=200000, seed=13)
    W = 25000
    want = oracle.run(s, d, W, partitions=world, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    nwin = (s.size + W - 1) // W
    if mode is None:
        ds = DisjointSet(cap, id_bits=32, stream=torch.cuda.current_stream())
        ts = torch.from_numpy(s.astype(np.int32)).cuda()
        td = torch.from_numpy(d.astype(np.int32)).cuda()
        assert ds.fold_windows(ts, td, W) == nwin
        assert ds.checksum()[0] == int(want["checksums"][-1])
        np.testing.assert_array_equal(ds.dense().astype(np.int64), want["final"])
        ds.close()
        return
    # rank r's slice of window w = the partition _run_local folds; laid out contiguously per rank
    # so one fold_windows call per rank takes every window
    per = []
    for r in range(world):
        ss, dd, lens = [], [], []
        for lo in range(0, s.size, W):
            ln = min(W, s.size - lo)
            a, b = lo + (ln * r) // world, lo + (ln * (r + 1)) // world
            ss.append(s[a:b]); dd.append(d[a:b]); lens.append(b - a)
        per.append((np.concatenate(ss), np.concatenate(dd), lens))
    if any(len(set(p[2][:-1])) > 1 or p[2][-1] > p[2][0] for p in per):
        pytest.skip("uneven rank slices: fold_windows takes one window size")
    comms = [Comm.create(unique_id(), 0, 1, 0)] if world == 1 else Comm.local_group(world, 0)
    finals, errors, wins = [None] * world, [], [0] * world

    def rank(r):
        try:
            ss, dd, lens = per[r]
            ts = torch.from_numpy(ss.astype(np.int32)).cuda()
            td = torch.from_numpy(dd.astype(np.int32)).cuda()
            ds = DisjointSet(cap, id_bits=32, track_marks=True)
            wins[r] = ds.fold_windows(ts, td, lens[0], comm=comms[r], mode=mode)
            finals[r] = (ds.checksum()[0], ds.dense().astype(np.int64))
            ds.close()
        except Exception as e:
            errors.append((r, repr(e)))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank hung"
    info = [c.info() for c in comms]
    for c in comms:
        c.close()
    assert not errors, errors
    assert wins == [nwin] * world
    assert all(i[4] == nwin for i in info), info            # one exchange per window
    for r in ([0] if mode in ("tree", "gather") else range(world)):   # tree / gather: rank 0 is the Merger
        assert finals[r][0] == int(want["checksums"][-1])
        np.testing.assert_array_equal(finals[r][1], want["final"])


def _sparse_ids(oracle, n, scale, seed):
    """An RMAT stream whose ids are spread over the whole int64 range (negative ids, ids >= 2^32,
    INT64_MIN and INT64_MAX among them) by a fixed injective map, as the reference's Long keys allow."""
    s, d = oracle.gen_rmat(0, n, scale, seed)
    mul = np.uint64(0x9E3779B97F4A7C15)                   # odd: a bijection of uint64
    with np.errstate(over="ignore"):
        ms = (s.astype(np.uint64) * mul).view(np.int64)
        md = (d.astype(np.uint64) * mul).view(np.int64)
    ms[:3] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max, -1]
    md[:3] = [-1, 5, np.iinfo(np.int64).min]
    return ms, md


@pytest.mark.parametrize("mode", ["allgather", "gather", "tree"])
@pytest.mark.parametrize("world", [1, 4])
def test_sparse_ids_through_the_exchange(oracle, world, mode):
    """Sparse (any int64) ids across ranks: every rank folds its slice of each window into a
    GS_CC_SPARSE_IDS handle; gs_cc_merge_window carries (id, root id) int64 pairs; the Merger's
    emission (every replica in allgather mode) equals the oracle's with `world` partitions, window
    by window (world 1: RCCL with one rank)."""
    import torch
    s, d = _sparse_ids(oracle, 120000, 14, 21 + world)
    W = 20000
    want = oracle.run(s, d, W, partitions=world, emit=EMIT_CHECKSUM)
    ts, td = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    torch.cuda.synchronize()
    comms = Comm.local_group(world, 0) if world > 1 else [Comm.create(unique_id(), 0, 1, 0)]
    sums = [[] for _ in range(world)]
    errors = []

    def rank(r):
        try:
            ds = DisjointSet(1 << 15, id_bits=64, track_marks=True, sparse=True)
            for lo in range(0, s.size, W):
                ln = min(W, s.size - lo)
                a, b = lo + (ln * r) // world, lo + (ln * (r + 1)) // world
                ds.fold(ts[a:b], td[a:b])
                ds.merge_window(comms[r], mode)
                sums[r].append(ds.checksum())
            ds.close()
        except Exception as e:
            errors.append((r, repr(e)))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank hung"
    for c in comms:
        c.close()
    assert not errors, errors
    exp = [(int(c), int(v), int(k)) for c, (v, k) in zip(want["checksums"], want["counts"])]
    for r in (range(world) if mode == "allgather" else [0]):
        assert [tuple(x) for x in sums[r]] == exp, "rank %d" % r
