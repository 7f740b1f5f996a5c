"""GPU parity of GS_MERGE_PREFILTER (csrc/comm.hip merge_prefilter): ranks 1..P-1 filter their
slices of every window against the giant bitmap rank 0 broadcasts and send the survivors; rank 0
(the Merger, SummaryBulkAggregation.java:76-83 / SummaryAggregation.java:106-119) folds its own
slice and every survivor, closes and emits. Rank 0's emission after every window is compared,
bit-exact, with the C oracle's (canonical labels do not depend on the partitioning).

* in-process groups of 2, 3 and 8 ranks (one thread per rank on this GPU) and RCCL at world 1;
* uneven slices (rank 0's share of a window 1/16 .. 1/2), one call per window and one call per
  stream, int32 and int64 ids;
* speculative slots past the exact young rounds, and survivor bursts that outgrow them (tail rounds);
* a sender's out-of-range id (GS_ERR_RANGE on that rank, the others unaffected), sparse handles and
  gs_cc_merge_window with this mode (rejected).
The hot / warm-set paths of the senders (a giant switching components between broadcasts) run in
tests/variant_check.py under every fold variant (test_gpu_variants.py).
"""
import threading

import numpy as np
import pytest

from gsgpu import Comm, DisjointSet, GsError, _abi
from gsgpu.comm import unique_id
from pyoracle import EMIT_CHECKSUM
from variant_check import rank_slices, run_prefilter

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def _rmat(oracle, scale, n, seed):
    """n edges: RMAT, then the largest ids, a self-loop and a duplicate (every window of a multiple
    of the window size is full, so no rank's slice is empty: each rank exchanges every window)."""
    s, d = oracle.gen_rmat(0, n - 4, scale, seed)
    cap = 1 << scale
    s = np.concatenate([s, [cap - 1, cap - 2, 5, 5]])          # the largest ids, a self-loop, a duplicate
    d = np.concatenate([d, [cap - 2, cap - 1, 5, 5]])
    return s, d, cap


@pytest.mark.parametrize("world,share0", [(2, 0.5), (3, 0.125), (8, 0.0625)])
def test_prefilter_every_window_vs_oracle(oracle, torch_cuda, world, share0):
    s, d, cap = _rmat(oracle, 15, 400000, 21)
    r = run_prefilter(torch_cuda, oracle, "rmat15", s, d, 8000, cap, world=world, share0=share0)
    assert r["ok"], r


@pytest.mark.parametrize("id_bits", [32, 64])
def test_prefilter_one_call_per_stream(oracle, torch_cuda, id_bits):
    s, d, cap = _rmat(oracle, 16, 600000, 22)                   # 100 windows, the same slices each
    r = run_prefilter(torch_cuda, oracle, "rmat16_one_call", s, d, 6000, cap, world=4, share0=0.25,
                      per_window=False, id_bits=id_bits)
    assert r["ok"], r


def test_prefilter_survivor_bursts_outgrow_slots(oracle, torch_cuda):
    """After the exact young rounds the slots follow each sender's last survivor count; windows of
    fresh vertices (every edge survives) between RMAT windows outgrow them: tail rounds, still exact."""
    rng = np.random.default_rng(4)
    scale, W = 18, 20000                                         # sender slices 8000 > the 4096-pair floor
    cap = 1 << scale
    s0, d0 = oracle.gen_rmat(0, 40 * W, scale - 1, 23)          # ids < 2^17: the giant's half
    src, dst = [s0[:30 * W]], [d0[:30 * W]]
    fresh = np.arange(1 << 17, 1 << 18)
    rng.shuffle(fresh)
    for k in range(3):                                           # bursts of new vertices (pairs)
        f = fresh[k * 2 * W:(k + 1) * 2 * W]
        src += [f[0::2], s0[(30 + 2 * k) * W:(31 + 2 * k) * W]]
        dst += [f[1::2], d0[(30 + 2 * k) * W:(31 + 2 * k) * W]]
    s, d = np.concatenate(src).astype(np.int64), np.concatenate(dst).astype(np.int64)
    r = run_prefilter(torch_cuda, oracle, "bursts", s, d, W, cap, world=3, share0=0.2)
    assert r["ok"], r
    assert sum(r["overflows"]) > 0, r                            # the bursts did outgrow their slots


def test_prefilter_rccl_world1(oracle, torch_cuda):
    """World 1 through RCCL: rank 0 alone (no senders), the emission of every window."""
    torch = torch_cuda
    s, d, cap = _rmat(oracle, 14, 200000, 24)
    W = 9000                                                     # (a short last window: world 1)
    want = oracle.run(s, d, W, partitions=1, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    comm = Comm.create(unique_id(), 0, 1, 0)
    ds = DisjointSet(cap, id_bits=32, stream=torch.cuda.current_stream())
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    got = []
    for lo in range(0, s.size, W):
        assert ds.fold_windows(ts[lo:lo + W], td[lo:lo + W], W, comm=comm, mode="prefilter") == 1
        got.append(ds.checksum()[0])
    assert got == [int(x) for x in want["checksums"]]
    np.testing.assert_array_equal(ds.dense().astype(np.int64), want["final"])
    ds.close()
    comm.close()


def test_prefilter_sender_range_error(oracle, torch_cuda):
    """An id >= capacity in a sender's slice: that rank's call fails with GS_ERR_RANGE after the
    stream (its filters skip the edge, as a fold does); rank 0 folds the rest and stays exact."""
    torch = torch_cuda
    s, d, cap = _rmat(oracle, 14, 120000, 25)
    W, world = 6000, 3
    sl = rank_slices(s.size, W, world, 0.25)
    lo, hi = sl[2][7]
    bad_at = lo + 3
    keep = np.ones(s.size, bool)
    keep[bad_at] = False
    s_bad = s.copy()
    s_bad[bad_at] = cap + 5
    comms = Comm.local_group(world, 0)
    res, errs = [None] * world, [None] * world

    def rank(r):
        ds = DisjointSet(cap, id_bits=32)
        ts = torch.from_numpy(s_bad.astype(np.int32)).cuda()
        td = torch.from_numpy(d.astype(np.int32)).cuda()
        for lo_, hi_ in sl[r]:
            try:                                                 # (the exchange itself completed)
                ds.fold_windows(ts[lo_:hi_], td[lo_:hi_], hi_ - lo_, comm=comms[r], mode="prefilter")
            except GsError as e:
                errs[r] = e.code
        res[r] = ds.dense().astype(np.int64) if r == 0 else True
        ds.close()

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank hung"
    for c in comms:
        c.close()
    assert errs[2] == _abi.GS_ERR_RANGE and errs[0] is None and errs[1] is None, errs
    # rank 0's final labels = the oracle's over every edge but the bad one
    fin = oracle.run(s[keep], d[keep], s.size, partitions=1, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    np.testing.assert_array_equal(res[0], fin["final"])


def test_prefilter_rejected_where_it_cannot_run(torch_cuda):
    torch = torch_cuda
    comm = Comm.create(unique_id(), 0, 1, 0)
    ds = DisjointSet(1 << 12, id_bits=32, track_marks=True, stream=torch.cuda.current_stream())
    ds.fold(torch.tensor([1, 2], dtype=torch.int32).cuda(), torch.tensor([2, 3], dtype=torch.int32).cuda())
    with pytest.raises(GsError) as ei:
        ds.merge_window(comm, "prefilter")                       # needs the window's edges
    assert ei.value.code == _abi.GS_ERR_INVALID
    ds.close()
    comm.close()
    comm = Comm.create(unique_id(), 0, 1, 0)
    sp = DisjointSet(1 << 12, id_bits=64, sparse=True, stream=torch.cuda.current_stream())
    t = torch.tensor([1, 2], dtype=torch.int64).cuda()
    with pytest.raises(GsError) as ei:
        sp.fold_windows(t, t, 2, comm=comm, mode="prefilter")
    assert ei.value.code == _abi.GS_ERR_UNSUPPORTED
    sp.close()
    comm.close()


def test_prefilter_host_edge_buffers(oracle, torch_cuda):
    """Host (numpy) slices on every rank: the senders' pre-filter stages them to the device
    (cc_filter_async's staging copy), rank 0's fold takes its host path; every window vs the oracle."""
    from variant_check import rank_slices
    s, d, cap = _rmat(oracle, 14, 96000, 26)
    W, world = 6000, 3
    want = oracle.run(s, d, W, partitions=world, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    sl = rank_slices(s.size, W, world, 0.3)
    s32, d32 = s.astype(np.int32), d.astype(np.int32)
    comms = Comm.local_group(world, 0)
    got, errs = [], []

    def rank(r):
        try:
            ds = DisjointSet(cap, id_bits=32)
            for lo, hi in sl[r]:
                ds.fold_windows(s32[lo:hi], d32[lo:hi], hi - lo, comm=comms[r], mode="prefilter")
                if r == 0:
                    got.append(ds.checksum()[0])
            ds.close()
        except Exception as e:                                   # noqa: BLE001
            errs.append((r, repr(e)))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank hung"
    for c in comms:
        c.close()
    assert not errs, errs
    assert got == [int(x) for x in want["checksums"]]


def test_prefilter_through_the_cpp_mirror(oracle, torch_cuda):
    """The C++ host mirror (csrc/host/gsgpu.hpp: Comm::local, DisjointSet::foldWindows) running the
    Merger-rank layout over 4 in-process ranks (csrc/host/cc_prefilter_check.cpp): rank 0's emission
    checksum, vertices and components after every window vs the oracle."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "gelly-streaming_amd", "gsgpu", "lib", "cc_prefilter_check")
    s, d, cap = _rmat(oracle, 14, 60000, 27)
    W, world = 5000, 4
    want = oracle.run(s, d, W, partitions=world, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    text = "".join("%d %d\n" % (a, b) for a, b in zip(s.tolist(), d.tolist()))
    out = subprocess.run([exe, str(W), str(world), "0.25", str(cap)], input=text, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    rows = [line.split() for line in out.stdout.splitlines()]
    assert len(rows) == len(want["checksums"])
    assert [int(r[1]) for r in rows] == [int(x) for x in want["checksums"]]


def _run_threads(world, body):
    comms = Comm.local_group(world, 0)
    errs = []

    def rank(r):
        try:
            body(r, comms[r])
        except Exception as e:                                   # noqa: BLE001
            errs.append((r, repr(e)))
    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank hung"
    for c in comms:
        c.close()
    assert not errs, errs


def test_prefilter_empty_slices(oracle, torch_cuda):
    """a rank whose slice of a window is empty still joins that window's exchange.
    (a) one call per window, the last global window shorter than the ranks (3 edges over 4 ranks:
    one rank's slice is empty, its call has n == 0); (b) one call per stream where rank 0 folds no
    slice at all (n == 0: it only merges, bench.py's layout at P = 8) and the senders' streams differ
    in length by that short last window. Rank 0's emission vs the oracle."""
    torch = torch_cuda
    s, d, cap = _rmat(oracle, 13, 24003, 28)
    W, world = 2000, 4
    want = oracle.run(s, d, W, partitions=1, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    nwin = len(want["checksums"])
    assert s.size % W == 3
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    got, fin = [], {}

    def per_window(r, comm):
        ds = DisjointSet(cap, id_bits=32)
        for w in range(nwin):
            lo = w * W
            ln = min(W, s.size - lo)
            a, b = lo + ln * r // world, lo + ln * (r + 1) // world
            nw = ds.fold_windows(ts[a:b], td[a:b], max(b - a, 1), comm=comm, mode="prefilter")
            assert nw == 1
            if r == 0:
                got.append(ds.checksum()[0])
        ds.close()
    _run_threads(world, per_window)
    assert got == [int(x) for x in want["checksums"]]

    def per_stream(r, comm):                     # rank 0: nothing; ranks 1..3: a third of each window
        ds = DisjointSet(cap, id_bits=32)
        parts_s, parts_d = [], []
        for w in range(nwin):
            lo = w * W
            ln = min(W, s.size - lo)
            if r:
                a, b = lo + ln * (r - 1) // (world - 1), lo + ln * r // (world - 1)
                parts_s.append(ts[a:b])
                parts_d.append(td[a:b])
        es = torch.cat(parts_s) if parts_s else ts[:0]
        ed = torch.cat(parts_d) if parts_d else td[:0]
        per = W // (world - 1) if r else 1
        nw = ds.fold_windows(es, ed, per, comm=comm, mode="prefilter")
        assert nw == nwin
        if r == 0:
            fin["sum"] = ds.checksum()[0]
            fin["dense"] = ds.dense().astype(np.int64)
        ds.close()
    # (W = 2000 splits into 666 / 667 / 667: equal per-window slices need W % 3 == 0 for a one-call
    # stream, so this part uses 1998-edge windows)
    W = 1998
    want = oracle.run(s, d, W, partitions=1, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    nwin = len(want["checksums"])
    _run_threads(world, per_stream)
    assert fin["sum"] == int(want["checksums"][-1])
    np.testing.assert_array_equal(fin["dense"], want["final"])


def test_prefilter_sender_slice_above_capacity(oracle, torch_cuda):
    """a sender's slice of a window may exceed the 2 x capacity pairs the exchange
    buffers are sized for (every edge of it may survive): its send buffers grow to the slice."""
    torch = torch_cuda
    scale = 10
    s, d = oracle.gen_rmat(0, 24000, scale, 29)
    cap = 1 << scale
    W, world = 12000, 2                          # sender slices of 9000 edges > 2 x 1024 - 1
    want = oracle.run(s, d, W, partitions=1, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    got = []

    def body(r, comm):
        ds = DisjointSet(cap, id_bits=32)
        for w in range(2):
            lo = w * W
            a, b = (lo, lo + 3000) if r == 0 else (lo + 3000, lo + W)
            ds.fold_windows(ts[a:b], td[a:b], b - a, comm=comm, mode="prefilter")
            if r == 0:
                got.append(ds.checksum()[0])
        ds.close()
    _run_threads(world, body)
    assert got == [int(x) for x in want["checksums"]]
