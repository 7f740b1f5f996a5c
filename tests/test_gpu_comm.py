"""GPU parity of the multi-GPU CombineCC under the C ABI (gs_comm_* / gs_cc_merge_window,
csrc/comm.hip): every emission bit-exact vs the C oracle run with the same number of partitions
(the reference's SummaryBulkAggregation dataflow, SummaryBulkAggregation.java:68-90;
ConnectedComponentsTree, SummaryTreeReduce.java:95-123).

* world 1 through RCCL itself (ncclCommInitRank with one rank: the exchange code path with real
  RCCL collectives; a one-GPU box cannot host two RCCL ranks);
* world 2..8 through the in-process group (gs_comm_create_local): one thread per rank, every
  rank a handle on this GPU — the same exchange code, collectives by device copies.
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


def _run_local(world, mode, s, d, cap, W):
    """One thread per rank: fold slice r of every window, merge_window; returns per-rank checksums."""
    import torch
    comms = Comm.local_group(world, 0)
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    torch.cuda.synchronize()
    sums = [[] for _ in range(world)]
    finals = [None] * world
    errors = []

    def rank(r):
        try:
            ds = DisjointSet(cap, id_bits=32, track_marks=True)
            for lo in range(0, s.size, W):
                ln = min(W, s.size - lo)
                a, b = lo + (ln * r) // world, lo + (ln * (r + 1)) // world
                ds.fold(ts[a:b], td[a:b])
                ds.merge_window(comms[r], mode)
                sums[r].append(ds.checksum()[0])
            finals[r] = ds.dense().astype(np.int64)
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


@pytest.mark.parametrize("world", [2, 4])
def test_local_group_speculative_slot_overflow(oracle, world):
    """allgather's speculative slot is sized from the last window's deltas: a tiny first window
    (one self-loop) then an Erdos-Renyi window whose deltas outgrow the 4K-pair slot — the exact
    round must carry the tails (overflow counted on every rank), and every emission stays exact."""
    cap = 1 << 16
    W = 1 << 17
    s1 = np.zeros(W, dtype=np.int64)                 # window 1: the self-loop (0, 0), W times
    s2, d2 = oracle.gen_er(0, 3 * W, cap, 4)        # windows 2-4: 3 x 2^17 uniform edges
    s = np.concatenate([s1, s2]); d = np.concatenate([s1, d2])
    want = oracle.run(s, d, W, partitions=world, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    sums, finals, info = _run_local(world, "allgather", s, d, cap, W)
    for r in range(world):
        assert sums[r] == [int(x) for x in want["checksums"]], "rank %d" % r
        np.testing.assert_array_equal(finals[r], want["final"])
    assert all(i[5] >= 1 for i in info) and len({i[5] for i in info}) == 1, info


def test_merge_window_errors():
    comms = Comm.local_group(1, 0)
    ds = DisjointSet(64, id_bits=32)                  # no marks tracked
    with pytest.raises(gsgpu.GsError) as e:
        ds.merge_window(comms[0])
    assert e.value.code == gsgpu._abi.GS_ERR_UNSUPPORTED
    ds2 = DisjointSet(64, id_bits=32, track_marks=True)
    with pytest.raises(gsgpu.GsError):
        gsgpu._abi.call("gs_cc_merge_window", ds2.handle, comms[0].handle, 7)
    ds2.fold(np.array([1, 2]), np.array([2, 3]))
    ds2.merge_window(comms[0], "tree")                # world 1: a plain close
    assert ds2.getMatches() == {1: 1, 2: 1, 3: 1}
    comms[0].close()
