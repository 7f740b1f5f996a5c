"""CPU, multi-process: the multi-GPU CombineCC exchanges (tests/gloo_tree.py: flat gather, pairwise
tree, replicated all-pairs delta exchange) under gloo, world 2 and 4.

Each rank folds its contiguous slice of every window into a CPU summary model with the same
export/fold contract as the device summary (oracle/pyoracle.py: PyMarkedSummary); the ranks run
the log2(P) pairwise tree; rank 0's emission after every window must equal the oracle pipeline's
(oracle/pipeline.c, same windows and partitions) bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, src, dst, W, cap, outdir, kind):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "gelly-streaming_amd"), os.path.join(root, "oracle"), os.path.join(root, "tests")]
    from gloo_tree import AllgatherMerge, GatherMerge, TreeMerge
    from pyoracle import PyMarkedSummary
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        summ = PyMarkedSummary(cap, track_marks=(kind == "allgather" or rank != 0))
        cls = {"tree": TreeMerge, "gather": GatherMerge, "allgather": AllgatherMerge}[kind]
        tm = cls(summ, capacity_pairs=cap, device=torch.device("cpu"))
        emis = []
        n = len(src)
        for lo in range(0, n, W):
            ln = min(W, n - lo)
            a, b = lo + (ln * rank) // world, lo + (ln * (rank + 1)) // world
            if kind == "gather":
                tm.before_fold()
            summ.fold(src[a:b], dst[a:b])
            if tm.merge_window() or kind == "allgather":      # allgather: every rank is a replica
                emis.append(summ.dense())
        if kind == "gather":
            tm.drain()
        if rank == 0 or kind == "allgather":
            np.save(os.path.join(outdir, "emis%d.npy" % rank), np.stack(emis))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["tree", "gather", "allgather"])
@pytest.mark.parametrize("world", [2, 4])
def test_tree_merge_gloo_matches_oracle(tmp_path, oracle, world, kind):
    s, d = oracle.gen_rmat(0, 6000, 10, 21)
    # add self-loop singletons that only a non-zero rank sees
    s = np.concatenate([s, [1000, 1001]]); d = np.concatenate([d, [1000, 1001]])
    cap, W = 1024, 1000
    mp.spawn(_worker, args=(world, _free_port(), s, d, W, cap, str(tmp_path), kind), nprocs=world, join=True)
    from pyoracle import EMIT_DENSE
    want = oracle.run(s, d, W, partitions=world, emit=EMIT_DENSE, label_cap=cap)["labels"]
    for r in range(world if kind == "allgather" else 1):
        got = np.load(tmp_path / ("emis%d.npy" % r))
        assert got.shape == want.shape
        np.testing.assert_array_equal(got, want, err_msg="rank %d" % r)


@pytest.mark.parametrize("kind", ["tree", "gather"])
def test_exports_of_twice_the_capacity(tmp_path, oracle, kind):
    """A window of self-loops on every vertex that also joins them all: each vertex is exported
    twice (its self-loop first touch, then its hook), 2 x capacity - 1 pairs per export, which the
    tree and gather models must carry (they used to reject n > capacity)."""
    cap = 256
    v = np.arange(cap, dtype=np.int64)
    s = np.concatenate([v, v[:-1]])                 # self-loops, then the chain v -- v+1
    d = np.concatenate([v, v[1:]])
    # every rank's slice of the one window: self-loops and chain links, so each export is big
    order = np.argsort(np.concatenate([2 * v, 2 * v[:-1] + 1]), kind="stable")
    s, d = s[order], d[order]
    W = len(s)
    mp.spawn(_worker, args=(2, _free_port(), s, d, W, cap, str(tmp_path), kind), nprocs=2, join=True)
    from pyoracle import EMIT_DENSE
    want = oracle.run(s, d, W, partitions=2, emit=EMIT_DENSE, label_cap=cap)["labels"]
    got = np.load(tmp_path / "emis0.npy")
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("bulk", [False, True])
def test_fold_slots_covers_real_pairs_only(monkeypatch, bulk):
    """AllgatherMerge's padded slots: every real pair is folded, no empty (garbage) slot is, and
    padding is only ever a copy of its own slot's first pair."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "gelly-streaming_amd"), os.path.join(root, "tests")]
    import gloo_tree as tree
    if bulk:
        monkeypatch.setattr(tree, "BULK_DELTA_PAIRS", 2)
    m, counts = 4, [3, 0, 4, 1, 0, 2]
    buf = torch.full((2 * m * len(counts),), -7, dtype=torch.int32)     # -7: garbage
    real = set()
    for q, c in enumerate(counts):
        for i in range(m if c else 0):
            j = i if i < c else 0                                         # padding = first pair
            buf[2 * (q * m + i)] = 100 * q + j
            buf[2 * (q * m + i) + 1] = 100 * q + j + 50
        real |= {(100 * q + j, 100 * q + j + 50) for j in range(c)}

    class Rec:
        def __init__(self):
            self.got = set()

        def fold_pairs(self, b, n, id_bits=32):
            p = b[: 2 * n].view(-1, 2).tolist()
            assert len(p) == n
            self.got |= {tuple(x) for x in p}

    r = Rec()
    tree.fold_slots(r, buf, m, counts)
    assert r.got == real
