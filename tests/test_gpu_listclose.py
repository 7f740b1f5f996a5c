"""GPU parity of the list-mode close (cc_kernels.hpp ListCtl): small windows whose close visits the
seen vertices outside the giant plus the window's first touches instead of V-bit bitmaps.

Every window's emission is bit-exact against the C oracle while the stream switches between list,
bitmap and full closes: windows folded in several calls, windows folded as pairs (a fold that does
not log), many small folds in one window, NGL overflow (an Erdos-Renyi
stream before its giant), empty intervals (two closes in a row), delta emission turned on mid-stream,
and a reset between passes.
"""
import numpy as np
import pytest

from gsgpu import DisjointSet
from pyoracle import EMIT_CHECKSUM, dense_checksum

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def _fold_window(ds, torch, ts, td, lo, hi, w):
    if w % 11 == 5:                                   # partial-summary path: pairs (not logged)
        pairs = torch.stack([ts[lo:hi], td[lo:hi]], dim=1).contiguous().view(-1)
        ds.fold_pairs(pairs)
    elif w % 7 == 3:                                  # several logged folds in one interval
        a, b = lo + (hi - lo) // 3, lo + 2 * (hi - lo) // 3
        for x, y in ((lo, a), (a, b), (b, hi)):
            ds.fold(ts[x:y], td[x:y])
    elif w % 17 == 9:                                 # 16 one-workgroup folds in one interval
        step = max(1, (hi - lo) // 16)
        for x in range(lo, hi, step):
            ds.fold(ts[x:min(hi, x + step)], td[x:min(hi, x + step)])
    else:
        ds.fold(ts[lo:hi], td[lo:hi])


@pytest.mark.parametrize("gen,scale,n,W", [("rmat", 16, 1 << 19, 4096), ("er", 16, 1 << 18, 2048),
                                           ("rmat", 20, 1 << 21, 1 << 14)])
def test_list_close_mixed_operations_vs_oracle(oracle, torch_cuda, gen, scale, n, W):
    torch = torch_cuda
    cap = 1 << scale
    if gen == "rmat":
        s, d = oracle.gen_rmat(0, n, scale, 11)
    else:
        s, d = oracle.gen_er(0, n, cap, 13)
    want = oracle.run(s, d, W, partitions=4, threads=4, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    ds = DisjointSet(cap, id_bits=32, stream=torch.cuda.current_stream())
    for step in range(2):
        ds.reset()
        mirror = np.full(cap, -1, dtype=np.int64)
        nwin = (n + W - 1) // W
        for w, lo in enumerate(range(0, n, W)):
            _fold_window(ds, torch, ts, td, lo, min(n, lo + W), w + step)
            ds.close_window()
            if w % 13 == 7:
                ds.close_window()                    # an empty interval
            if step == 1 and w >= nwin // 2:         # delta emission from mid-stream on (pass 2)
                v, l = ds.delta()
                mirror[v.astype(np.int64)] = l
                if w == nwin // 2:
                    pv, pl = ds.pairs()
                    mirror[:] = -1
                    mirror[pv.astype(np.int64)] = pl
                assert dense_checksum(mirror)[0] == int(want["checksums"][w]), "pass %d window %d (delta)" % (step, w)
            h, nv, nc = ds.checksum()
            assert h == int(want["checksums"][w]), "pass %d window %d" % (step, w)
        np.testing.assert_array_equal(ds.dense().astype(np.int64), want["final"])
        assert ds.stats() == (want["final_vertices"], want["final_components"])


def test_list_close_find_and_emission_between_windows(oracle, torch_cuda):
    """find/pairs/dense read between list-mode windows leave the next close exact."""
    torch = torch_cuda
    scale, n, W = 17, 1 << 20, 1 << 13
    cap = 1 << scale
    s, d = oracle.gen_rmat(0, n, scale, 21)
    want = oracle.run(s, d, W, partitions=4, threads=4, emit=EMIT_CHECKSUM, label_cap=cap)
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    ds = DisjointSet(cap, id_bits=32, stream=torch.cuda.current_stream())
    rng = np.random.default_rng(3)
    for w, lo in enumerate(range(0, n, W)):
        ds.fold(ts[lo:lo + W], td[lo:lo + W])
        if w % 9 == 4:
            q = rng.integers(0, cap, 64)
            ds.find_batch(q)
        ds.close_window()
        if w % 5 == 2:
            ds.pairs()
        assert ds.checksum()[0] == int(want["checksums"][w]), "window %d" % w


def test_handle_on_its_own_stream_reads_torch_inputs_in_order(oracle, torch_cuda):
    """A handle on its own stream (no stream= argument) folding device tensors that torch has just
    produced on its current stream: gsgpu waits for torch's stream first (summary.py _after_torch).
    Round 4's list-close diagnostic ran the test above without stream= and failed at a fold_pairs
    window (w % 11 == 5: the torch.stack had not finished when the library read it)."""
    torch = torch_cuda
    scale, n, W = 16, 1 << 19, 4096
    cap = 1 << scale
    s, d = oracle.gen_rmat(0, n, scale, 11)
    want = oracle.run(s, d, W, partitions=4, threads=4, emit=EMIT_CHECKSUM, label_cap=cap)
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    ds = DisjointSet(cap, id_bits=32)                # its own stream
    for w, lo in enumerate(range(0, n, W)):
        # produced on torch's stream right before the call (a larger torch op in front of it, so
        # that an unordered read would see a buffer still being written)
        junk = torch.empty(1 << 24, device="cuda").uniform_()
        pairs = torch.stack([ts[lo:lo + W], td[lo:lo + W]], dim=1).contiguous().view(-1)
        ds.fold_pairs(pairs)
        ds.close_window()
        del junk
        assert ds.checksum()[0] == int(want["checksums"][w]), "window %d" % w


def test_handle_on_the_null_stream_reads_a_torch_side_stream_in_order(oracle, torch_cuda):
    """The handle on the HIP null stream (set_stream(0)), the inputs produced on a torch side stream:
    torch's pool streams are non-blocking, so the null stream is not ordered with them — gsgpu makes
    the null stream wait for torch's current stream like any other (summary.py _as_torch_stream)."""
    torch = torch_cuda
    scale, n, W = 16, 1 << 18, 4096
    cap = 1 << scale
    s, d = oracle.gen_rmat(0, n, scale, 12)
    want = oracle.run(s, d, W, partitions=4, threads=4, emit=EMIT_CHECKSUM, label_cap=cap)
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    ds = DisjointSet(cap, id_bits=32)
    ds.set_stream(0)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for w, lo in enumerate(range(0, n, W)):
            junk = torch.empty(1 << 24, device="cuda").uniform_()
            pairs = torch.stack([ts[lo:lo + W], td[lo:lo + W]], dim=1).contiguous().view(-1)
            ds.fold_pairs(pairs)
            ds.close_window()
            del junk
            assert ds.checksum()[0] == int(want["checksums"][w]), "window %d" % w
    torch.cuda.synchronize()
    ds.close()


@pytest.mark.parametrize("W", [4096, 1 << 15])
def test_giant_root_changes_every_window(oracle, torch_cuda, W):
    """The giant's root (its minimum id) drops in every window: a smaller id joins it each time, so
    every close is a full pass over a giant whose gbits were built for its previous root — the
    rename shortcut (cc_kernels.hpp k_compress s_ren: members labelled with the new root without a
    walk), in both close kernels (list-mode windows and bitmap windows) — window by window vs the
    oracle, with claimed first touches (cbits) and stragglers outside the giant in the mix."""
    torch = torch_cuda
    scale = 17
    cap = 1 << scale
    rng = np.random.default_rng(9)
    hi0 = cap // 2
    nwin = 40
    src, dst = [], []
    for w in range(nwin):
        a = rng.integers(hi0, cap, W)
        b = rng.integers(hi0, cap, W)
        if w >= 2:                                   # a smaller id joins the giant: its root changes
            a[:4] = hi0 - 1 - 64 * w
            b[:4] = rng.integers(hi0, cap, 4)
            a[4:8] = rng.integers(0, hi0 // 2, 4)    # and a few stragglers outside it
            b[4:8] = rng.integers(0, hi0 // 2, 4)
        p = rng.permutation(W)
        src.append(a[p]); dst.append(b[p])
    s = np.concatenate(src).astype(np.int64)
    d = np.concatenate(dst).astype(np.int64)
    want = oracle.run(s, d, W, partitions=2, threads=2, emit=EMIT_CHECKSUM, label_cap=cap, want_final=True)
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    ds = DisjointSet(cap, id_bits=32, stream=torch.cuda.current_stream())
    for w, lo in enumerate(range(0, s.size, W)):
        ds.fold(ts[lo:lo + W], td[lo:lo + W])
        ds.close_window()
        assert ds.checksum()[0] == int(want["checksums"][w]), "window %d" % w
    np.testing.assert_array_equal(ds.dense().astype(np.int64), want["final"])
    ds.reset()                                       # the same through gs_cc_fold_windows
    assert ds.fold_windows(ts, td, W) == nwin
    assert ds.checksum()[0] == int(want["checksums"][-1])
