"""GPU parity of the streaming edge-file ingestion (gs_cc_fold_text / gs_cc_fold_file; SURVEY.md
8(f) row 3, ConnectedComponentsExample.java:108-119 -> edges.aggregate(ConnectedComponents), :61).

The text is cut into chunks smaller than the stream (partial lines carried between chunks), copied
through pinned staging, parsed on the device into the edge ring and folded from it in count
windows. Every window's emission (checksum of the canonical pairs, read in the per-window callback)
is compared with the C oracle run on the Java parse of the same text (tests/test_gpu_parity.py
_java_parse = split("\\s") + Long.parseLong), for pageable, pinned and device text and for files,
int32 / int64 / sparse-id summaries, windows that span chunks and chunks that hold many windows,
the bad-line and long-line errors.
"""
import numpy as np
import pytest

from gsgpu import DisjointSet, GsError, _abi
from pyoracle import EMIT_CHECKSUM

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def _text(s, d, seed=0):
    """Edge lines with the separators / trailing forms the Java rules accept."""
    rng = np.random.default_rng(seed)
    seps = [b" ", b"\t"]
    tails = [b"", b"", b"", b" ", b"\r", b" x y"]
    out = []
    for i, (a, b) in enumerate(zip(s.tolist(), d.tolist())):
        out.append(b"%d%s%d%s\n" % (a, seps[i % 2], b, tails[int(rng.integers(0, len(tails)))]))
    return b"".join(out)


def _run(ds, fold, W):
    sums = []
    edges, wins = fold(lambda w: sums.append(ds.checksum()[0]))
    return edges, wins, sums


@pytest.mark.parametrize("W,chunk", [(4096, 1 << 16), (256, 1 << 16), (1 << 16, 1 << 15), (5000, 4099)])
@pytest.mark.parametrize("source", ["pageable", "pinned", "file"])
def test_fold_text_windows_vs_oracle(oracle, torch_cuda, tmp_path, source, W, chunk):
    torch = torch_cuda
    scale, n = 16, 200000
    s, d = oracle.gen_rmat(0, n, scale, 4)
    text = _text(s, d, 1)
    assert len(text) > 4 * chunk                     # several chunks, lines cut at their ends
    want = oracle.run(s, d, W, partitions=3, threads=3, emit=EMIT_CHECKSUM, label_cap=1 << scale, want_final=True)
    ds = DisjointSet(1 << scale, id_bits=32, stream=torch.cuda.current_stream())
    if source == "pageable":
        fold = lambda cb: ds.fold_text(text, W, chunk_bytes=chunk, on_window=cb)
    elif source == "pinned":
        t = torch.frombuffer(bytearray(text), dtype=torch.uint8).pin_memory()
        fold = lambda cb: ds.fold_text(t, W, chunk_bytes=chunk, on_window=cb)
    else:
        f = tmp_path / "edges.txt"
        f.write_bytes(text)
        from gsgpu.edgefile import fold_edge_file       # the example's file path (the streaming fold)
        fold = lambda cb: fold_edge_file(ds, str(f), W, chunk_bytes=chunk, on_window=cb)
    edges, wins, sums = _run(ds, fold, W)
    assert edges == n and wins == len(want["checksums"]) == len(sums)
    assert sums == [int(x) for x in want["checksums"]]
    np.testing.assert_array_equal(ds.dense().astype(np.int64), want["final"])
    # a second call continues the same summary (the ring and staging are reused)
    ds.reset()
    edges2, wins2 = fold(None)
    assert (edges2, wins2) == (edges, wins)
    assert ds.checksum()[0] == int(want["checksums"][-1])


def test_fold_text_device_text_int64_and_no_final_newline(oracle, torch_cuda):
    torch = torch_cuda
    scale, n, W = 17, 150000, 3000
    s, d = oracle.gen_rmat(0, n, scale, 9)
    text = _text(s, d, 2).rstrip(b"\n")               # a last line without '\n' still counts
    want = oracle.run(s, d, W, partitions=2, threads=2, emit=EMIT_CHECKSUM, label_cap=1 << scale, want_final=True)
    dt = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
    ds = DisjointSet(1 << scale, id_bits=64, stream=torch.cuda.current_stream())
    edges, wins, sums = _run(ds, lambda cb: ds.fold_text(dt, W, on_window=cb), W)
    assert edges == n and sums == [int(x) for x in want["checksums"]]
    np.testing.assert_array_equal(ds.dense().astype(np.int64), want["final"])


def test_fold_file_sparse_long_ids(oracle, torch_cuda, tmp_path):
    """Any Java long ids (negative, >= 2^32) through a sparse-id summary: the canonical pairs after
    every window vs the oracle's."""
    torch = torch_cuda
    rng = np.random.default_rng(5)
    base, n = 1 << 14, 60000
    ids = rng.choice(np.concatenate([rng.integers(-(1 << 62), 1 << 62, 4 * base), [-(1 << 63), (1 << 63) - 1]]),
                     base, replace=False).astype(np.int64)
    s0, d0 = oracle.gen_rmat(0, n, 14, 3)
    s, d = ids[s0], ids[d0]
    W = 7000
    want = oracle.run(s, d, W, partitions=2, threads=2, emit=EMIT_CHECKSUM)
    f = tmp_path / "long_edges.txt"
    f.write_bytes(_text(s, d, 3))
    ds = DisjointSet(base, id_bits=64, sparse=True, stream=torch.cuda.current_stream())
    edges, wins, sums = _run(ds, lambda cb: ds.fold_file(str(f), W, chunk_bytes=1 << 16, on_window=cb), W)
    assert edges == n and sums == [int(x) for x in want["checksums"]]


@pytest.mark.parametrize("where", ["first_chunk", "third_chunk", "last_line"])
def test_fold_text_bad_line_folds_everything_before_it(oracle, torch_cuda, where):
    torch = torch_cuda
    scale, n, W, chunk = 15, 50000, 1000, 1 << 14
    s, d = oracle.gen_rmat(0, n, scale, 6)
    lines = _text(s, d, 4).split(b"\n")[:-1]
    k = {"first_chunk": 100, "third_chunk": (3 * chunk) // 12, "last_line": n - 1}[where]
    lines[k] = b"12  34"                                 # two separators: an empty field 1 (rejected)
    text = b"\n".join(lines) + b"\n"
    ds = DisjointSet(1 << scale, id_bits=32, stream=torch.cuda.current_stream())
    with pytest.raises(GsError) as ei:
        ds.fold_text(text, W, chunk_bytes=chunk)
    assert ei.value.code == _abi.GS_ERR_INVALID and "line %d " % (k + 1) in str(ei.value)
    assert ei.value.edges == k and ei.value.windows == k // W
    ds.close_window()                                    # the open window's prefix was folded
    want = oracle.run(s[:k], d[:k], W, partitions=1, threads=1, emit=EMIT_CHECKSUM)
    assert ds.checksum()[0] == int(want["checksums"][-1])


@pytest.mark.parametrize("source", ["pageable", "file"])
def test_fold_text_long_line_after_whole_chunks(oracle, torch_cuda, tmp_path, source):
    """A line longer than a chunk, several chunks into the text: the next chunk cannot be staged,
    every chunk before it is still parsed and folded (the call used to return before
    folding the chunk already counted), the call fails with GS_ERR_CAPACITY and edges_out = the
    lines before the long one."""
    scale, n, W = 12, 3000, 500
    s, d = oracle.gen_rmat(0, n, scale, 6)
    text = _text(s, d, 2) + b"7 8" + b" " * 5000 + b"\n5 6\n"
    ds = DisjointSet(1 << scale, id_bits=32, stream=torch_cuda.cuda.current_stream())
    if source == "pageable":
        fold = lambda: ds.fold_text(text, W, chunk_bytes=4096)
    else:
        path = tmp_path / "long.txt"
        path.write_bytes(text)
        fold = lambda: ds.fold_file(str(path), W, chunk_bytes=4096)
    with pytest.raises(GsError) as ei:
        fold()
    assert ei.value.code == _abi.GS_ERR_CAPACITY
    assert ei.value.edges == n and ei.value.windows == n // W
    want = oracle.run(s, d, W, partitions=1, threads=1, emit=EMIT_CHECKSUM)
    assert ds.checksum()[0] == int(want["checksums"][-1])


def test_fold_text_line_longer_than_chunk(torch_cuda):
    ds = DisjointSet(1 << 10, id_bits=64, stream=torch_cuda.cuda.current_stream())
    text = b"1 2\n" + b"3 4" + b" " * 5000 + b"\n5 6\n"
    with pytest.raises(GsError) as ei:
        ds.fold_text(text, 10, chunk_bytes=4096)
    assert ei.value.code == _abi.GS_ERR_CAPACITY
