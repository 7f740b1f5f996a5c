"""bench_rows.py — measurement lines of SURVEY.md §8(f)'s next rows, run through bench.py:

  --workload parse   edge-file ingestion (§8(f) row 3, gs_parse_edges, csrc/parse.hip): the text
                     of an RMAT edge stream ("src dst\\n" lines, ConnectedComponentsExample.java:
                     108-119) resident in HBM, parsed into int64 (src, dst) device arrays.
  --workload parse_file  streaming ingestion end to end (gs_cc_fold_text): config 2's stream as text in
                     pinned host memory -> chunked H2D -> device parse -> folds + closes per window.
  --workload bip     BipartitenessCheck (§8(f) row 4, gs_bip_*, csrc/bip.hip): a bipartite
                     stream (RMAT endpoints a, b -> 2a, 2b + 1) folded window by window, each
                     window closed (the Merger's emission), like the connected-components step.

Each prints bench.py's one JSON line (value, roofline of the whole call / step, cpu_baseline of
the oracle restatement on the host, a verification of the outputs). The oracle (oracle/) is used
only as the checker and as cpu_baseline.
"""
from __future__ import annotations

import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))

HBM_PEAK_GBS = 8000.0


def edge_text(src, dst):
    """The text of a stream on the device: one "src dst\\n" line per edge (ids >= 0, decimal)."""
    import torch
    s = src.to(torch.int64)
    d = dst.to(torch.int64)

    def ndig(x):
        n = torch.ones_like(x)
        for k in range(1, 19):
            n += (x >= 10 ** k).to(x.dtype)
        return n
    ls, ld = ndig(s), ndig(d)
    ll = ls + ld + 2
    end = torch.cumsum(ll, 0)
    off = end - ll
    out = torch.empty(int(end[-1].item()), dtype=torch.uint8, device=src.device)
    for x, lx, base in ((s, ls, off), (d, ld, off + ls + 1)):
        p = 1
        for k in range(int(lx.max().item())):
            m = k < lx
            out[(base + lx - 1 - k)[m]] = ((x[m] // p) % 10 + 48).to(torch.uint8)
            p *= 10
    out[off + ls] = 32
    out[end - 1] = 10
    return out


def _line(a, metric, value, unit, ms, workload, extra):
    line = {"metric": metric, "value": value, "unit": unit, "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "data": "synthetic"}
    line.update(extra)
    line["config"] = workload
    return line


def run_parse(a, out):
    import torch
    import gsgpu  # noqa: F401  (loads libgsgpu after torch)
    from gsgpu import gen
    from gsgpu._abi import call
    scale = a.scale
    n = a.edge_factor << a.scale
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.empty(n, dtype=torch.int32, device=dev)
    d = torch.empty(n, dtype=torch.int32, device=dev)
    gen.rmat(s, d, 0, scale, a.seed)
    text = edge_text(s, d)
    nbytes = int(text.numel())
    ps = torch.empty(n, dtype=torch.int64, device=dev)
    pd = torch.empty(n, dtype=torch.int64, device=dev)
    got = ctypes.c_uint64()
    stream = torch.cuda.current_stream().cuda_stream

    def one():
        call("gs_parse_edges", ctypes.c_void_p(text.data_ptr()), nbytes, 64, ctypes.c_void_p(ps.data_ptr()),
             ctypes.c_void_p(pd.data_ptr()), n, ctypes.byref(got), 0, ctypes.c_void_p(stream))
    for _ in range(a.warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.steps
    ok = int(got.value) == n and bool(torch.equal(ps, s.to(torch.int64))) and bool(torch.equal(pd, d.to(torch.int64)))
    alg = nbytes + 16 * n                                  # text read once + int64 (src, dst) written
    achieved = alg / (ms * 1e-3) / 1e9
    extra = {"dtype": "u8 text -> int64",
             "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                          "definition": "algorithmic bytes per call (the text read once + 16 B of int64 ids "
                                        "written per line) / the whole gs_parse_edges call's wall time (device "
                                        "text and outputs; the call's scratch allocations and its one host "
                                        "sync for the line count included); kernels in profiles/r04_rows_*"},
             "text_bytes": nbytes, "text_GBps": nbytes / (ms * 1e-3) / 1e9,
             "verify": {"lines": int(got.value), "equal_to_generated_ids": ok}}
    if not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from pyoracle import coracle
        host = text.cpu().numpy().tobytes()
        r_s, r_d, secs = coracle().parse_edges(host)
        same = r_d is not None and len(r_s) == n
        extra["cpu_baseline"] = {"value": n / secs, "unit": "edges/s", "cores": 1, "kind": "port",
                                 "sample": "the whole text (%d lines, %d bytes) parsed by oracle/parse.c on one host "
                                           "thread (%.2f s); lines parsed %s" % (n, nbytes, secs, "equal" if same else "DIFFER")}
    print(_json(_line(a, "edge-file ingestion edges/sec (gs_parse_edges, text resident in HBM)", n / (ms * 1e-3),
                      "edges/s", ms, {"workload": "parse_rmat%d_%dedges" % (scale, n), "id_bits": 64,
                                      "text": "one 'src dst\\n' line per edge, decimal"}, extra)), file=out, flush=True)


def run_parse_file(a, out):
    """Streaming edge-file ingestion end to end (gs_cc_fold_text): the text of
    BASELINE config 2's stream (RMAT-20 EF16, 2^24 "src dst\\n" lines) in PINNED host memory, moved
    in 64 MiB chunks over PCIe through the double-buffered staging, parsed on the device into the
    edge ring and folded straight from it in 2^20-edge windows, every window closed (the Merger's
    canonical emission, resident in HBM). PCIe-inclusive: the text starts on the host."""
    import torch
    import gsgpu
    from gsgpu import gen
    scale, ef, wl = a.scale, a.edge_factor, a.window_log2
    n, W = ef << scale, 1 << wl
    V = 1 << scale
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.empty(n, dtype=torch.int32, device=dev)
    d = torch.empty(n, dtype=torch.int32, device=dev)
    gen.rmat(s, d, 0, scale, a.seed)
    text_dev = edge_text(s, d)
    nbytes = int(text_dev.numel())
    text = text_dev.cpu().pin_memory()
    del text_dev
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    ds = gsgpu.DisjointSet(V, id_bits=32, stream=st)
    res = {}

    def step():
        ds.reset()
        res["ew"] = ds.fold_text(text, W)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.steps
    final = ds.checksum()
    # the PCIe ceiling of this path: one pinned -> device copy of the whole text
    dbuf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(3):
        dbuf.copy_(text, non_blocking=True)
    torch.cuda.synchronize()
    h2d_gbs = 3 * nbytes / (time.perf_counter() - t1) / 1e9
    del dbuf
    achieved = nbytes / (ms * 1e-3) / 1e9
    extra = {"dtype": "u8 text -> int32 ids",
             "roofline": {"bound": "pcie", "achieved": achieved, "peak": h2d_gbs, "unit": "GB/s",
                          "frac": achieved / h2d_gbs, "traffic": None,
                          "hbm_frac": (nbytes + 16 * n) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                          "definition": "text bytes per step / the whole gs_cc_fold_text call's wall time, against "
                                        "the measured pinned host -> device copy rate of the same text (one "
                                        "hipMemcpy, 'peak'); hbm_frac: the text + 16 B per edge over the step / 8 TB/s"},
             "text_bytes": nbytes,
             "verify": {"edges": res["ew"][0], "windows": res["ew"][1], "final_checksum": str(final[0]),
                        "final_vertices": final[1], "final_components": final[2]}}
    if not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from pyoracle import EMIT_FLATTEN, coracle
        o = coracle()
        host = text.numpy().tobytes()
        r_s, r_d, psecs = o.parse_edges(host)
        cores = os.cpu_count() or 1
        r = o.run(r_s, r_d, W, partitions=cores, threads=cores, emit=EMIT_FLATTEN, label_cap=V, want_final=True)
        secs = psecs + r["seconds"]
        ok = (r["final_vertices"], r["final_components"]) == (final[1], final[2])
        extra["verify"]["oracle_counts_equal"] = bool(ok)
        extra["cpu_baseline"] = {"value": n / secs, "unit": "edges/s", "cores": cores, "kind": "port",
                                 "sample": "the whole text: oracle/parse.c (one thread, %.2f s) then the C pipeline "
                                           "(P=%d partitions on %d threads, %d-edge windows, FlattenSet emission per "
                                           "window, %.2f s)" % (psecs, cores, cores, W, r["seconds"])}
    print(_json(_line(a, "streaming edge-file ingestion + CC edges/sec (gs_cc_fold_text, text in pinned host memory, "
                         "PCIe-inclusive)", n / (ms * 1e-3), "edges/s", ms,
                      {"workload": "parse_file_rmat%d_ef%d_window%d" % (scale, ef, W), "id_bits": 32,
                       "text": "one 'src dst\\n' line per edge, decimal, pinned host memory",
                       "chunk_bytes": 64 << 20, "windows": (n + W - 1) // W}, extra)), file=out, flush=True)


def run_bip(a, out):
    import torch
    import gsgpu
    from gsgpu import gen
    from gsgpu.bipartite import Candidates
    scale, ef, wl = a.scale, a.edge_factor, a.window_log2
    E, W = ef << scale, 1 << wl
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.empty(E, dtype=torch.int32, device=dev)
    d = torch.empty(E, dtype=torch.int32, device=dev)
    gen.rmat(s, d, 0, scale, a.seed)
    s.mul_(2)
    d.mul_(2).add_(1)                                      # bipartite: even ids on one side, odd on the other
    torch.cuda.synchronize()
    cap = 2 << scale
    st = torch.cuda.current_stream()
    c = Candidates(cap, id_bits=32, stream=st)

    def step():
        c.reset()
        for lo in range(0, E, W):
            c.fold(s[lo:lo + W], d[lo:lo + W])
            c.close_window()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.steps
    ok_b, nv, nc = c.status()
    ds = gsgpu.DisjointSet(cap, id_bits=32, stream=st)     # the same graph's components (check)
    ds.fold(s, d)
    ds.close_window()
    cv, cc = ds.stats()
    alg = 16 * E                                           # 8 B edge read + 2 x 4 B summary words per edge
    achieved = alg / (ms * 1e-3) / 1e9
    extra = {"dtype": "int32",
             "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                          "definition": "16 B per edge (edge read + 2 summary words, as SURVEY.md 8(d) for CC) x "
                                        "the stream's edges / the whole step's wall time (reset, every window's "
                                        "fold and close)"},
             "verify": {"bipartite": bool(ok_b), "vertices": nv, "components": nc,
                        "equal_to_cc_counts": (nv, nc) == (cv, cc)}}
    if not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from bipartite import literal_run
        from pyoracle import coracle
        cores = os.cpu_count() or 1
        m = min(E, 16 * W)                                 # the first 16 windows
        b_ok, b_nv, b_nc, secs = coracle().bip_run(s[:m].cpu().numpy(), d[:m].cpu().numpy(), W, partitions=cores,
                                                   threads=cores)
        extra["cpu_baseline"] = {"value": m / secs, "unit": "edges/s", "cores": cores, "kind": "port",
                                 "sample": "the first %d windows (%d edges) of the same stream through oracle/bipartite.c "
                                           "(the semantics the reference's tests pin, in the reference's dataflow: a "
                                           "parity union-find per partition per window, P=%d partitions on %d threads, "
                                           "combine in partition order, the Merger; %.2f s); bipartite %s"
                                           % (m // W, m, cores, cores, secs, b_ok)}
        # the reference's literal Candidates.merge (TreeMap scans per edge, quadratic): pure Python on a
        # small prefix; NOT a baseline, reported for scale only
        ml, wl = 1 << 13, 1 << 11
        t1 = time.perf_counter()
        literal_run(s[:ml].cpu().tolist(), d[:ml].cpu().tolist(), wl)
        extra["literal_reference_python"] = {"edges_per_s": ml / (time.perf_counter() - t1), "edges": ml,
                                             "note": "oracle/bipartite.py literal_run, one thread; not a baseline"}
    print(_json(_line(a, "BipartitenessCheck edges/sec (gs_bip_*, windowed, stream in HBM)", E / (ms * 1e-3),
                      "edges/s", ms, {"workload": "bip_rmat%d_ef%d_window%d" % (scale, ef, W),
                                      "stream": "RMAT endpoints a, b -> (2a, 2b+1)", "windows": E // W}, extra)),
          file=out, flush=True)


def _json(x):
    import json
    return json.dumps(x)
