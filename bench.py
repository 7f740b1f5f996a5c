"""bench.py — streaming Connected Components edges/s on MI355X (+ % of the HBM roofline).

Workload (BASELINE.json metric "streaming CC edges/sec (RMAT-26) at 1/2/4/8 MI355X", configs[2]):
  RMAT scale 26 (Graph500 a,b,c,d = .57,.19,.19,.05, ids scrambled), edge factor 16: ONE stream of
  2^30 edges (seed 1) in 64 global windows of 2^24 edges; after each window the partial summaries
  are merged (CombineCC) and the window is closed (full compression = the canonical per-window
  emission, resident in HBM). Inputs are generated in HBM by the counter-based generator before the
  timed region.
  --scaling strong (default): the stream is fixed; rank r of P folds slice r of every global window
      (2^24 / P edges: the PartitionMapper split of each window, SummaryBulkAggregation.java:76-80,
      93-106), so each GPU holds E/P edges.
  --scaling weak: every rank folds 2^30 edges; global window = P x 2^24 edges of a P x 2^30 stream.
  N > 1: the exchange runs under the C ABI (gs_cc_merge_window over RCCL, csrc/comm.hip) with
  --dist-backend nccl; --dist-backend gloo runs the Python exchange (tests/gloo_tree.py) over host
  staging, for several ranks on one GPU.
One step = one whole pass over the stream from an empty summary (reset included).

Other lines (not the headline): --workload c2 | c4 | c5 | c3_single (the whole stream as one
window), --id-bits 64 (the reference's Long ids), --host-input (edges in pinned host memory: the
PCIe-inclusive rate of gs_cc_fold's staged path); --workload parse | bip: SURVEY.md 8(f)'s
edge-file ingestion and BipartitenessCheck (bench_rows.py).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N>1 under torch.distributed.run.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gelly-streaming_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import gsgpu  # noqa: E402
from gsgpu import gen  # noqa: E402
from gsgpu._abi import (GS_K_COMPRESS, GS_K_EXPORT, GS_K_FOLD, GS_K_MERGE, GS_K_RING,  # noqa: E402
                        GS_TIMING_MASK, LIB_PATH, lib_source_sha)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "streaming CC edges/sec (RMAT-26) at 1/2/4/8 MI355X + % of HBM roofline"
# SURVEY.md §8(d) / BASELINE.md: per edge 8 B edge read + 2 x 4 B parent reads (int32 ids; x2 for
# int64), per window 4 B (8 B) canonical label write per seen vertex
WORKLOADS = {  # name: (generator, scale or n, edge factor, window log2, seed)
    "c3": ("rmat", 26, 16, 24, 1), "c3_single": ("rmat", 26, 16, 30, 1),
    "c2": ("rmat", 20, 16, 20, 1), "c4": ("er", 24, 1, 20, 2), "c5": ("rmat", 24, 16, 16, 3),
    # SURVEY.md 8(f) rows (bench_rows.py): edge-file ingestion of 2^24 lines; BipartitenessCheck
    "parse": ("parse", 24, 1, 24, 1), "bip": ("bip", 22, 16, 20, 1),
    "parse_file": ("parse_file", 20, 16, 20, 1),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS),
                    help="c3 (default, the headline): RMAT-26 EF16, 2^24-edge windows; c3_single: the same "
                         "stream as one window; c2: RMAT-20 EF16, 2^20-edge windows; c4: Erdos-Renyi n=m=2^24, "
                         "2^20-edge windows; c5: RMAT-24 EF16, 2^16-edge windows + per-window emission latency; "
                         "parse: edge-file ingestion (gs_parse_edges) of an RMAT-24 stream's text, 2^24 lines; "
                         "bip: BipartitenessCheck (gs_bip_*) on a bipartite RMAT-22 EF16 stream, 2^20-edge windows; "
                         "parse_file: config 2's stream as text in pinned host memory streamed through gs_cc_fold_text "
                         "(chunked H2D, device parse, folds + closes per window; PCIe-inclusive)")
    ap.add_argument("--scale", type=int, default=None, help="override the workload's RMAT scale")
    ap.add_argument("--edge-factor", type=int, default=None)
    ap.add_argument("--window-log2", type=int, default=None, help="global window = 2^this edges")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    ap.add_argument("--id-bits", type=int, default=32, choices=[32, 64])
    ap.add_argument("--host-input", action="store_true",
                    help="edges in pinned host memory, folded through gs_cc_fold's staged H2D path")
    ap.add_argument("--emit-host", action="store_true",
                    help="per window, the emission's delta (gs_cc_emit_delta: pairs new or changed since the last "
                         "window) copied to pinned host memory, inside the timed region: what a host-side Merger / "
                         "FlattenSet consumer costs (SummaryAggregation.java:110-111); async by default "
                         "(gs_cc_emit_delta_async: the copy of window w overlaps the fold of window w+1)")
    ap.add_argument("--emit-sync", action="store_true",
                    help="with --emit-host: the blocking gs_cc_emit_delta per window instead")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true", help="check final labels with an independent torch CC "
                    "(multi-rank: rank 0 regenerates the whole global stream; small scales only)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = the C-ABI exchange over RCCL/xGMI (production); gloo = the Python exchange "
                         "over host staging (several ranks on one GPU, tests)")
    ap.add_argument("--exchange-world1", action="store_true",
                    help="one GPU through the C-ABI exchange (RCCL with one rank): the per-window cost of "
                         "export + collective + delta fold + close that a multi-GPU window adds (a measurement line)")
    ap.add_argument("--host-loop", action="store_true",
                    help="drive the windows from Python (fold + close / merge per window) instead of one "
                         "gs_cc_fold_windows call per step (an A/B of the host loop)")
    ap.add_argument("--merge", default=None, choices=["allgather", "gather", "tree", "prefilter"],
                    help="multi-rank CombineCC: allgather = replicated global summary (every rank folds every "
                         "delta); gather = windowAll gather to rank 0 (SummaryBulkAggregation.java:81); tree = "
                         "log2(P) pairwise rounds (SummaryTreeReduce.java:95-123); prefilter = ranks 1..P-1 "
                         "filter their slices against rank 0's broadcast giant bitmap and send the survivors, "
                         "rank 0 (the Merger) folds and emits (C ABI / RCCL only). Default: prefilter over "
                         "RCCL at P > 1 (the one-GPU rank model's best: DESIGN.md section 6), else allgather")
    ap.add_argument("--share0", type=float, default=None,
                    help="prefilter, strong layout: rank 0's share of every global window (default "
                         "(1 + 1/8) / P - 1/8 below P = 4 (P=2 0.44), 0 from P = 4 on: rank 0 then only "
                         "merges); the other ranks split the rest evenly")
    ap.add_argument("--no-fold-timing", action="store_true",
                    help="no HIP events on the timed region's fold launches (value only; the roofline "
                         "figures are then omitted)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "fold_traffic.json"),
                    help="PMC-derived HBM bytes per k_fold_ring launch (profiles/pmc_traffic.py)")
    a = ap.parse_args()
    kind, scale, ef, wl, seed = WORKLOADS[a.workload]
    a.kind = kind
    a.scale = scale if a.scale is None else a.scale
    a.edge_factor = ef if a.edge_factor is None else a.edge_factor
    a.window_log2 = wl if a.window_log2 is None else a.window_log2
    a.seed = seed if a.seed is None else a.seed
    return a


def prefilter_share0(world: int) -> float:
    """Rank 0's default share of a window under --merge prefilter: its per-window work beyond its
    own slice (the survivors' fold, the close, the launch gaps) costs about as much as filtering 1/8
    of a window (tools/sim_ranks.py prefilter, profiles/r05_prefilter_sim_*), so the slices balance
    at W1 = (1 + 1/8) W / P for the filtering ranks and W0 = W1 - W / 8 for rank 0. From P = 4 on rank
    0 folds no slice of its own (the filtering ranks take the whole window, layout()): with the
    senders filtering while rank 0 folds the previous window (round 6), rank 0's own fold of a small
    slice is mostly launch and latency (~38 us per 2^20 edges against the senders' ~14 us), and the
    round-6 rank model at P = 4 gives 1.79x with no slice, 1.70 / 1.66 / 1.57x with 5 / 10 / 15.6 %
    (profiles/r06_g_sim_p4_*.txt); at P = 2 the formula's 0.44 stays best (1.22x vs 1.16x at 0.35)."""
    if world >= 4:
        return 0.0
    s = max(0.0, (1.0 + 0.125) / world - 0.125)
    return s if s >= 1.0 / 32 else 0.0


def layout(a, world: int, rank: int):
    """(edges this rank folds, its slice per window, global window, windows, global stream edges,
    the slice's offset inside a global window)."""
    E = a.edge_factor << a.scale
    if a.scaling == "strong":
        W_glob = min(1 << a.window_log2, E)
        nwin = (E + W_glob - 1) // W_glob
        if E % W_glob:
            raise SystemExit("stream of %d edges is not a whole number of %d-edge windows" % (E, W_glob))
        if a.merge == "prefilter" and world > 1:
            # the Merger (rank 0) takes share0 of each window, the filtering ranks the rest; slices
            # are multiples of 4 edges (16-B aligned SoA groups)
            share0 = a.share0 if a.share0 is not None else prefilter_share0(world)
            W1 = int(W_glob * (1 - share0) / (world - 1)) // 4 * 4
            W0 = W_glob - (world - 1) * W1
            sizes = [W0] + [W1] * (world - 1)
            if share0 == 0.0:
                # no slice on rank 0 (it still joins every window's exchange: the ranks agree on the
                # window count in gs_cc_fold_windows); the remainder (< 4 (P - 1) edges, a multiple
                # of 4) goes 4 edges at a time to the first filtering ranks
                sizes[0] = 0
                for r in range(W0 // 4):
                    sizes[1 + r % (world - 1)] += 4
            W_rank = sizes[rank]
            off = sum(sizes[:rank])
            return nwin * W_rank, W_rank, W_glob, nwin, E, off
        if W_glob % world:
            raise SystemExit("global window %d does not split over %d ranks" % (W_glob, world))
        W_rank = W_glob // world
        return nwin * W_rank, W_rank, W_glob, nwin, E, rank * W_rank
    W_rank = min(1 << a.window_log2, E)
    nwin = (E + W_rank - 1) // W_rank
    return E, W_rank, W_rank * world, nwin, E * world, rank * W_rank


def main():
    a = parse()
    # stdout carries exactly the one JSON line: native libraries print banners there (RCCL's version
    # block at communicator init), so fd 1 is pointed at stderr for the run and the line goes to a
    # duplicate of the original stdout
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w", buffering=1)
    os.dup2(2, 1)
    if a.kind in ("parse", "bip", "parse_file"):  # SURVEY.md 8(f) rows, one GPU
        import bench_rows
        {"parse": bench_rows.run_parse, "bip": bench_rows.run_bip, "parse_file": bench_rows.run_parse_file}[a.kind](a, out)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if a.merge is None:
        a.merge = "prefilter" if world > 1 and a.dist_backend == "nccl" else "allgather"
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)          # more ranks than GPUs only in the gloo test mode
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    if a.gpus != world and rank == 0:
        print("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (a.gpus, world), file=sys.stderr)

    V = (1 << a.scale) if a.kind == "rmat" else (1 << a.scale)
    E_rank, W_rank, W_glob, nwin, E_glob, off_rank = layout(a, world, rank)
    if a.merge == "prefilter" and world > 1 and a.dist_backend != "nccl":
        raise SystemExit("--merge prefilter runs over the C ABI (RCCL) only")
    idt = torch.int32 if a.id_bits == 32 else torch.int64

    # ---- inputs resident in HBM (or pinned host memory) before timing ----
    src = torch.empty(E_rank, dtype=idt, device=dev)
    dst = torch.empty(E_rank, dtype=idt, device=dev)
    for w in range(nwin if W_rank else 0):
        lo, first = w * W_rank, w * W_glob + off_rank
        if a.kind == "er":
            gen.erdos_renyi(src[lo:lo + W_rank], dst[lo:lo + W_rank], first, V, a.seed)
        else:
            gen.rmat(src[lo:lo + W_rank], dst[lo:lo + W_rank], first, a.scale, a.seed)
    torch.cuda.synchronize()
    if a.host_input:
        hsrc, hdst = src.cpu().pin_memory(), dst.cpu().pin_memory()
        fsrc, fdst = hsrc, hdst
    else:
        fsrc, fdst = src, dst

    stream = torch.cuda.current_stream()
    marks = ((world > 1 and (a.merge == "allgather" or a.dist_backend == "nccl" or rank != 0)) or a.exchange_world1) \
        and a.merge != "prefilter"                   # the pre-filter exports no deltas
    ds = gsgpu.DisjointSet(V, id_bits=a.id_bits, device=local, track_marks=marks, stream=stream)
    comm = tree = None
    if world > 1 and a.dist_backend == "nccl":
        comm = gsgpu.Comm.from_process_group(local)                  # C ABI: gs_comm_create (RCCL)
    elif a.exchange_world1:
        from gsgpu.comm import unique_id
        comm = gsgpu.Comm.create(unique_id(), 0, 1, local)
    elif world > 1:
        sys.path.insert(0, os.path.join(ROOT, "tests"))          # test mode: the Python exchange model
        from gloo_tree import AllgatherMerge, GatherMerge, TreeMerge
        cls = {"allgather": AllgatherMerge, "gather": GatherMerge, "tree": TreeMerge}[a.merge]
        tree = cls(ds, capacity_pairs=V, device=dev)
    gather = tree is not None and a.merge == "gather"
    emitted = [0, 0]                                  # delta pairs copied to the host, windows
    if a.emit_host:                                   # two pinned slots: window w's delta lands in w & 1
        hv = [torch.empty(V, dtype=idt).pin_memory() for _ in range(2)]
        hl = [torch.empty(V, dtype=idt).pin_memory() for _ in range(2)]

    def consume(done):
        for v, _ in done:
            emitted[0] += v.numel()
            emitted[1] += 1

    def window(w, after=None):
        lo = w * W_rank
        if gather:
            tree.before_fold()
        if comm is not None and a.merge == "prefilter":    # (the exchange takes the window's edges)
            ds.fold_windows(fsrc[lo:lo + W_rank], fdst[lo:lo + W_rank], max(W_rank, 1), comm=comm, mode="prefilter")
        else:
            ds.fold(fsrc[lo:lo + W_rank], fdst[lo:lo + W_rank])
        if comm is not None and a.merge == "prefilter":
            pass
        elif comm is not None:
            ds.merge_window(comm, a.merge)
        elif tree is not None:
            tree.merge_window()
        else:
            ds.close_window()
        if a.emit_host and a.emit_sync:
            consume([ds.delta(hv[0], hl[0])])
        elif a.emit_host:                             # enqueue w's delta, take w-1's
            ds.delta_async(hv[w & 1], hl[w & 1])
            consume(ds.emit_wait(1))

    fold_mask = GS_TIMING_MASK | (1 << GS_K_FOLD) | (1 << GS_K_RING) | \
        ((1 << GS_K_MERGE) | (1 << GS_K_EXPORT) if world > 1 else 0)

    # the plain per-window loop runs inside the library (gs_cc_fold_windows: one ABI call per step
    # instead of two per window); per-window host work (delta copies, the gloo model) keeps the loop
    batched = not a.emit_host and tree is None and not a.host_loop

    def step():
        ds.reset()
        if batched:
            n_all = nwin * W_rank
            ds.fold_windows(fsrc[:n_all], fdst[:n_all], max(W_rank, 1), comm=comm, mode=a.merge)
        else:
            for w in range(nwin):
                window(w)
            if a.emit_host:
                consume(ds.emit_wait(0))

    log = lambda m: print("[bench rank %d] %s" % (rank, m), file=sys.stderr, flush=True)
    log("inputs ready: %d edges/rank, %d windows of %d (global %d), %s scaling" % (E_rank, nwin, W_rank, W_glob, a.scaling))
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    log("warmup done")
    # timing events only on the kernels the JSON line reports from the timed region (each timed
    # launch costs ~3 us of dispatch); the close is timed afterwards, outside the timed region
    # HIP events ride on the fold launches of the LAST timed step only: events on every launch of
    # every step cost 0.37 ms per 17 ms step (profiles/r02_aq). Turning them on before that step
    # resolves nothing (no event is pending), so the host does not wait on the GPU there.
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        if i == a.steps - 1 and not a.no_fold_timing:
            ds.timing(fold_mask)
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the timed path's own result: the emission checksum of the last window of the last timed step
    # (rank 0 holds the whole stream's summary in every merge mode), compared with the C oracle's
    # fixture of the same stream where one exists (tests/golden/, minted in the build container)
    final_sum = ds.checksum() if rank == 0 else None
    young_ms, young_n = ds.kernel_time(GS_K_FOLD)
    ring_ms, ring_n = ds.kernel_time(GS_K_RING)
    young_e, ring_e = (ds.kernel_units(k) for k in (GS_K_FOLD, GS_K_RING))
    merge_ms, _ = ds.kernel_time(GS_K_MERGE)
    export_ms, _ = ds.kernel_time(GS_K_EXPORT)
    ds.timing(False)
    # one more (untimed) step: the close's kernel time
    ds.timing(GS_TIMING_MASK | (1 << GS_K_COMPRESS))
    ds.reset()
    for w in range(nwin):
        window(w)
    comp_ms, comp_n = ds.kernel_time(GS_K_COMPRESS)
    ds.timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if a.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    sender_filter = None
    if world > 1 and a.merge == "prefilter":
        # the filtering ranks' k_filter_out launches (timed as GS_K_RING on their handles): rank 0,
        # the Merger, folds only survivors, so the line's dominant kernel is theirs (slowest rank)
        try:                                          # (reporting only: never fail the run on it)
            mine = torch.tensor([ring_ms / ring_n if ring_n else 0.0, ring_e / ring_n if ring_n else 0.0,
                                 float(ring_n)], dtype=torch.float64, device=dev)
            allv = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(allv, mine)
            rows = [v.tolist() for v in allv[1:]]
            slow = max(rows, key=lambda x: x[0])
            sender_filter = {"avg_launch_ms": slow[0], "edges_per_launch": slow[1], "launches": int(slow[2])}
        except Exception as e:                        # noqa: BLE001
            print("[bench] sender filter timings not gathered: %r" % (e,), file=sys.stderr)

    latency = None
    if a.workload == "c5":                    # per-window emission latency: fold -> emission ready
        lat = []
        ds.reset()
        for w in range(nwin):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if world == 1 and not a.emit_host:       # one library call: fold + close (gs_cc_fold_windows)
                lo = w * W_rank
                ds.fold_windows(fsrc[lo:lo + W_rank], fdst[lo:lo + W_rank], W_rank)
            else:
                window(w)
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t1) * 1e6)
        lat.sort()
        latency = {"p50_us": lat[len(lat) // 2], "p99_us": lat[min(len(lat) - 1, int(len(lat) * 0.99))],
                   "max_us": lat[-1], "windows": len(lat)}

    verify = None
    if a.verify and rank == 0:
        if world == 1:
            verify = verify_labels(ds, src, dst, V)
        else:                                   # the union of every rank's slices
            gs = torch.empty(nwin * W_glob, dtype=idt, device=dev)
            gd = torch.empty(nwin * W_glob, dtype=idt, device=dev)
            if a.kind == "er":
                gen.erdos_renyi(gs, gd, 0, V, a.seed)
            else:
                gen.rmat(gs, gd, 0, a.scale, a.seed)
            verify = verify_labels(ds, gs, gd, V)

    if rank == 0:
        eb = 8 if a.id_bits == 32 else 16            # edge bytes; parent words are 4 B either way
        # bytes an edge's fold actually moves: the edge + 2 parent words (4 B whatever the id width:
        # parent[] stays uint32 for int64 ids); SURVEY §8(d)'s int64 figure doubles
        # every term (32 B) and is reported beside it as frac_survey_int64
        per_edge = eb + 8
        per_edge_survey = eb + 8 if a.id_bits == 32 else 2 * 16
        total_edges = a.steps * E_glob
        folds = nwin                                  # the timed launches: the last step's
        fold_win_ms = (young_ms + ring_ms) / max(folds, 1) or float("nan")
        # the dominant kernel: the steady fold k_fold_ring, bytes per launch from the edges each timed
        # launch actually folded (a long fold call is cut into launches of at most 2^24 edges)
        k_bytes = per_edge                            # algorithmic bytes per edge of the dominant kernel
        k_def = "edge read + 2 parent words, SURVEY.md 8(d); 4-B parent words for int64 ids too"
        if sender_filter and sender_filter["launches"]:
            kernel, avg_ms, n_l, e_l = ("k_filter_out (filtering ranks; slowest)", sender_filter["avg_launch_ms"],
                                        sender_filter["launches"], sender_filter["edges_per_launch"])
            # the filter never touches parent[]: its algorithmic bytes are the edge read (plus the
            # survivors it writes, a few % of a steady window: not counted) — not comparable with
            # k_fold_ring rows; PMC traffic stays the comparable figure
            k_bytes = eb
            k_def = "filter: edge read only (k_filter_out reads no parent word)"
        elif ring_n:
            kernel, avg_ms, n_l, e_l = "k_fold_ring", ring_ms / ring_n, ring_n, ring_e / ring_n
        else:                                        # no steady launches (small ids: plain k_fold)
            kernel, avg_ms, n_l, e_l = "k_fold (every window)", fold_win_ms, folds, W_rank
        if not avg_ms:                               # --no-fold-timing
            avg_ms = float("nan")
        alg_launch = k_bytes * e_l
        achieved = alg_launch / (avg_ms * 1e-3) / 1e9
        prof, prof_note = steady_profile(a, kernel, e_l)
        step_b = per_edge * E_glob                                  # SURVEY 8(d) edge term per step
        step_gbs = step_b * a.steps / elapsed / 1e9
        nv, nc = ds.stats()
        fx_path, fx_last = fixture_last(a, world)
        line = {
            "metric": METRIC,
            "value": total_edges / elapsed,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": "int32" if a.id_bits == 32 else "int64",
            "data": "synthetic: counter-based %s stream generated in HBM (seed %d), no dataset"
                    % ("Erdos-Renyi" if a.kind == "er" else "RMAT", a.seed),
            "config": {
                "workload": "%s_%s%d_ef%d_window%s%s%s" % (a.workload.split("_")[0], "er" if a.kind == "er" else "rmat",
                                                         a.scale, a.edge_factor, _pow2(W_glob),
                                                         ("_int64" if a.id_bits == 64 else "") +
                                                         ("_xchg1" if a.exchange_world1 else ""),
                                                         "_hostinput" if a.host_input else "") +
                            ("_emithost" + ("sync" if a.emit_sync else "") if a.emit_host else ""),
                "scale": a.scale, "vertices": V, "edge_factor": a.edge_factor,
                "edges_total": E_glob, "edges_per_gpu": E_rank, "window_edges": W_glob,
                "window_edges_per_gpu": W_rank, "windows": nwin, "id_bits": a.id_bits,
                "input": "pinned host memory (PCIe-inclusive)" if a.host_input else "HBM",
                "parallelism": "1 subtask per GPU x %d, %s" % (
                    world, ("%s merge, %s" % (a.merge, "C ABI over RCCL" if comm is not None else "torch.distributed gloo"))
                    if world > 1 else ("%s merge through the C-ABI exchange at world 1 (RCCL, one rank)" % a.merge
                                       if a.exchange_world1 else "no merge")),
                "emission": ("per window, canonical min-id labels resident in HBM, and the delta (pairs new or changed "
                             "since the last window) copied to pinned host memory (%s)" % ("gs_cc_emit_delta" if a.emit_sync else
                             "gs_cc_emit_delta_async, waited one window later")) if a.emit_host
                            else "per window, canonical min-id labels resident in HBM",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": prof.get("hbm_bytes_per_launch") if prof else None,
                "frac_survey_int64": (per_edge_survey * e_l / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS)
                if a.id_bits == 64 else None,
                "traffic_source": prof_note,
                "kernel": kernel,
                "alg_bytes_per_launch": alg_launch,
                "edges_per_launch": e_l,
                "avg_launch_ms": avg_ms,
                "launches": n_l,
                "definition": "dominant kernel: %d B per edge (%s) x the edges each launch folded / its average "
                              "launch duration (HIP events on the launch stream, the last step of the timed region)"
                              % (k_bytes, k_def),
                "fold_all": {"achieved": per_edge * W_rank / (fold_win_ms * 1e-3) / 1e9,
                             "frac": per_edge * W_rank / (fold_win_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                             "ms_per_window": fold_win_ms, "young_launches": young_n,
                             "definition": "every UpdateCC launch of a window (young k_fold + steady k_fold_ring)"},
                "requests": request_roofline(prof, avg_ms) if prof else None,
                "step": {"achieved": step_gbs, "frac": step_gbs / (world * HBM_PEAK_GBS),
                         "alg_bytes_per_step": step_b,
                         "definition": "the whole timed step (every kernel, closes and exchange included): %d B per "
                                       "edge x the stream's edges / wall time / (P x 8 TB/s); no label-write term (the "
                                       "incremental close leaves giant members' labels resident and never rewrites "
                                       "them, so crediting 4 B per seen vertex per window would count bytes that are "
                                       "never moved)" % per_edge},
            },
            "kernels": {
                "fold_share": (young_ms + ring_ms) / (elapsed / a.steps * 1e3),   # timed: the last step's folds
                "compress_ms_per_window": comp_ms / max(comp_n, 1),
                "compress_share": comp_ms / (elapsed / a.steps * 1e3),
            },
            "library": os.path.relpath(LIB_PATH, ROOT),
            "final_vertices": nv,
            "final_components": nc,
            "final_checksum": str(final_sum[0]),
            "final_checksum_vs_fixture": None if fx_last is None else {
                "fixture": os.path.relpath(fx_path, ROOT), "match": tuple(final_sum) == fx_last,
                "definition": "emission checksum (sum of pair_mix(v, min-id label) over the cumulative summary), vertex "
                              "and component counts of the last window of the last timed step vs the C oracle's "
                              "fixture for that window"},
        }
        if world > 1:                                # rank 0's side of the exchange
            overflows = None
            if comm is not None:
                _, _, sent, recv, nex, overflows = comm.info()
            else:
                sent, recv, nex = tree.bytes_sent, tree.bytes_recv, (a.warmup + a.steps + 1) * nwin
            line["exchange"] = {
                "merge": a.merge, "transport": "RCCL (C ABI)" if comm is not None else "gloo (Python)",
                "merge_fold_ms_per_window": merge_ms / max(folds, 1),
                "export_ms_per_window": export_ms / max(folds, 1),
                "bytes_sent_per_window": sent / max(nex, 1),
                "bytes_recv_per_window": recv / max(nex, 1),
                "wall_ms_per_window": elapsed / a.steps / nwin * 1e3,
                "slot_overflows": overflows,
            }
        if a.emit_host and emitted[1]:
            per = emitted[0] / emitted[1]
            line["emit_host"] = {"delta_pairs_per_window": per,
                                 "delta_bytes_per_window": per * 2 * (4 if a.id_bits == 32 else 8),
                                 "windows": emitted[1]}
        if verify is not None:
            line["verify"] = verify
        if latency is not None:
            line["window_latency"] = latency
        if not a.no_cpu_baseline and world == 1:
            log("timed region done (%.1f ms/step); cpu baseline..." % (elapsed / a.steps * 1e3))
            line["cpu_baseline"] = cpu_baseline(a, ds, window, src, dst, W_rank, nwin)
        print(json.dumps(line), file=out, flush=True)
    if gather:
        tree.drain()
    ds.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


def fixture_last(a, world: int):
    """(path, (checksum, vertices, components) of the stream's last window) of the C oracle's fixture
    for this workload, or (None, None) where none was minted (tests/golden/make_headline.py,
    make_c5.py)."""
    fixtures = {("rmat", 26, 16, 24, 1): "headline_rmat26.json", ("rmat", 24, 16, 16, 3): "c5_rmat24.json"}
    name = fixtures.get((a.kind, a.scale, a.edge_factor, a.window_log2, a.seed))
    if name is None or (a.scaling == "weak" and world > 1):
        return None, None
    path = os.path.join(ROOT, "tests", "golden", name)
    if not os.path.exists(path):
        return None, None
    fx = json.load(open(path))
    return path, (int(fx["checksums"][-1]), int(fx["vertices"][-1]), int(fx["components"][-1]))


def _pow2(x: int) -> str:
    for suf, sh in (("G", 30), ("M", 20), ("K", 10)):
        if x >= (1 << sh) and x % (1 << sh) == 0:
            return "%d%s" % (x >> sh, suf)
    return str(x)


def steady_profile(a, kernel, edges_per_launch):
    """PMC counts of the dominant kernel from the committed profile (profiles/pmc_traffic.py), only
    if they were taken on this configuration AND on these kernel sources (the profile carries the
    lib_source_sha of the library it measured; any kernel change makes it stale and drops it)."""
    if not os.path.exists(a.traffic_json):
        return None, "no profile"
    try:
        tj = json.load(open(a.traffic_json))
    except Exception as e:
        return None, "unreadable profile: %r" % (e,)
    st = tj.get("steady") or {}
    sha = lib_source_sha()
    if tj.get("lib_source_sha") != sha:
        return None, "stale: profile of library %s, this library %s" % (tj.get("lib_source_sha"), sha)
    if (tj.get("scale"), tj.get("id_bits", 32), st.get("kernel")) != (a.scale, a.id_bits, kernel) or \
            abs(st.get("edges_per_launch", 0) - edges_per_launch) > 4:
        return None, "profile of another configuration"
    return st, "%s (PMC, library %s)" % (os.path.relpath(a.traffic_json, ROOT), sha)


def request_roofline(prof, avg_ms):
    """What bounds the steady fold besides bytes: memory requests. Per launch, the PMC passes give
    its TCC requests, their L2 hit rate and its HBM bytes; tools/request_lab.hip measured what this
    chip sustains: random 4-B loads over an L2-resident table (1 MiB: the request rate of the L2
    channels), over a table far larger than an L2 (64 MiB: the rate of requests that MISS the L2 and
    go to the fabric / Infinity Cache / HBM), and a streaming read. Bound = max(requests / L2 rate,
    L2 misses / miss rate, HBM bytes / stream rate): the three are served by different units and
    overlap. The miss term is the tight one for the ring fold (round 6): its ~9 M misses per launch
    are the gbits lines of cold ids (8 MiB bitmap against a 4 MiB L2 that also holds the 2 MiB warm
    set), the survivors' parent[] lines and the edge stream."""
    lab_path = os.path.join(ROOT, "profiles", "r03_request_lab.json")
    if not os.path.exists(lab_path):
        return None
    try:
        lab = json.load(open(lab_path))
        req, hbm = prof["tcc_requests_per_launch"], prof["hbm_bytes_per_launch"]
        req_gps, stream_tbps = lab["rand4B_1MiB_32w_Gps"], lab["stream_read_TBps"]
        miss_gps = lab["rand4B_64MiB_32w_Gps"]
        hit = prof.get("l2_hit_rate")
        misses = req * (1.0 - hit) if hit is not None else None
        t_req = req / (req_gps * 1e3)                                     # us
        t_miss = misses / (miss_gps * 1e3) if misses is not None else 0.0
        t_bytes = hbm / (stream_tbps * 1e6)
        bound_us = max(t_req, t_miss, t_bytes)
        bound = "l2-misses" if bound_us == t_miss else ("l2-requests" if bound_us == t_req else "hbm-bytes")
        return {"bound": bound, "tcc_requests_per_launch": req, "l2_hit_rate": hit, "l2_misses_per_launch": misses,
                "hbm_bytes_per_launch": hbm, "request_peak_Gps": req_gps, "miss_peak_Gps": miss_gps,
                "stream_peak_TBps": stream_tbps, "requests_us": t_req, "misses_us": t_miss, "bytes_us": t_bytes,
                "bound_us": bound_us, "avg_launch_us": avg_ms * 1e3, "frac": bound_us / (avg_ms * 1e3),
                "frac_requests_only": t_req / (avg_ms * 1e3),
                "definition": "max(TCC requests / L2 random-request rate, L2 misses / random-miss rate, PMC HBM "
                              "bytes / streaming-read rate) per launch (counts: profiles/fold_traffic.json; rates: "
                              "tools/request_lab.hip, profiles/r03_request_lab.json: 1 MiB / 64 MiB random 4-B "
                              "loads, streaming read) / the launch's average duration"}
    except Exception:
        return None


def torch_min_labels(src, dst, V):
    """Independent min-label CC with torch ops (hook labels to the min, pointer-jump to the fixpoint)."""
    lab = torch.arange(V, dtype=torch.int64, device=src.device)
    s, d = src.long(), dst.long()
    while True:
        ls, ld = lab[s], lab[d]
        m = torch.minimum(ls, ld)
        new = lab.clone()
        new.scatter_reduce_(0, ls, m, reduce="amin")
        new.scatter_reduce_(0, ld, m, reduce="amin")
        while True:
            j = new[new]
            if torch.equal(j, new):
                break
            new = j
        if torch.equal(new, lab):
            break
        lab = new
    seen = torch.zeros(V, dtype=torch.bool, device=src.device)
    seen[s] = True
    seen[d] = True
    return torch.where(seen, lab, torch.full_like(lab, -1))


def verify_labels(ds, src, dst, V):
    lab = torch.empty(V, dtype=torch.int32 if ds.id_bits == 32 else torch.int64, device=src.device)
    ds.dense(out=lab)
    lab = lab.long()
    s, d = src.long(), dst.long()
    ok_edges = bool((lab[s] == lab[d]).all())
    seen = lab >= 0
    v = torch.arange(V, device=src.device)
    ok_min = bool((lab[seen] <= v[seen]).all()) and bool((lab[lab[seen]] == lab[seen]).all())
    ok_exact = bool(torch.equal(lab, torch_min_labels(src, dst, V)))
    return {"edges_consistent": ok_edges, "labels_minimal_idempotent": ok_min, "equals_torch_cc": ok_exact}


def cpu_baseline(a, ds, window, src, dst, W, nwin):
    """Reference-semantics CPU restatement (oracle/, C): hash-map DisjointSet per partition on P
    host threads (P = the host's core count), single-thread CombineCC + Merger,
    FlattenSet emission per window (SummaryBulkAggregation.java:76-83, SummaryAggregation.java:106-119,
    ConnectedComponentsExample.java:143-156). Sampled windows from the start, the middle and the end
    of the stream: the Merger's cumulative summary makes a window's cost depend on everything
    before it, so a span that starts at window s is run from the Merger restored (untimed, as
    restoreState would) from the canonical emission of window s-1, taken from the GPU run."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import EMIT_FLATTEN, coracle
    import numpy as np
    cores = os.cpu_count() or 1
    try:
        share = len(os.sched_getaffinity(0))
    except Exception:
        share = cores
    o = coracle()
    spans = sorted({(0, min(2, nwin)), (nwin // 2, 1), (nwin - 1, 1)})
    edges = 0
    secs = 0.0
    names = []
    for s0, ln in spans:
        if s0 + ln > nwin or s0 < 0:
            continue
        init = None
        if s0:
            ds.reset()
            for w in range(s0):
                window(w)
            init = ds.pairs()                      # the canonical emission of window s0-1 (host)
        lo, hi = s0 * W, (s0 + ln) * W
        r = o.run(src[lo:hi].cpu().numpy().astype(np.int64), dst[lo:hi].cpu().numpy().astype(np.int64), W,
                  partitions=cores, threads=cores, emit=EMIT_FLATTEN, init=init)
        edges += hi - lo
        secs += r["seconds"]
        names.append("%d-%d" % (s0 + 1, s0 + ln) if ln > 1 else "%d" % (s0 + 1))
    return {"value": edges / secs, "unit": "edges/s", "cores": cores, "kind": "port",
            "sample": "windows %s of %d (%d edges) of the same %s stream, window %d edges; a span starting at "
                      "window s runs from the Merger restored from window s-1's emission (untimed); P=%d "
                      "partitions on %d threads (nproc=%d, CPUs in this process's affinity=%d), FlattenSet "
                      "emission per window; %.1f s timed" % (", ".join(names), nwin, edges,
                                                              "RMAT-%d" % a.scale if a.kind == "rmat" else "ER",
                                                              W, cores, cores, os.cpu_count() or 1, share, secs)}


if __name__ == "__main__":
    main()
