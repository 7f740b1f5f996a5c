"""bench.py — streaming Connected Components edges/s on MI355X (+ % of the HBM roofline).

Workload (BASELINE.json metric "streaming CC edges/sec (RMAT-26) at 1/2/4/8 MI355X"):
  RMAT scale 26 (Graph500 a,b,c,d = .57,.19,.19,.05, ids scrambled), edge factor 16 per GPU:
  every rank folds 2^30 edges of the counter-based stream (int32 ids, generated in HBM before the
  timed region) in 64 windows of 2^24 edges; after each window the partial summaries are merged
  (rank 0 = Merger: log2(P) pairwise tree over RCCL, gsgpu/tree.py) and rank 0 closes the window
  (full compression = the canonical per-window emission, resident in HBM).
  Weak scaling: at P GPUs the stream has P*2^30 edges over the same 2^26-vertex space; window w of
  the global stream is P*2^24 edges, rank r owns slice r of it.
One step = one whole pass over the stream from an empty summary (reset included).

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
from gsgpu._abi import GS_K_COMPRESS, GS_K_EXPORT, GS_K_FOLD, GS_K_MERGE, GS_TIMING_MASK  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "streaming CC edges/sec (RMAT-26) at 1/2/4/8 MI355X + % of HBM roofline"
BYTES_PER_EDGE_ALG = 16        # 8 B edge read + 2 x 4 B parent reads


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--window-log2", type=int, default=24)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--workload", default="c3", choices=["c3", "c2", "c4", "c5"],
                    help="c3 (default, the headline): RMAT-26 EF16 per GPU, 2^24-edge windows; "
                         "c2: RMAT-20 EF16, 2^20-edge windows; c4: Erdos-Renyi n=m=2^24, 2^20-edge windows; "
                         "c5: RMAT-24 EF16, 2^16-edge windows, per-window emission latency p50/p99")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-edges", type=int, default=1 << 25,
                    help="cpu_baseline sample: the first this-many edges (whole windows) of the same stream")
    ap.add_argument("--verify", action="store_true", help="check final labels with an independent torch CC "
                    "(multi-rank: rank 0 regenerates the whole global stream; small scales only)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (production); gloo = host-staged, for testing the "
                         "multi-rank path with several ranks on one GPU")
    ap.add_argument("--merge", default="allgather", choices=["allgather", "gather", "tree"],
                    help="multi-rank CombineCC: allgather = replicated global summary, all-pairs delta exchange "
                         "(fastest, tools/sim_ranks.py); gather = flat windowAll gather to rank 0 (ConnectedComponents, "
                         "SummaryBulkAggregation.java:81); tree = log2(P) pairwise rounds (ConnectedComponentsTree, "
                         "SummaryTreeReduce.java:95-123)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "fold_traffic.json"),
                    help="PMC-derived HBM bytes per fold launch (written by profiles/pmc_traffic.py)")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
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

    if a.workload != "c3":                     # BASELINE.json configs other than the headline
        a.scale, a.edge_factor, a.window_log2, a.seed = {
            "c2": (20, 16, 20, 1), "c4": (24, 1, 20, 2), "c5": (24, 16, 16, 3)}[a.workload]
    V = 1 << a.scale
    E_rank = a.edge_factor << a.scale
    W_rank = min(1 << a.window_log2, E_rank)
    nwin = (E_rank + W_rank - 1) // W_rank
    W_glob = W_rank * world

    # ---- inputs resident in HBM before timing ----
    src = torch.empty(E_rank, dtype=torch.int32, device=dev)
    dst = torch.empty(E_rank, dtype=torch.int32, device=dev)
    for w in range(nwin):
        lo = w * W_rank
        n = min(W_rank, E_rank - lo)
        if a.workload == "c4":
            gen.erdos_renyi(src[lo:lo + n], dst[lo:lo + n], w * W_glob + rank * W_rank, V, a.seed)
        else:
            gen.rmat(src[lo:lo + n], dst[lo:lo + n], w * W_glob + rank * W_rank, a.scale, a.seed)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    marks = world > 1 and (a.merge == "allgather" or rank != 0)
    ds = gsgpu.DisjointSet(V, id_bits=32, device=local, track_marks=marks, stream=stream)
    tree = None
    if world > 1:
        from gsgpu.tree import AllgatherMerge, GatherMerge, TreeMerge
        cls = {"allgather": AllgatherMerge, "gather": GatherMerge, "tree": TreeMerge}[a.merge]
        tree = cls(ds, capacity_pairs=V, device=dev)
    gather = world > 1 and a.merge == "gather"

    def step():
        ds.reset()
        for w in range(nwin):
            lo = w * W_rank
            if gather:
                tree.before_fold()
            ds.fold(src[lo:lo + W_rank], dst[lo:lo + W_rank])
            if tree is not None:
                tree.merge_window()
            else:
                ds.close_window()

    log = lambda m: print("[bench rank %d] %s" % (rank, m), file=sys.stderr, flush=True)
    log("inputs ready: %d edges/rank, %d windows of %d" % (E_rank, nwin, W_rank))
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    log("warmup done")
    # timing events only on the kernels the JSON line reports from the timed region (every timed
    # launch costs ~3 us of dispatch: all kernels timed = +0.7 ms per 64-window step, the fold
    # alone +0.3 ms); the close is timed afterwards, outside the timed region
    ds.timing(GS_TIMING_MASK | (1 << GS_K_FOLD) | ((1 << GS_K_MERGE) | (1 << GS_K_EXPORT) if world > 1 else 0))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    fold_ms, fold_n = ds.kernel_time(GS_K_FOLD)
    merge_ms, _ = ds.kernel_time(GS_K_MERGE)
    export_ms, _ = ds.kernel_time(GS_K_EXPORT)
    ds.timing(False)
    # the close's kernels, timed over one more (untimed-region) step
    ds.timing(GS_TIMING_MASK | (1 << GS_K_COMPRESS))
    step()
    torch.cuda.synchronize()
    comp_ms, comp_n = ds.kernel_time(GS_K_COMPRESS)        # one step
    ds.timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    latency = None
    if a.workload == "c5":                    # per-window emission latency: fold -> emission ready
        lat = []
        ds.reset()
        for w in range(nwin):
            lo = w * W_rank
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if gather:
                tree.before_fold()
            ds.fold(src[lo:lo + W_rank], dst[lo:lo + W_rank])
            if tree is not None:
                tree.merge_window()
            else:
                ds.close_window()
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t0) * 1e6)
        lat.sort()
        latency = {"p50_us": lat[len(lat) // 2], "p99_us": lat[min(len(lat) - 1, int(len(lat) * 0.99))],
                   "max_us": lat[-1], "windows": len(lat)}

    verify = None
    if a.verify and rank == 0:
        if world == 1:
            verify = verify_labels(ds, src, dst, V)
        else:                                   # the union of every rank's slices
            gs = torch.empty(E_rank * world, dtype=torch.int32, device=dev)
            gd = torch.empty(E_rank * world, dtype=torch.int32, device=dev)
            gen.rmat(gs, gd, 0, a.scale, a.seed)
            verify = verify_labels(ds, gs, gd, V)

    if rank == 0:
        total_edges = a.steps * E_rank * world
        folds = a.steps * nwin                       # window folds in the timed region (this rank)
        fold_win_ms = fold_ms / max(folds, 1)        # fold time per window (window 1 = several launches)
        achieved = BYTES_PER_EDGE_ALG * W_rank / (fold_win_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(a.traffic_json):
            try:
                tj = json.load(open(a.traffic_json))
                if tj.get("window_edges") == W_rank and tj.get("scale") == a.scale:
                    traffic = tj.get("hbm_bytes_per_window")
            except Exception:
                traffic = None
        nv, nc = ds.stats()
        line = {
            "metric": METRIC,
            "value": total_edges / elapsed,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: counter-based %s stream generated in HBM (seed %d), no dataset"
                    % ("Erdos-Renyi" if a.workload == "c4" else "RMAT", a.seed),
            "config": {
                "workload": "%s_%s%d_ef%d_window%s" % (a.workload, "er" if a.workload == "c4" else "rmat",
                                                        a.scale, a.edge_factor, _pow2(W_rank)),
                "scale": a.scale, "vertices": V, "edge_factor_per_gpu": a.edge_factor,
                "edges_per_gpu": E_rank, "window_edges_per_gpu": W_rank, "windows": nwin,
                "parallelism": "1 subtask per GPU x %d, %s" % (world, ("RCCL %s merge" % a.merge) if world > 1 else "no merge"),
                "emission": "per window, canonical min-id labels resident in HBM",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "UpdateCC per window: k_fold_ring (steady windows) / k_fold (young-forest launches)",
                "alg_bytes_per_window": BYTES_PER_EDGE_ALG * W_rank,
                "fold_ms_per_window": fold_win_ms,
                "fold_launches": fold_n,
                "windows_timed": folds,
            },
            "kernels": {
                "fold_share": fold_ms / (elapsed * 1e3),
                "compress_ms_per_window": comp_ms / max(comp_n, 1),
                "compress_share": comp_ms / (elapsed / a.steps * 1e3),
            },
            "final_vertices": nv,
            "final_components": nc,
        }
        if world > 1:                                # rank 0's side of the exchange
            line["exchange"] = {
                "merge": a.merge,
                "merge_fold_ms_per_window": merge_ms / max(folds, 1),
                "export_ms_per_window": export_ms / max(folds, 1),
                "bytes_sent_per_window": tree.bytes_sent / (a.warmup + a.steps + 1) / nwin,
                "bytes_recv_per_window": tree.bytes_recv / (a.warmup + a.steps + 1) / nwin,
                "wall_ms_per_window": elapsed / a.steps / nwin * 1e3,
            }
        if verify is not None:
            line["verify"] = verify
        if latency is not None:
            line["window_latency"] = latency
        if not a.no_cpu_baseline and world == 1:
            log("timed region done (%.1f ms/step); cpu baseline..." % (elapsed / a.steps * 1e3))
            line["cpu_baseline"] = cpu_baseline(a, src, dst, W_rank)
        print(json.dumps(line), flush=True)
    if gather:
        tree.drain()
    ds.close()
    if world > 1:
        dist.destroy_process_group()


def _pow2(x: int) -> str:
    for suf, sh in (("G", 30), ("M", 20), ("K", 10)):
        if x >= (1 << sh) and x % (1 << sh) == 0:
            return "%d%s" % (x >> sh, suf)
    return str(x)


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
    lab = torch.empty(V, dtype=torch.int32, device=src.device)
    ds.dense(out=lab)
    lab = lab.long()
    s, d = src.long(), dst.long()
    ok_edges = bool((lab[s] == lab[d]).all())
    seen = lab >= 0
    v = torch.arange(V, device=src.device)
    ok_min = bool((lab[seen] <= v[seen]).all()) and bool((lab[lab[seen]] == lab[seen]).all())
    ok_exact = bool(torch.equal(lab, torch_min_labels(src, dst, V)))
    return {"edges_consistent": ok_edges, "labels_minimal_idempotent": ok_min, "equals_torch_cc": ok_exact}


def cpu_baseline(a, src, dst, W):
    """Reference-semantics CPU restatement (oracle/, C): hash-map DisjointSet per partition on P
    host threads, single-thread CombineCC + Merger, FlattenSet emission per window; timed on a
    bounded sample (the first windows of the same stream)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import EMIT_FLATTEN, coracle
    import numpy as np
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    cores = max(1, min(cores, 16, os.cpu_count() or 1))
    n = min(max(a.cpu_sample_edges // W, 1) * W, src.numel())
    hs = src[:n].cpu().numpy().astype(np.int64)
    hd = dst[:n].cpu().numpy().astype(np.int64)
    r = coracle().run(hs, hd, W, partitions=cores, threads=cores, emit=EMIT_FLATTEN)
    return {"value": n / r["seconds"], "unit": "edges/s", "cores": cores, "kind": "port",
            "sample": "first %d windows (%d edges) of the same RMAT-%d stream, window %d edges, "
                      "P=%d partitions on %d threads, FlattenSet emission per window; %.1f s"
                      % (r["windows"], n, a.scale, W, cores, cores, r["seconds"])}


if __name__ == "__main__":
    main()
