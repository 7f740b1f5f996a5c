"""Fold rocprofv3 --pmc CSVs (tools/pmc_traffic.sh) into per-window HBM traffic of k_fold.

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of wide (16 B/lane) coalesced streaming reads, so the streaming edge read
is doubled; the random 4-B gathers of this kernel are an uncalibrated width, reported raw beside.
Output: profiles/fold_traffic.json-shaped dict (bench.py reads hbm_bytes_per_window from it).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gelly-streaming_amd"))
from gsgpu._abi import lib_source_sha  # noqa: E402



def load(passdir):
    files = glob.glob(os.path.join(passdir, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(lambda: defaultdict(float))    # kernel -> counter -> sum over dispatches
    calls = defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add(r.get("Dispatch_Id", r.get("Correlation_Id")))
    return vals, calls


def fold_sequence(passdir):
    """Counters of each fold launch (k_fold / k_fold_ring) in dispatch order."""
    files = glob.glob(os.path.join(passdir, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: defaultdict(float))
    name = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "k_fold" not in k:
                continue
            d = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            name[d] = k
    return [(name[d], per[d]) for d in sorted(per)]


def young_windows(root, window_edges):
    """Per-window fold counters of the first bench step: window 1 = the two young k_fold launches
    (split at capacity/16), window w >= 2 = its k_fold_ring launch; windows 13.. averaged."""
    seqs = [fold_sequence(p) for p in sorted(glob.glob(os.path.join(root, "p*"))) if os.path.isdir(p)]
    seqs = [q for q in seqs if q]
    if not seqs:
        return None
    n = min(len(q) for q in seqs)
    launches = []
    for i in range(n):
        c = {}
        for q in seqs:
            c.update(q[i][1])
        launches.append((seqs[0][i][0], c))
    wins = []
    i = 0
    while i < n and len(wins) < 64:
        k, c = launches[i]
        group = [c]
        if "k_fold_ring" not in k and i + 1 < n and "k_fold_ring" not in launches[i + 1][0] and not wins:
            group.append(launches[i + 1][1])     # window 1: young head + rest
            i += 1
        i += 1
        tot = defaultdict(float)
        for g in group:
            for kk, vv in g.items():
                tot[kk] += vv
        wins.append(tot)
    rows = []
    for w, t in enumerate(wins, 1):
        h, m = t.get("TCC_HIT_sum", 0.0), t.get("TCC_MISS_sum", 0.0)
        rows.append({"window": w, "fetch_bytes_raw": t.get("FETCH_SIZE", 0.0) * 1024,
                     "write_bytes": t.get("WRITE_SIZE", 0.0) * 1024,
                     "hbm_bytes": t.get("FETCH_SIZE", 0.0) * 1024 + 4 * window_edges + t.get("WRITE_SIZE", 0.0) * 1024,
                     "tcc_requests": h + m, "l2_hit_rate": h / (h + m) if h + m else None,
                     "memory_side_atomics": t.get("TCC_EA0_ATOMIC_sum", 0.0)})
    steady = rows[12:]
    avg = {k: sum(r[k] for r in steady) / len(steady) for k in ("fetch_bytes_raw", "write_bytes", "hbm_bytes",
                                                              "tcc_requests", "memory_side_atomics")} if steady else None
    return {"windows_1_12": rows[:12], "steady_mean_13_on": avg,
            "note": "per window of the first bench step; hbm_bytes adds back half the 8 B/edge stream "
                    "(gfx950 FETCH_SIZE reports wide streaming reads at 1/2)"}


def main():
    root = sys.argv[1]
    agg = defaultdict(dict)
    ncalls = {}
    for p in sorted(glob.glob(os.path.join(root, "p*"))):
        if not os.path.isdir(p):
            continue
        v, c = load(p)
        for k in v:
            agg[k].update(v[k])
            ncalls[k] = len(c[k])
    comp = [k for k in agg if "k_compress" in k]
    windows = ncalls[comp[0]] if comp else 1
    fold = [k for k in agg if "k_fold" in k]
    out = {"windows": windows, "kernels": {}}
    for k in agg:
        out["kernels"][k] = dict(agg[k], dispatches=ncalls.get(k))
    fetch = sum(agg[k].get("FETCH_SIZE", 0.0) for k in fold) * 1024
    write = sum(agg[k].get("WRITE_SIZE", 0.0) for k in fold) * 1024
    hit = sum(agg[k].get("TCC_HIT_sum", 0.0) for k in fold)
    miss = sum(agg[k].get("TCC_MISS_sum", 0.0) for k in fold)
    out["fold"] = {
        "fetch_bytes_raw_per_window": fetch / windows,
        "write_bytes_per_window": write / windows,
        "l2_hit_rate": hit / (hit + miss) if hit + miss else None,
        "atomic_requests_per_window": sum(agg[k].get("TCC_EA0_ATOMIC_sum", 0.0) for k in fold) / windows,
    }
    edges_per_launch = None
    try:
        bj = os.path.join(root, "..", "bench.json")
        if os.path.exists(bj):
            b = json.load(open(bj))
        else:                                          # the bench line in the first pass's log
            lines = [l for l in open(os.path.join(root, "p1.log")) if l.startswith("{")]
            b = json.loads(lines[-1])
        out["window_edges"] = b["config"]["window_edges_per_gpu"]
        out["scale"] = b["config"]["scale"]
        out["id_bits"] = b["config"].get("id_bits", 32)
        edges_per_launch = b["roofline"].get("edges_per_launch")
    except Exception:
        pass
    out["lib_source_sha"] = lib_source_sha()
    # the steady fold per launch (what bench.py's roofline.traffic / requests report): k_fold_ring
    ks, name = [k for k in agg if "k_fold_ring" in k], "k_fold_ring"
    if ks:
        nl = max(sum(ncalls.get(k) or 0 for k in ks), 1)
        f_ = sum(agg[k].get("FETCH_SIZE", 0.0) for k in ks) * 1024 / nl
        w_ = sum(agg[k].get("WRITE_SIZE", 0.0) for k in ks) * 1024 / nl
        h_ = sum(agg[k].get("TCC_HIT_sum", 0.0) for k in ks)
        m_ = sum(agg[k].get("TCC_MISS_sum", 0.0) for k in ks)
        e_b = 8 * (edges_per_launch or 0) * (2 if out.get("id_bits", 32) == 64 else 1)
        out["steady"] = {
            "kernel": name, "kernels": ks, "launches": nl, "edges_per_launch": edges_per_launch,
            "fetch_bytes_raw_per_launch": f_, "write_bytes_per_launch": w_,
            # gfx950: FETCH_SIZE reports half the bytes of wide (16 B/lane) streaming reads — the
            # edge stream (MI355X_MICROARCH.md, HBM section): that half is added back; list reads and
            # random gathers are counted raw (uncalibrated widths)
            "hbm_bytes_per_launch": f_ + e_b / 2 + w_,
            "l2_hit_rate": h_ / (h_ + m_) if h_ + m_ else None,
            "tcc_requests_per_launch": (h_ + m_) / nl,
            "memory_side_atomics_per_launch": sum(agg[k].get("TCC_EA0_ATOMIC_sum", 0.0) for k in ks) / nl,
        }
    # the dominant kernel alone, per launch (what bench.py's roofline.traffic reports): k_fold_ring
    ring = [k for k in agg if "k_fold_ring" in k]
    if ring:
        k = ring[0]
        nl = max(ncalls.get(k) or 1, 1)
        f_ring = agg[k].get("FETCH_SIZE", 0.0) * 1024 / nl
        w_ring = agg[k].get("WRITE_SIZE", 0.0) * 1024 / nl
        e_ring = 8 * out.get("window_edges", 0) * (2 if out.get("id_bits", 32) == 64 else 1)
        h_, m_ = agg[k].get("TCC_HIT_sum", 0.0), agg[k].get("TCC_MISS_sum", 0.0)
        out["ring"] = {
            "kernel": k, "launches": nl,
            "fetch_bytes_raw_per_launch": f_ring, "write_bytes_per_launch": w_ring,
            # gfx950: FETCH_SIZE reports half the bytes of the wide (16 B/lane) streaming edge read
            # (MI355X_MICROARCH.md, HBM section): add that half back; random 4-B gathers uncalibrated
            "hbm_bytes_per_launch": f_ring + e_ring / 2 + w_ring,
            "l2_hit_rate": h_ / (h_ + m_) if h_ + m_ else None,
            "tcc_requests_per_launch": (h_ + m_) / nl,
            "memory_side_atomics_per_launch": agg[k].get("TCC_EA0_ATOMIC_sum", 0.0) / nl,
        }
    out["per_window"] = young_windows(root, out.get("window_edges", 0))
    # streaming edge read (8 B/edge, 16 B/lane loads) is under-reported 2x: add it back once
    edge_bytes = 8 * out.get("window_edges", 0)
    out["hbm_bytes_per_window"] = out["fold"]["fetch_bytes_raw_per_window"] + edge_bytes / 2 + out["fold"]["write_bytes_per_window"]
    out["note"] = ("hbm_bytes_per_window = FETCH_SIZE*1024 + half the 8 B/edge stream (gfx950 reports wide "
                   "streaming reads at 1/2) + WRITE_SIZE*1024, per window fold; gathers uncalibrated")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
