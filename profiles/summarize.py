"""Summarise a rocprofv3 --kernel-trace CSV of bench.py into the per-window figures bench.py
reports (profiles/README: how each committed summary was produced).

usage: python profiles/summarize.py <run_kernel_trace.csv> <bench.json> [--window-edges N] [--windows-per-step W]
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    b = json.loads(open(bench).read().strip().splitlines()[-1])
    W = b["config"]["window_edges_per_gpu"]
    nwin = b["config"]["windows"]
    rows = list(csv.DictReader(open(trace)))
    per = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)   # ms
    kern = {k: {"calls": len(v), "total_ms": sum(v), "avg_ms": sum(v) / len(v)} for k, v in per.items()}
    fold = sum(v["total_ms"] for k, v in kern.items() if "k_fold" in k or k.endswith("k_bin"))
    comp = [v for k, v in kern.items() if "k_compress" in k]
    windows = comp[0]["calls"] if comp else None           # one compress per window on rank 0
    out = {
        "source_trace": trace, "bench": bench,
        "kernels": kern,
        "windows_in_trace": windows,
        "fold_ms_per_window_rocprof": fold / windows if windows else None,
        "fold_ms_per_window_bench": b["roofline"].get("fold_ms_per_window"),
        "alg_bytes_per_window": 16 * W,
    }
    if windows:
        out["achieved_GBs_rocprof"] = 16 * W / (fold / windows * 1e-3) / 1e9
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
