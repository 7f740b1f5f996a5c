"""Host-bound or GPU-bound? Reads a rocprofv3 --kernel-trace --hip-trace CSV pair and, for the
kernels of the run's last stretch, splits every gap between consecutive kernels into
  host-late : the API call that enqueued the kernel returned after the previous kernel had ended
              (the GPU waited for the host), and
  dispatch  : the call returned before that (the GPU-side launch latency of a dependent kernel).
Also sums the host's blocking calls (event / stream synchronisation) over the same stretch.

usage: python tools/hosttrace.py <rocprofv3 output dir> [kernels to analyse, default 6000 | first:last]
(first:last = a slice of the kernels sorted by start time, e.g. one timed step)
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def rows(pattern):
    fs = glob.glob(pattern, recursive=True)
    if not fs:
        raise SystemExit("no file matches " + pattern)
    with open(fs[0], newline="") as f:
        return list(csv.DictReader(f))


def short(name):
    n = name.split("(")[0]
    for p in ("void ", "gsgpu::", "(anonymous namespace)::"):
        n = n.replace(p, "")
    return n[:40]


def main():
    d = sys.argv[1]
    sel = sys.argv[2] if len(sys.argv) > 2 else "6000"
    ks = rows(os.path.join(d, "**", "*kernel_trace.csv"))
    api = rows(os.path.join(d, "**", "*hip_api_trace.csv"))
    by_corr = {}
    for r in api:
        by_corr[int(r["Correlation_Id"])] = r
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    if ":" in sel:
        lo, hi = (int(x) for x in sel.split(":"))
        ks = ks[lo:hi]
    else:
        ks = ks[-int(sel):]
    t_lo, t_hi = int(ks[0]["Start_Timestamp"]), int(ks[-1]["End_Timestamp"])
    busy = sum(int(k["End_Timestamp"]) - int(k["Start_Timestamp"]) for k in ks)
    late = defaultdict(lambda: [0, 0])          # kernel name -> [ns the GPU waited for the host, count]
    disp = defaultdict(lambda: [0, 0])          # kernel name -> [dispatch-gap ns, count]
    host_cost = defaultdict(lambda: [0, 0])     # API function -> [ns inside the call, count]
    prev_end = int(ks[0]["End_Timestamp"])
    for k in ks[1:]:
        s, e = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
        gap = s - prev_end
        a = by_corr.get(int(k["Correlation_Id"]))
        name = short(k["Kernel_Name"])
        if gap > 0:
            if a is not None and int(a["End_Timestamp"]) > prev_end:
                hl = min(gap, int(a["End_Timestamp"]) - prev_end)
                late[name][0] += hl
                late[name][1] += 1
                disp[name][0] += gap - hl
            else:
                disp[name][0] += gap
            disp[name][1] += 1
        prev_end = max(prev_end, e)
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t_lo <= s <= t_hi:
            host_cost[r["Function"]][0] += e - s
            host_cost[r["Function"]][1] += 1
    span = t_hi - t_lo
    print("last %d kernels: span %.3f ms, GPU busy %.3f ms (%.1f %%), gaps %.3f ms" %
          (len(ks), span / 1e6, busy / 1e6, 100.0 * busy / span, (span - busy) / 1e6))
    tl = sum(v[0] for v in late.values())
    td = sum(v[0] for v in disp.values())
    print("  GPU waiting for the host (enqueue returned after the previous kernel ended): %.3f ms" % (tl / 1e6))
    print("  dispatch gaps (kernel already enqueued): %.3f ms" % (td / 1e6))
    print("\nper kernel: host-late ns total / count, dispatch-gap ns total / count")
    for n in sorted(set(late) | set(disp), key=lambda n: -(late[n][0] + disp[n][0])):
        print("  %-40s late %10d / %5d   gap %10d / %5d  (avg gap %.1f us)" %
              (n, late[n][0], late[n][1], disp[n][0], disp[n][1], (late[n][0] + disp[n][0]) / max(1, disp[n][1]) / 1e3))
    print("\nHIP API calls inside the stretch: total ns / count (avg us)")
    for f, (t, c) in sorted(host_cost.items(), key=lambda x: -x[1][0])[:25]:
        print("  %-36s %12d / %6d  (%.2f us)" % (f, t, c, t / c / 1e3))


if __name__ == "__main__":
    main()
