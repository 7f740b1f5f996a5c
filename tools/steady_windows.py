"""Per-window durations of the steady fold's kernels from a rocprofv3 kernel trace (last step):
usage: python tools/steady_windows.py <kernel_trace.csv> [first_window]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
first = int(sys.argv[2]) if len(sys.argv) > 2 else 13
ks = sorted(((r["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1], int(r["Start_Timestamp"]),
             int(r["End_Timestamp"])) for r in rows), key=lambda x: x[1])
HEADS = ("k_fold_ring",)
heads = [i for i, k in enumerate(ks) if k[0].startswith(HEADS)]
last = heads[-63:]                                  # windows 2..64 of the last step
tot = defaultdict(float)
n = 0
span = 0.0
for w, i in enumerate(last, 2):
    if w < first:
        continue
    n += 1
    j = i
    t0 = ks[i][1]
    while j < len(ks) and (j == i or not ks[j][0].startswith(HEADS)):
        if ks[j][0].startswith(("k_compress", "k_pick")):
            break
        tot[ks[j][0]] += (ks[j][2] - ks[j][1]) / 1000
        span_end = ks[j][2]
        j += 1
    span += (span_end - t0) / 1000
print("windows %d-64 (%d): mean us per window" % (first, n))
for k, v in tot.items():
    print("  %-28s %8.1f" % (k, v / n))
print("  %-28s %8.1f" % ("sum of kernels", sum(tot.values()) / n))
print("  %-28s %8.1f" % ("first start -> last end", span / n))
