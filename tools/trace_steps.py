"""Per-window kernel durations of one bench step from a rocprofv3 --kernel-trace CSV.
usage: python tools/trace_steps.py <run_kernel_trace.csv> [step index (0 = warmup), default 1]
A step's windows are cut at its k_compress launches (window 1 of a 2^26-id stream has two: the
young split's internal close); steps are cut at the young k_fold that follows a reset's memsets."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
step_ix = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gsgpu::", "").split("<")[0]) for r in rows)
# steps: a young k_fold following a k_compress (or at the start) opens a step
steps, cur, prev, filled = [], [], None, False
for k in ks:
    # a step opens with the summary's reset (memsets) followed by the young k_fold
    if k[2] == "k_fold" and filled and prev in (None, "k_compress", "k_compress_list", "k_stats") and cur and \
            any(x[2].startswith("k_compress") for x in cur):
        steps.append(cur)
        cur = []
    if k[2].startswith("k_gen") or k[2].startswith("__amd"):
        # generator / memsets: not part of a window; a reset's parent[] fill is the long one
        filled = filled or ("fill" in k[2] and k[1] - k[0] > 20000)
        continue
    filled = False
    cur.append(k)
    prev = k[2]
steps.append(cur)
if step_ix >= len(steps):
    print("only %d steps found; using the last" % len(steps))
    step_ix = len(steps) - 1
st = steps[step_ix]
wins, w = [], []
for k in st:
    w.append(k)
    if k[2] == "k_compress" or k[2] == "k_compress_list":
        wins.append(w)
        w = []
print("steps found: %d; step %d: %d closes, span %.1f us" % (len(steps), step_ix, len(wins), (st[-1][1] - st[0][0]) / 1e3))
tot = defaultdict(float)
for i, w in enumerate(wins):
    d = defaultdict(float)
    for s, e, n in w:
        d[n] += (e - s) / 1e3
        tot[n] += (e - s) / 1e3
    span = (w[-1][1] - w[0][0]) / 1e3
    if i < 14 or i % 16 == 0 or i == len(wins) - 1:
        print("close-interval %2d span %7.1f  " % (i + 1, span) + "  ".join("%s %.1f" % (n, t) for n, t in sorted(d.items())))
print("totals: " + "  ".join("%s %.1f" % (n, t) for n, t in sorted(tot.items())))
