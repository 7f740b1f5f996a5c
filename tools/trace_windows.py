"""Per-window kernel time of one timed bench step from a rocprofv3 kernel trace (bench.py run
with --steps S --warmup W): windows are cut at each emission close (k_compress preceded by a
fold launch), step boundaries at the reset fills. usage: trace_windows.py run_kernel_trace.csv"""
import csv, re, sys, collections

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = [re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("gsgpu::", "") for r in rows]
st = [int(r["Start_Timestamp"]) for r in rows]
en = [int(r["End_Timestamp"]) for r in rows]
# the timed steps: the rows between the first and the last k_stats-free stretch; take the second
# full step (warmup 1 + timed 2): a step starts at k_fold after a reset fill
def after_reset(i):          # gs_cc_reset's memsets: several fills right before the step's first fold
    return i >= 3 and all("fill" in name[j] for j in range(i - 3, i))


starts = [i for i in range(1, len(rows)) if name[i].startswith("k_fold<") and after_reset(i)]
if len(starts) < 3:
    sys.exit("need >= 3 steps in the trace")
a, b = starts[1], starts[2]
win, cur = [], collections.defaultdict(float)
for i in range(a, b):
    short = name[i].split("<")[0]
    cur[short] += (en[i] - st[i]) / 1e3
    cur["gap"] += (st[i] - en[i - 1]) / 1e3
    if short == "k_compress" and i + 1 < b and not name[i + 1].startswith("k_compress"):
        nxt = name[i + 1].split("<")[0]
        if nxt in ("k_fold_ring", "k_fold", "__amd_rocclr_fillBufferAligned"):
            win.append(cur)
            cur = collections.defaultdict(float)
if cur:
    win.append(cur)
keys = sorted({k for w in win for k in w})
print("window " + " ".join("%14s" % k[:14] for k in keys) + "      total")
for j, w in enumerate(win):
    print("%6d " % (j + 1) + " ".join("%14.1f" % w.get(k, 0.0) for k in keys) + " %10.1f" % sum(w.values()))
tot = collections.defaultdict(float)
for w in win:
    for k, v in w.items():
        tot[k] += v
print("step   " + " ".join("%14.1f" % tot[k] for k in keys) + " %10.1f" % sum(tot.values()))
