"""Per-dispatch distribution of one PMC counter for one kernel, from a rocprofv3 --pmc pass
directory (tools/pmc_traffic.sh layout). usage: python tools/pmc_dist.py <passdir> <kernel-substr> [counter]"""
import csv
import glob
import os
import sys
from collections import defaultdict

passdir, ksub = sys.argv[1], sys.argv[2]
counter = sys.argv[3] if len(sys.argv) > 3 else "FETCH_SIZE"
vals = defaultdict(float)
for f in glob.glob(os.path.join(passdir, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if ksub in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[int(r.get("Dispatch_Id") or r.get("Correlation_Id"))] += float(r["Counter_Value"])
seq = [vals[d] * (1024 if counter in ("FETCH_SIZE", "WRITE_SIZE") else 1) for d in sorted(vals)]
if not seq:
    sys.exit("no dispatches")
s = sorted(seq)
q = lambda p: s[min(len(s) - 1, int(p * len(s)))]
print({"kernel": ksub, "counter": counter, "dispatches": len(seq), "mean": sum(seq) / len(seq),
       "p10": q(0.1), "p50": q(0.5), "p90": q(0.9), "p99": q(0.99), "max": s[-1],
       "first_16": [round(x) for x in seq[:16]], "windows_1000_1016": [round(x) for x in seq[1000:1016]],
       "last_8": [round(x) for x in seq[-8:]]})
