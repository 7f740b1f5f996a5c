"""Dispatch sequence of the last N kernel dispatches of a rocprofv3 --kernel-trace CSV, with gaps:
python tools/trace_seq.py <run_kernel_trace.csv> [N] [name-filter]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 80
filt = sys.argv[3] if len(sys.argv) > 3 else ""
rows = [r for r in rows if filt in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("void ", "").split("(")[0].replace("gsgpu::", "")
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print("%9.1f us  gap %7.1f  grid %8s  %s" % ((e - s) / 1e3, gap, r["Grid_Size_X"], name))
    prev = e
