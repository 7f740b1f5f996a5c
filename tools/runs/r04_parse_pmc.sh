#!/bin/bash
# PMC passes over the parse line: bytes, L2, and instruction mix of k_parse_chunk
set -u
TAG=${1:-r04_parse_pmc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/p$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload parse --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($C) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
cd "$GRAFT_REPO_ROOT"
for i in 1 2 3 4 5; do
  python3 - "$OUT/p$i" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
vals = defaultdict(lambda: defaultdict(float)); calls = defaultdict(set)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "gsgpu" not in k: continue
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"]); calls[k].add(r.get("Dispatch_Id"))
for k in vals:
    print(k[:40], {c: round(v / max(1, len(calls[k]))) for c, v in vals[k].items()})
PY
done
rm -rf "$OUT"/p[0-9]
