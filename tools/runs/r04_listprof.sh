#!/bin/bash
# kernel stats of config 5 with and without list-mode closes (rocprofv3 --kernel-trace --stats)
set -u
TAG=${1:-r04_listprof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 1 0; do
  GSGPU_LIST_CLOSE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_$v" -o run --output-format csv -- python3 -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/b_$v.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_$v.log"; exit 3; }
  f=$(find "$OUT/prof_$v" -name "*kernel_stats.csv" | head -1)
  echo "LIST=$v"; python3 -c "
import csv,sys
for r in csv.reader(open('$f')):
    print(r[0][:50], r[1], r[3])
" | head -8
done
exit 0
