#!/bin/bash
# Round-4 same-box A/B: config-5 bench with and without a library switch, alternated, after the
# config-5 fixture check of the production path. usage: bash tools/r04_ab.sh <tag> <VAR> [workload]
set -u
TAG=${1:-r04_ab}; VAR=${2:-GSGPU_PREFETCH}; WL=${3:-c5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tests/headline_check.py --fixture c5 --fold-windows --chunk 256 > "$OUT/c5fix.json" 2> "$OUT/c5fix.err"
rc=$?; echo "c5fix rc=$rc"; tail -1 "$OUT/c5fix.json" | cut -c1-300; [ $rc -eq 0 ] || { tail -5 "$OUT/c5fix.err"; exit 3; }
for i in 1 2; do
  for v in 1 0; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --workload $WL --steps 3 --no-cpu-baseline > "$OUT/b_${v}_$i.json" 2> "$OUT/b_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_${v}_$i.err"; exit 3; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/b_${v}_$i.json') if l.startswith('{')][-1]); print('$VAR=$v run $i: %.3f G edges/s, %.3f ms/step, p50 %s' % (d['value']/1e9, d['ms_per_step'], (d.get('window_latency') or {}).get('p50_us')))"
  done
done
exit 0
