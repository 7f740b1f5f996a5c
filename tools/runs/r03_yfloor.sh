#!/bin/bash
# Workgroup floor of the first young launch after reset (GSGPU_YOUNG_FIRST_MIN): config 2 (its
# first launch is 2^18 edges, at the floor) and config 5. usage: bash tools/r03_yfloor.sh <tag>
set -u
TAG=${1:-r03_yfloor}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for F in ${FLOORS:-32 8 16 64 32}; do
  for w in c2; do
    n=${w}_f$F
    GSGPU_YOUNG_FIRST_MIN=$F timeout -k 10 300 python -u bench.py --workload $w --steps 10 --no-cpu-baseline > "$OUT/$n.json" 2> "$OUT/$n.err"
    rc=$?; echo "$n rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('%.3f G/s %.4f ms/step'%(d['value']/1e9,d['ms_per_step']))" 2>/dev/null)"
    [ $rc -eq 0 ] || { tail -3 "$OUT/$n.err"; exit 3; }
  done
done
exit 0
