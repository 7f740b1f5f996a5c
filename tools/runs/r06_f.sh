#!/bin/bash
# Round 6: rank model at P = 8 — variance of the default, and the Merger's survivor folds at one edge
# per thread up to 2^20 / 2^22 edges (GSGPU_SMALL_FOLD).
set -u
TAG=${1:-r06_f}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in default 1048576 4194304 default2; do
  if [ ${v#default} != $v ]; then e=""; else e="GSGPU_SMALL_FOLD=$v"; fi
  env $e SIM_WLOG2=21 timeout -k 10 600 python -u tools/sim_ranks.py 8 64 prefilter > "$OUT/sim_p8_$v.txt" 2>&1
  rc=$?; echo "sim $v rc=$rc $(grep TOTAL $OUT/sim_p8_$v.txt)"; [ $rc -eq 0 ] || { tail -5 "$OUT/sim_p8_$v.txt"; exit 3; }
done
exit 0
