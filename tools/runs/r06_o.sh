#!/bin/bash
# Round 6: the rank model with one lagging summary per sender (each sender's hot-set admission at the
# protocol's cadence) at P = 2 / 4 / 8, and the shared-summary model at P = 8 on the same box.
set -u
TAG=${1:-r06_o}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "8 21 per" "8 21 shared" "4 22 per" "2 23 per"; do
  set -- $cfg
  if [ $3 = shared ]; then e="SIM_SHARED_LAG=1"; else e="X=1"; fi
  env $e SIM_WLOG2=$2 timeout -k 10 600 python -u tools/sim_ranks.py $1 64 prefilter > "$OUT/sim_p$1_$3.txt" 2>&1
  rc=$?; echo "P=$1 $3 rc=$rc $(grep TOTAL $OUT/sim_p$1_$3.txt)"; [ $rc -eq 0 ] || { tail -5 "$OUT/sim_p$1_$3.txt"; exit 3; }
done
exit 0
