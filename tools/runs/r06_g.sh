#!/bin/bash
# Round 6: rank model with pair folds at one edge per thread (kSmallPairFold), rank 0's share swept
# at P = 4 and 2 (SIM_SHARE0 = bench.py --share0), P = 8 at its default.
set -u
TAG=${1:-r06_g}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "8 21 -" "4 22 0" "4 22 0.05" "4 22 0.1" "4 22 -" "2 23 0.25" "2 23 0.35" "2 23 -"; do
  set -- $cfg
  if [ "$3" = "-" ]; then e="SIM_X=1"; else e="SIM_SHARE0=$3"; fi
  env $e SIM_WLOG2=$2 timeout -k 10 600 python -u tools/sim_ranks.py $1 64 prefilter > "$OUT/sim_p$1_s$3.txt" 2>&1
  rc=$?; echo "sim P=$1 share0=$3 rc=$rc $(grep TOTAL $OUT/sim_p$1_s$3.txt)"; [ $rc -eq 0 ] || { tail -5 "$OUT/sim_p$1_s$3.txt"; exit 3; }
done
exit 0
