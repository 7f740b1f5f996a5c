#!/bin/bash
# Round 6: rank model with no synchronous broadcast at all (SIM_SYNC=0: window 2's edges all go to
# rank 0, filtered there by its own giant) against the shipped one-broadcast schedule, P = 8 and 4.
set -u
TAG=${1:-r06_p}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "8 21 1" "8 21 0" "4 22 1" "4 22 0"; do
  set -- $cfg
  SIM_SYNC=$3 SIM_WLOG2=$2 timeout -k 10 600 python -u tools/sim_ranks.py $1 64 prefilter > "$OUT/sim_p$1_sync$3.txt" 2>&1
  rc=$?; echo "P=$1 sync=$3 rc=$rc $(grep TOTAL $OUT/sim_p$1_sync$3.txt)"; [ $rc -eq 0 ] || { tail -5 "$OUT/sim_p$1_sync$3.txt"; exit 3; }
  grep "^w  [1-4] " "$OUT/sim_p$1_sync$3.txt"
done
exit 0
