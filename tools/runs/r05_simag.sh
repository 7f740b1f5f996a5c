#!/bin/bash
# Round 5: the replicated all-gather exchange in the one-GPU rank model, kernel-time accounting
# (the same clock as the prefilter model in r05_pre2).
set -u
OUT=gpurun_out/r05_simag
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "2 23" "4 22" "8 21"; do
  set -- $cfg
  SIM_WLOG2=$2 timeout -k 10 600 python -u tools/sim_ranks.py $1 64 allgather > "$OUT/sim_p$1.txt" 2>&1
  rc=$?; echo "sim P=$1 rc=$rc"; grep TOTAL "$OUT/sim_p$1.txt"; [ $rc -eq 0 ] || { tail -5 "$OUT/sim_p$1.txt"; exit 3; }
done
exit 0
