#!/bin/bash
# Round 6: the strong-layout rank model (tools/sim_ranks.py) — prefilter as shipped vs senders with a
# partition forest (prefilter_forest); P = 8 (2^21 per rank) unless given.
set -u
TAG=${1:-r06_sim}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "${@:-8 21}"; do
  set -- $cfg
  SIM_WLOG2=$2 timeout -k 10 900 python -u tools/sim_ranks.py $1 64 prefilter prefilter_forest > "$OUT/sim_p$1.txt" 2>&1
  rc=$?; echo "sim P=$1 rc=$rc"; grep TOTAL "$OUT/sim_p$1.txt"; [ $rc -eq 0 ] || { tail -5 "$OUT/sim_p$1.txt"; exit 3; }
done
exit 0
