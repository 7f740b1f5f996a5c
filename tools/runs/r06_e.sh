#!/bin/bash
# Round 6: asynchronous filter-state broadcasts in GS_MERGE_PREFILTER — parity (prefilter tests, the
# 8-rank headline layout in every mode), then the rank model at P = 2, 4, 8.
set -u
TAG=${1:-r06_e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_prefilter.py tests/test_gpu_variants.py -k "prefilter or eight_ranks" -x -v --timeout 600 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || { tail -40 "$OUT/pytest.log"; exit 3; }
for cfg in "8 21" "4 22" "2 23"; do
  set -- $cfg
  SIM_WLOG2=$2 timeout -k 10 900 python -u tools/sim_ranks.py $1 64 prefilter > "$OUT/sim_p$1.txt" 2>&1
  rc=$?; echo "sim P=$1 rc=$rc $(grep TOTAL $OUT/sim_p$1.txt)"; [ $rc -eq 0 ] || { tail -5 "$OUT/sim_p$1.txt"; exit 3; }
done
exit 0
