#!/bin/bash
# Round 5: GS_MERGE_PREFILTER with the balanced rank-0 share and 16-window broadcasts — its GPU
# tests, the 8-rank RMAT-26 headline layout (hot / warm sets on the senders), and the rank model.
set -u
OUT=gpurun_out/r05_pre2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_prefilter.py tests/test_gpu_variants.py -k "prefilter" -x -v \
    --timeout 850 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert" "$OUT/pytest.log" | head -20; exit 3; }
for cfg in "2 23" "4 22" "8 21"; do
  set -- $cfg
  SIM_WLOG2=$2 timeout -k 10 600 python -u tools/sim_ranks.py $1 64 prefilter > "$OUT/sim_p$1.txt" 2>&1
  rc=$?; echo "sim P=$1 rc=$rc"; grep TOTAL "$OUT/sim_p$1.txt"; [ $rc -eq 0 ] || { tail -5 "$OUT/sim_p$1.txt"; exit 3; }
done
exit 0
