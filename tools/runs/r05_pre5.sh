#!/bin/bash
# Round 5: the Merger's raw-edge survivor fold takes the young split — prefilter tests, the
# variant checker (all streams), the 8-rank headline layout, the rank model at P = 2, 4, 8.
set -u
OUT=gpurun_out/r05_pre5
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_prefilter.py tests/test_gpu_comm.py tests/test_gpu_variants.py -k "prefilter or batch or gather" -x -v \
    --timeout 850 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert" "$OUT/pytest.log" | head -20; exit 3; }
for cfg in "2 23" "4 22" "8 21"; do
  set -- $cfg
  SIM_WLOG2=$2 timeout -k 10 600 python -u tools/sim_ranks.py $1 64 prefilter > "$OUT/sim_p$1.txt" 2>&1
  rc=$?; echo "sim P=$1 rc=$rc"; grep TOTAL "$OUT/sim_p$1.txt"; [ $rc -eq 0 ] || { tail -5 "$OUT/sim_p$1.txt"; exit 3; }
done
exit 0
