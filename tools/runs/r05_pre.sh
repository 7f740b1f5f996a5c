#!/bin/bash
# Round 5: GS_MERGE_PREFILTER — its GPU tests, the variant checker's prefilter cases (production
# environment), and the one-GPU rank model of the strong layout at P = 2, 4, 8.
set -u
PART=${1:-all}
OUT=gpurun_out/r05_pre
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$PART" = all ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_prefilter.py -x -v --timeout 600 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert" "$OUT/pytest.log" | head -20; exit 3; }
timeout -k 10 600 python -u tests/variant_check.py > "$OUT/variant.json" 2> "$OUT/variant.err"
rc=$?; echo "variant rc=$rc"; python -c "
import json; d=json.loads([l for l in open('$OUT/variant.json') if l.startswith('{')][-1]); print('ok', d['ok']); [print(c) for c in d['cases'] if 'prefilter' in c['case'] or not c['ok']]"
[ $rc -eq 0 ] || exit 3
fi
for cfg in "2 23" "4 22" "8 21"; do
  set -- $cfg
  SIM_WLOG2=$2 timeout -k 10 600 python -u tools/sim_ranks.py $1 64 prefilter > "$OUT/sim_p$1.txt" 2>&1
  rc=$?; echo "sim P=$1 rc=$rc"; grep TOTAL "$OUT/sim_p$1.txt"; [ $rc -eq 0 ] || { tail -5 "$OUT/sim_p$1.txt"; exit 3; }
done
exit 0
