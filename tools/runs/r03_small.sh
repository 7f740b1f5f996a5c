#!/bin/bash
# Small plain folds, edges per thread (GSGPU_SMALL_FOLD / GSGPU_SMALL_EPT): configs 5 and 2.
# usage: bash tools/r03_small.sh <tag>
set -u
TAG=${1:-r03_small}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # name workload env...
  local n=$1 w=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $w --steps 3 --no-cpu-baseline > "$OUT/$n.json" 2> "$OUT/$n.err"
  local rc=$?
  echo "$n rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('%.3f G/s %.3f ms/step'%(d['value']/1e9,d['ms_per_step']), d.get('window_latency',{}).get('p50_us',''))" 2>/dev/null)"
  [ $rc -eq 0 ] || { tail -3 "$OUT/$n.err"; exit 3; }
}
run c5_base c5 GSGPU_SMALL_FOLD=0
run c5_e1 c5 GSGPU_SMALL_FOLD=1048576 GSGPU_SMALL_EPT=1
run c5_e2 c5 GSGPU_SMALL_FOLD=1048576 GSGPU_SMALL_EPT=2
run c2_base c2 GSGPU_SMALL_FOLD=0
run c2_e1 c2 GSGPU_SMALL_FOLD=1048576 GSGPU_SMALL_EPT=1
run c2_e2 c2 GSGPU_SMALL_FOLD=1048576 GSGPU_SMALL_EPT=2
run c4_base c4 GSGPU_SMALL_FOLD=0
run c4_e1 c4 GSGPU_SMALL_FOLD=1048576 GSGPU_SMALL_EPT=1
GSGPU_SMALL_FOLD=1048576 GSGPU_SMALL_EPT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "baseline_config or c5_small or random_streams" > "$OUT/pytest_e1.log" 2>&1
rc=$?; echo "pytest e1 rc=$rc $(tail -1 $OUT/pytest_e1.log)"
exit 0
