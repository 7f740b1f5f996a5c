#!/bin/bash
# small-fold claims (k_fold one edge per thread next to the giant, GSGPU_SMALL_CLAIM): parity,
# then a config-5 A/B, 4 alternations
set -u
TAG=${1:-r04_claim5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_listclose.py \
  tests/test_gpu_parity.py tests/test_gpu_variants.py -k "listclose or list_close or c5 or random_streams or baseline_config or emit_delta or streams_golden" \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -20; exit 3; }
for i in 1 2 3 4; do
  for v in 1 0; do
    GSGPU_SMALL_CLAIM=$v timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --no-cpu-baseline > "$OUT/b_${v}_$i.json" 2> "$OUT/b_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_${v}_$i.err"; exit 3; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/b_${v}_$i.json') if l.startswith('{')][-1]); print('c5 CLAIM=$v run $i: %.3f G edges/s, %.3f ms/step, p50 %.1f, fold ms/launch %.4f' % (d['value']/1e9, d['ms_per_step'], (d.get('window_latency') or {}).get('p50_us'), d['roofline']['avg_launch_ms']))"
  done
done
exit 0
