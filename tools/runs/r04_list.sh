#!/bin/bash
# Round-4 list-mode close: parity (list-close tests, small-window and delta tests, config-5 fixture
# through the timed path), then a same-box A/B of GSGPU_LIST_CLOSE on configs 5, 4 and 3.
set -u
TAG=${1:-r04_list}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_listclose.py \
  tests/test_gpu_parity.py -k "listclose or list_close or c5 or random_streams or baseline_config or emit_delta or streams_golden" \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -20; exit 3; }
timeout -k 10 300 python -u tests/headline_check.py --fixture c5 --fold-windows --chunk 256 > "$OUT/c5fix.json" 2> "$OUT/c5fix.err"
rc=$?; echo "c5fix rc=$rc"; tail -1 "$OUT/c5fix.json" | cut -c1-200; [ $rc -eq 0 ] || { tail -5 "$OUT/c5fix.err"; exit 3; }
for wl in c5 c4 c3; do
for i in 1 2; do
  for v in 1 0; do
    GSGPU_LIST_CLOSE=$v timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --no-cpu-baseline > "$OUT/b_${wl}_${v}_$i.json" 2> "$OUT/b_${wl}_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_${wl}_${v}_$i.err"; exit 3; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/b_${wl}_${v}_$i.json') if l.startswith('{')][-1]); k=d.get('kernels') or {}; print('$wl LIST=$v run $i: %.3f G edges/s, %.3f ms/step, p50 %s, close/window %s' % (d['value']/1e9, d['ms_per_step'], (d.get('window_latency') or {}).get('p50_us'), k.get('compress_ms_per_window')))"
  done
done
done
exit 0
