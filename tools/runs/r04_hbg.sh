#!/bin/bash
# Round-4 A/B: hooked-root marks with a giant (k_fold, GSGPU_HB_GIANT) for the incremental close;
# parity first (production defaults = marks on)
set -u
TAG=${1:-r04_hbg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_listclose.py \
  tests/test_gpu_parity.py -k "listclose or list_close or c5 or random_streams or baseline_config or emit_delta or streams_golden" \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -20; exit 3; }
for wl in c4 c2 c5; do
for i in 1 2; do
  for v in 1 0; do
    GSGPU_HB_GIANT=$v timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --no-cpu-baseline > "$OUT/b_${wl}_${v}_$i.json" 2> "$OUT/b_${wl}_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_${wl}_${v}_$i.err"; exit 3; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/b_${wl}_${v}_$i.json') if l.startswith('{')][-1]); k=d.get('kernels') or {}; print('$wl HB_GIANT=$v run $i: %.3f G edges/s, %.3f ms/step, fold_share %.3f close/window %.4f' % (d['value']/1e9, d['ms_per_step'], k.get('fold_share') or 0, k.get('compress_ms_per_window') or 0))"
  done
done
done
exit 0
