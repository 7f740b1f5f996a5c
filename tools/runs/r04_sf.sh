#!/bin/bash
# Round-4 A/B: one edge per thread up to 2^20-edge folds (GSGPU_SMALL_FOLD=1048576) against the
# production 2^18, configs 2 and 4 (2^20-edge windows); parity of the variant on the config fixtures
set -u
TAG=${1:-r04_sf}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
GSGPU_SMALL_FOLD=1048576 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "baseline_config or random_streams" > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert" "$OUT/pytest.log" | head; exit 3; }
for wl in c2 c4; do
for i in 1 2; do
  for v in 1048576 262144; do
    GSGPU_SMALL_FOLD=$v timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --no-cpu-baseline > "$OUT/b_${wl}_${v}_$i.json" 2> "$OUT/b_${wl}_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_${wl}_${v}_$i.err"; exit 3; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/b_${wl}_${v}_$i.json') if l.startswith('{')][-1]); k=d.get('kernels') or {}; print('$wl SMALL_FOLD=$v run $i: %.3f G edges/s, %.3f ms/step, fold_share %s close/window %s' % (d['value']/1e9, d['ms_per_step'], k.get('fold_share'), k.get('compress_ms_per_window')))"
  done
done
done
exit 0
