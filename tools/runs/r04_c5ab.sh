#!/bin/bash
# config-5 A/B of GSGPU_LIST_CLOSE, 4 alternations
set -u
TAG=${1:-r04_c5ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2 3 4; do
  for v in 1 0; do
    GSGPU_LIST_CLOSE=$v timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --no-cpu-baseline > "$OUT/b_${v}_$i.json" 2> "$OUT/b_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_${v}_$i.err"; exit 3; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/b_${v}_$i.json') if l.startswith('{')][-1]); k=d.get('kernels') or {}; print('c5 LIST=$v run $i: %.3f G edges/s, %.3f ms/step, p50 %.1f, close/window %.4f' % (d['value']/1e9, d['ms_per_step'], (d.get('window_latency') or {}).get('p50_us'), k.get('compress_ms_per_window')))"
  done
done
exit 0
