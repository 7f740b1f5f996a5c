#!/bin/bash
# Round 6: per-window full-label checks in the headline / c5 parity runs, and config 5's latency at
# the C ABI (csrc/host/cc_latency) beside bench.py's Python-driven line.
set -u
TAG=${1:-r06_h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_variants.py -k "headline_config_production or c5" -x -v -s --timeout 900 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || { tail -40 "$OUT/pytest.log"; exit 3; }
for i in 1 2; do
  timeout -k 10 300 gelly-streaming_amd/gsgpu/lib/cc_latency > "$OUT/cc_latency_$i.json" 2> "$OUT/cc_latency_$i.err"
  rc=$?; echo "cc_latency rc=$rc $(cat $OUT/cc_latency_$i.json)"; [ $rc -eq 0 ] || exit 3
  timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --no-cpu-baseline > "$OUT/bench_c5_$i.json" 2> "$OUT/bench_c5_$i.err"
  rc=$?; echo "bench c5 rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_c5_$i.json'));print('%.3f G'%(d['value']/1e9), d.get('window_latency',''))")"; [ $rc -eq 0 ] || exit 3
done
exit 0
