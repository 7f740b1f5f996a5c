#!/bin/bash
# Round-4: parity of the hooked-root close (config 2/4 per window, variants, golden streams) and the
# config-4 / config-5 / headline bench lines. usage: bash tools/r04_hb.sh <tag>
set -u
TAG=${1:-r04_hb}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_variants.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "baseline_config or c5_small or random_streams or variant_parity or streams_golden or full_size or c5_config" \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 3
for w in c4 c5 c3; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$w.err"; exit 3; }
  python -c "import json; d=json.loads([l for l in open('$OUT/bench_$w.json') if l.startswith('{')][-1]); print('$w: %.3f G edges/s, %.3f ms/step, close %.1f us/window, fixture %s' % (d['value']/1e9, d['ms_per_step'], d['kernels']['compress_ms_per_window']*1e3, (d.get('final_checksum_vs_fixture') or {}).get('match')))"
done
exit 0
