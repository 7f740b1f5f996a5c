#!/bin/bash
# gs_parse_edges A/B: the parse parity tests on the current library, then bench --workload parse
# alternated between it and the library built before the change (gsgpu/lib/exp/libgsgpu_base.so)
set -u
TAG=${1:-r04_parse_ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_rows.py -k "parse" -v > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -20; exit 3; }
BASE=$GRAFT_REPO_ROOT/gelly-streaming_amd/gsgpu/lib/exp/libgsgpu_base.so
for i in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then export GSGPU_LIB=$BASE; else unset GSGPU_LIB; fi
    timeout -k 10 300 python -u bench.py --workload parse --steps 20 --no-cpu-baseline > "$OUT/b_${v}_$i.json" 2> "$OUT/b_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_${v}_$i.err"; exit 3; }
    python -c "import json; d=json.loads([l for l in open('$OUT/b_${v}_$i.json') if l.startswith('{')][-1]); print('$v $i parse: %.2f G lines/s %.4f ms/call ok=%s' % (d['value']/1e9, d['ms_per_step'], d['verify']['equal_to_generated_ids']))"
  done
done
unset GSGPU_LIB
exit 0
