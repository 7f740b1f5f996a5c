#!/bin/bash
# Round 6: the ADVICE fixes on the GPU (prefilter empty slices / big slices, ingest staging error)
# plus the default bench line. usage: bash tools/runs/r06_a.sh <tag>
set -u
TAG=${1:-r06_a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_prefilter.py tests/test_gpu_ingest.py -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || { tail -40 "$OUT/pytest.log"; exit 3; }
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc $(cut -c1-160 $OUT/bench.json)"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit 3; }
exit 0
