#!/bin/bash
# Round 6: parity of the one-synchronous-broadcast schedule (kBcastSync = 1): the prefilter GPU tests,
# the 8-rank RMAT-26 layout in prefilter mode, the C++ mirror's prefilter check.
set -u
TAG=${1:-r06_l}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_prefilter.py tests/test_gpu_variants.py -x -v --timeout 900 --timeout-method thread \
  -k "prefilter" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || { tail -40 "$OUT/pytest.log"; exit 3; }
exit 0
