#!/bin/bash
# Round 6: BipartitenessCheck reference-literal mode on the GPU (and the intended mode's suite).
set -u
TAG=${1:-r06_b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bipartite.py -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || { tail -60 "$OUT/pytest.log"; exit 3; }
exit 0
