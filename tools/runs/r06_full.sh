#!/bin/bash
# Round 6: the whole GPU suite + smoke on the current tree (one process for the suite).
set -u
TAG=${1:-r06_full}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || { tail -40 "$OUT/pytest_gpu.log"; exit 3; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $OUT/smoke.log)"; [ $rc -eq 0 ] || exit 3
exit 0
