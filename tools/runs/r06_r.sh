#!/bin/bash
# Round 6: gs_bip_restore (literal snapshots loaded entry by entry; intended ones through the C ABI
# too): the bipartiteness GPU tests.
set -u
TAG=${1:-r06_r}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bipartite.py -x -v --timeout 600 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || { tail -40 "$OUT/pytest.log"; exit 3; }
exit 0
