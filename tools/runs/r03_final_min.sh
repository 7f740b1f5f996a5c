#!/bin/bash
# The minimum evidence for a changed library (GPU box, repo root): the whole GPU suite, smoke, the
# headline PMC passes (refreshes fold_traffic.json for these sources), one headline bench line.
# usage: bash tools/r03_final_min.sh <tag>
set -u
TAG=${1:-r03_min}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $OUT/smoke.log)"; [ $rc -eq 0 ] || exit 3
bash tools/pmc_traffic.sh "$TAG" > "$OUT/pmc.out" 2>&1 || { echo "pmc failed"; tail -5 "$OUT/pmc.out"; exit 3; }
echo "pmc ok"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc $(cut -c1-200 $OUT/bench.json)"; [ $rc -eq 0 ] || exit 3
exit 0
