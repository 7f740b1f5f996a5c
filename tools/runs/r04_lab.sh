#!/bin/bash
# Round-4 labs (GPU box, repo root): window-boundary cost (tools/barrier_lab) and a kernel trace of
# BASELINE config 5. Every GPU step has its own limit. usage: bash tools/r04_lab.sh <tag>
set -u
TAG=${1:-r04_lab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 90 ./tools/barrier_lab 1000 > "$OUT/barrier_lab.json" 2> "$OUT/barrier_lab.err"
rc=$?; echo "barrier_lab rc=$rc"; cat "$OUT/barrier_lab.json"; tail -3 "$OUT/barrier_lab.err"; [ $rc -eq 0 ] || exit 3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_c5" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof_c5.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof c5 rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/prof_c5.log"; exit 3; }
exit 0
