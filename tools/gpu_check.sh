#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace. Each GPU step has
# its own time limit; a timeout / kill / abort / segfault stops the script (no further GPU use).
# Usage (from the repo root on the box): bash tools/gpu_check.sh [tag] [bench args...]
set -u
TAG=${1:-r01}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|137|134|139|143) return 0;; *) return 1;; esac; }
# a device fault surfaces as a Python exception (rc 1): stop on it too
faulted() { grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault|HSA_STATUS_ERROR" "$@" 2>/dev/null; }

timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
if fatal $rc || faulted "$OUT/pytest_gpu.log"; then echo "fatal in tests"; exit 3; fi

timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
if fatal $rc || faulted "$OUT/smoke.log"; then exit 3; fi

timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
if [ $rc -ne 0 ]; then exit 3; fi

cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/$OUT/prof.log"
exit 0
