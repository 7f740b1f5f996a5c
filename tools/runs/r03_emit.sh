#!/bin/bash
# Async delta emission (GPU box, repo root): the delta GPU tests, then the RMAT-26 --emit-host lines
# (async and the blocking call) and a kernel trace of the async line. usage: bash tools/r03_emit.sh <tag>
set -u
TAG=${1:-r03_emit}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "emit_delta" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -u bench.py --emit-host --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_async.json" 2> "$OUT/bench_async.err"
rc=$?; tail -1 "$OUT/bench_async.json" | cut -c1-200; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_async.err"; exit 3; }
timeout -k 10 300 python -u bench.py --emit-host --emit-sync --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_sync.json" 2> "$OUT/bench_sync.err"
rc=$?; tail -1 "$OUT/bench_sync.json" | cut -c1-200; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_sync.err"; exit 3; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --emit-host --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/prof.log"; exit 3; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | head -14
exit 0
