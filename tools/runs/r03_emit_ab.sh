#!/bin/bash
# Async delta emission A/B (GPU box): delta GPU tests, then --emit-host lines with 4 / 16 / 64
# copy-out workgroups and the blocking call, a kernel trace of the default. usage: bash tools/r03_emit_ab.sh <tag>
set -u
TAG=${1:-r03_emit_ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "emit_delta or emit_pairs or pairs" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 3
for B in 4 16 64; do
  GSGPU_EMIT_COPY_BLOCKS=$B timeout -k 10 300 python -u bench.py --emit-host --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_b$B.json" 2> "$OUT/bench_b$B.err"
  rc=$?; echo "blocks $B: $(tail -1 "$OUT/bench_b$B.json" | cut -c90-200)"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_b$B.err"; exit 3; }
done
timeout -k 10 300 python -u bench.py --emit-host --emit-sync --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_sync.json" 2> "$OUT/bench_sync.err"
rc=$?; echo "sync: $(tail -1 "$OUT/bench_sync.json" | cut -c90-200)"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_sync.err"; exit 3; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --emit-host --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/prof.log"; exit 3; }
exit 0
