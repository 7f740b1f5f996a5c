#!/bin/bash
# the row tests, the parse and bip bench lines, and their kernel stats
set -u
TAG=${1:-r04_rows}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rows.py \
  tests/test_gpu_bipartite.py tests/test_gpu_parity.py -k "rows or bip or parse" > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -20; exit 3; }
for w in parse bip; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 5 > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  rc=$?; echo "bench $w rc=$rc $(cut -c1-400 $OUT/bench_$w.json)"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$w.err"; exit 3; }
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_$w" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --workload $w --steps 2 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof_$w.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof $w rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/prof_$w.log"; exit 3; }
done
exit 0
