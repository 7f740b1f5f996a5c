#!/bin/bash
# Round-3 config evidence (GPU box, repo root): GPU parity of the parity configs and the variant
# streams, headline parity, then bench lines of configs 2, 4, 5 with a rocprofv3 kernel-stats run
# of each. Every GPU step has its own limit; a failure stops the script. usage: bash tools/r03_cfg.sh <tag>
set -u
TAG=${1:-r03_cfg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_variants.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "baseline_config or c5_small or random_streams or variant_parity or streams_golden or production" \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 3
for w in c2 c4 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  rc=$?; echo "bench $w rc=$rc"; tail -1 "$OUT/bench_$w.json" | cut -c1-300; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$w.err"; exit 3; }
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_$w" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --workload $w --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof_$w.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof $w rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/prof_$w.log"; exit 3; }
  f=$(find "$OUT/prof_$w" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | head -8
done
exit 0
