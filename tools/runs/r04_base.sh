#!/bin/bash
# Round-4 baseline (GPU box, repo root): bench lines of the headline and configs 4 / 5, a per-window
# fold profile of the headline and a kernel-stats run. Every GPU step has its own limit; a failure
# stops the script. usage: bash tools/r04_base.sh <tag>
set -u
TAG=${1:-r04_base}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc"; tail -1 "$OUT/$name.json" | cut -c1-400
  [ $rc -eq 0 ] || { tail -5 "$OUT/$name.err"; exit 3; }
}
run c5fix 600 python -u tests/headline_check.py --fixture c5 --fold-windows --chunk 256
run c3fw 600 python -u tests/headline_check.py --fold-windows --no-torch --steps 0
run bench_c3 300 python -u bench.py --steps 5 --no-cpu-baseline
run bench_c5 300 python -u bench.py --workload c5 --steps 3 --no-cpu-baseline
run bench_c4 300 python -u bench.py --workload c4 --steps 3 --no-cpu-baseline
run wprof 300 python -u tools/window_profile.py
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/prof.log"; exit 3; }
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -16
exit 0
