#!/bin/bash
# Per-window cost of the multi-GPU exchange path, measured on one GPU (GPU box, repo root): bench
# lines at the per-rank window of BASELINE config 3 on 8 GPUs (2^21 edges) and at 2^24, without and
# with the C-ABI exchange at world 1 (RCCL, one rank), and a kernel trace of the 2^21 exchange run.
# usage: bash tools/r03_xchg.sh <tag>
set -u
TAG=${1:-r03_xchg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err"
  local rc=$?
  echo "$n rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_$n.json")"
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/bench_$n.err"; exit 3; fi
}
run w21 --window-log2 21 --steps 3
run w21_xchg_allgather --window-log2 21 --steps 3 --exchange-world1 --merge allgather
run w21_xchg_gather --window-log2 21 --steps 3 --exchange-world1 --merge gather
run w21_xchg_tree --window-log2 21 --steps 3 --exchange-world1 --merge tree
run w24_xchg_allgather --steps 3 --exchange-world1 --merge allgather
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_w21x" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --window-log2 21 --steps 1 --warmup 1 --no-cpu-baseline --exchange-world1 \
  > "$GRAFT_REPO_ROOT/$OUT/prof_w21x.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -n 5 "$OUT/prof_w21x.log"; exit 3; }
f=$(find "$OUT/prof_w21x" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | head -14
exit 0
