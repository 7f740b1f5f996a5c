#!/bin/bash
# Extra bench lines on the GPU box (int64 ids, pinned-host input, single window) + the per-window
# profile of the headline stream: bash tools/lines_run.sh <tag>
set -u
TAG=${1:-r02}
OUT=gpurun_out/$TAG/lines
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err"
  local rc=$?
  echo "$n rc=$rc"; cut -c1-300 "$OUT/bench_$n.json"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/bench_$n.err"; exit 3; fi
}
run int64 --id-bits 64 --steps 3 --no-cpu-baseline
run host --host-input --steps 3 --no-cpu-baseline
run host_int64 --host-input --id-bits 64 --steps 2 --no-cpu-baseline
run single --workload c3_single --steps 3 --no-cpu-baseline
timeout -k 10 300 python -u tools/window_profile.py > "$OUT/window_profile.txt" 2>&1 || { tail -5 "$OUT/window_profile.txt"; exit 3; }
head -14 "$OUT/window_profile.txt"
