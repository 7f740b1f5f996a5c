#!/bin/bash
# Extra bench lines of the round-3 library (GPU box, repo root): int64 ids, pinned-host input (int32
# and int64), the stream as one window, per-window delta emission to the host, the exchange at
# world 1, then the headline's per-window profile. usage: bash tools/r03_lines.sh <tag>
set -u
TAG=${1:-r03_lines}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err"
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.e+]*' "$OUT/bench_$n.json") $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_$n.json")"
  if [ $rc -ne 0 ]; then tail -n 5 "$OUT/bench_$n.err"; exit 3; fi
}
run int64 --id-bits 64 --steps 3
run host --host-input --steps 3
run host_int64 --host-input --id-bits 64 --steps 2
run single --workload c3_single --steps 3
run emithost --emit-host --steps 2
run xchg1 --exchange-world1 --steps 3
timeout -k 10 300 python -u tools/window_profile.py > "$OUT/window_profile.txt" 2>&1 || { tail -n 5 "$OUT/window_profile.txt"; exit 3; }
tail -n 2 "$OUT/window_profile.txt"
exit 0
