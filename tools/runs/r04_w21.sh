#!/bin/bash
# Round-4: the 8-rank strong layout's per-rank window (2^21 edges of RMAT-26) on one GPU, with and
# without the C-ABI exchange at world 1, plus a kernel trace of the exchange line.
# usage: bash tools/r04_w21.sh <tag>
set -u
TAG=${1:-r04_w21}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc"; tail -1 "$OUT/$name.json" | cut -c1-300
  [ $rc -eq 0 ] || { tail -5 "$OUT/$name.err"; exit 3; }
}
run w21 300 python -u bench.py --window-log2 21 --steps 3 --no-cpu-baseline
run w21x_allgather 300 python -u bench.py --window-log2 21 --steps 3 --no-cpu-baseline --exchange-world1 --merge allgather
run w21x_gather 300 python -u bench.py --window-log2 21 --steps 3 --no-cpu-baseline --exchange-world1 --merge gather
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --window-log2 21 --steps 1 --warmup 1 --no-cpu-baseline --exchange-world1 > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/prof.log"; exit 3; }
exit 0
