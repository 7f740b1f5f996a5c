#!/bin/bash
# PMC passes over a short bench run (one pass per counter group, no trace domains combined with
# --pmc), then profiles/pmc_traffic.py folds them into per-window HBM bytes of k_fold.
# usage (repo root, GPU box): bash tools/pmc_traffic.sh <tag> [bench args]
set -u
TAG=${1:-r01}; shift || true
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_ATOMIC_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C -d "$OUT/p$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($C) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
cd "$GRAFT_REPO_ROOT" && python3 profiles/pmc_traffic.py "$OUT" > "$OUT/traffic.json" && cat "$OUT/traffic.json"
