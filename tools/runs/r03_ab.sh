#!/bin/bash
# Same-box A/B of fold variants (GPU box, repo root): one bench step under rocprofv3 --kernel-trace
# per environment, then the steady windows' per-kernel means (tools/steady_windows.py).
# usage: bash tools/r03_ab.sh <tag> "ENV=1 ENV2=x" "..."   ("-" = production)
set -u
TAG=${1:-r03_ab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for ENVS in "$@"; do
  i=$((i+1))
  [ "$ENVS" = "-" ] && ENVS=""
  cd /tmp
  env $ENVS timeout -k 10 240 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/v$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/v$i.log" 2>&1
  rc=$?
  cd "$GRAFT_REPO_ROOT"
  echo "== v$i [$ENVS] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/v$i.log"; exit 3; fi
  grep -o '"ms_per_step": [0-9.]*' "$OUT/v$i.log" | head -1
  f=$(find "$OUT/v$i" -name "*kernel_trace.csv" | head -1)
  python3 tools/steady_windows.py "$f" 13
done
exit 0
