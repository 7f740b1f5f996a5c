#!/bin/bash
# Routed-fold timing lab (GPU box, repo root): parity of the production build, then kernel traces of
# one bench step under GSGPU_ROUTE_EXP knobs (wrong results on purpose: timing only).
# usage: bash tools/r03_route_lab.sh <tag> [exp values...]
set -u
TAG=${1:-r03_lab}; shift || true
EXPS=${@:-0}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tests/headline_check.py --no-torch > "$OUT/headline.json" 2> "$OUT/headline.err"
rc=$?; echo "headline rc=$rc"; cut -c1-300 "$OUT/headline.json"
if [ $rc -ne 0 ]; then tail -5 "$OUT/headline.err"; exit 3; fi
if [ -n "${RING_VARIANT:-}" ]; then
  GSGPU_RING_MIN_BITS=20 timeout -k 10 300 python -u tests/variant_check.py > "$OUT/variant_ring.json" 2> "$OUT/variant_ring.err"
  rc=$?; echo "variant ring rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/variant_ring.json'));print('ring variant ok', d['ok'], [c['case'] for c in d['cases'] if not c['ok']])"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/variant_ring.err"; exit 3; fi
fi
for E in $EXPS; do
  cd /tmp
  GSGPU_ROUTE_EXP=$E timeout -k 10 240 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/exp$E" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/exp$E.log" 2>&1
  rc=$?
  cd "$GRAFT_REPO_ROOT"
  echo "== GSGPU_ROUTE_EXP=$E rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/exp$E.log"; exit 3; fi
  f=$(find "$OUT/exp$E" -name "*kernel_trace.csv" | head -1)
  python3 tools/route_windows.py "$f" 13
  grep "\[route\]" "$OUT/exp$E.log" | tail -3
done
exit 0
