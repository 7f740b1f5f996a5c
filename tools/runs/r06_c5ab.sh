#!/bin/bash
# Round 6: config-5 regression, same box, alternated: the round-3 tree (c3fa4c6), the round-4 tree
# (b6012cd) and HEAD, 4 runs each: bench.py --workload c5 (throughput + per-window latency).
set -u
TAG=${1:-r06_c5ab}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2 3 4; do
  for t in r03 r04 head; do
    if [ $t = head ]; then d=$GRAFT_REPO_ROOT; else d=$GRAFT_REPO_ROOT/abtrees/$t; fi
    (cd $d && timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --no-cpu-baseline > "$OUT/c5_${t}_$rep.json" 2> "$OUT/c5_${t}_$rep.err")
    rc=$?; [ $rc -eq 0 ] || { echo "$t rep $rep rc=$rc"; tail -5 "$OUT/c5_${t}_$rep.err"; exit 3; }
    python3 -c "import json;d=json.load(open('$OUT/c5_${t}_$rep.json'));l=d.get('window_latency') or {};print('$t rep $rep: %.3f G edges/s  p50 %.1f us  p99 %.1f us' % (d['value']/1e9, l.get('p50_us',0), l.get('p99_us',0)))"
  done
done
exit 0
