#!/bin/bash
# Round 6: the leaner Python per-window path (stream checks) — stream-order parity tests, config-5
# latency vs the round-3 tree (same box, alternated) — then the rank model at P = 8.
set -u
TAG=${1:-r06_d}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_listclose.py tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || { tail -30 "$OUT/pytest.log"; exit 3; }
for rep in 1 2 3; do
  for t in r03 head; do
    if [ $t = head ]; then d=$GRAFT_REPO_ROOT; else d=$GRAFT_REPO_ROOT/abtrees/$t; fi
    (cd $d && timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --no-cpu-baseline > "$OUT/c5_${t}_$rep.json" 2> "$OUT/c5_${t}_$rep.err")
    rc=$?; [ $rc -eq 0 ] || { echo "$t rep $rep rc=$rc"; tail -5 "$OUT/c5_${t}_$rep.err"; exit 3; }
    python3 -c "import json;d=json.load(open('$OUT/c5_${t}_$rep.json'));l=d.get('window_latency') or {};print('$t rep $rep: %.3f G edges/s  p50 %.1f us  p99 %.1f us' % (d['value']/1e9, l.get('p50_us',0), l.get('p99_us',0)))"
  done
done
bash tools/runs/r06_sim.sh $1_sim "8 21"
exit $?
