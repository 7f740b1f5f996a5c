#!/bin/bash
# Round 5, box 2: the split fold with one survivor per union thread — parity (variant_check, ring
# from 2^20 ids), then the headline with the run-ahead on (1), off (0) and split-but-serialised (2);
# the 8-rank per-rank window (2^21 edges) through the exchange at world 1, on/off; the config-2 A/B
# of the round-3 library against HEAD.
set -u
TAG=${1:-r05_run2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
show() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); r=d['roofline']; print('$2: %.3f G edges/s %.3f ms/step kernel %s avg %.4f ms split %s' % (d['value']/1e9, d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r.get('split')))"; }
GSGPU_RING_MIN_BITS=20 timeout -k 10 300 python -u tests/variant_check.py > "$OUT/variant.json" 2> "$OUT/variant.err"
rc=$?; echo "variant rc=$rc"; python -c "import json; d=json.loads(open('$OUT/variant.json').read().splitlines()[-1]); print('variant ok', d['ok'])"
[ $rc -eq 0 ] || { tail -5 "$OUT/variant.err"; exit 3; }
for v in 1 0 2; do
  GSGPU_RUN_AHEAD=$v timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$v.err"; exit 3; }
  show "$OUT/bench_$v.json" "head run_ahead=$v"
done
for v in 1 0; do
  GSGPU_RUN_AHEAD=$v timeout -k 10 300 python -u bench.py --window-log2 21 --exchange-world1 --steps 3 --no-cpu-baseline > "$OUT/w21_$v.json" 2> "$OUT/w21_$v.err"
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/w21_$v.err"; exit 3; }
  show "$OUT/w21_$v.json" "w21 xchg1 run_ahead=$v"
  python -c "import json; d=json.loads([l for l in open('$OUT/w21_$v.json') if l.startswith('{')][-1]); print('   per window %.1f us' % (d['ms_per_step']/d['config']['windows']*1e3))"
done
OLD=$GRAFT_REPO_ROOT/_ab/r03/libgsgpu.so
for i in 1 2 3; do
  for v in head r03; do
    if [ $v = r03 ]; then export GSGPU_LIB=$OLD; else unset GSGPU_LIB; fi
    timeout -k 10 300 python -u bench.py --workload c2 --steps 10 --no-cpu-baseline > "$OUT/c2_${v}_$i.json" 2> "$OUT/c2_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/c2_${v}_$i.err"; exit 3; }
    python -c "import json; d=json.loads([l for l in open('$OUT/c2_${v}_$i.json') if l.startswith('{')][-1]); print('c2 $v $i: %.3f G edges/s %.4f ms/step' % (d['value']/1e9, d['ms_per_step']))"
  done
done
unset GSGPU_LIB
exit 0
