#!/bin/bash
# 2^21-edge windows at RMAT-26 (the 8-rank per-rank window): ring vs plain fold, without and with
# the C-ABI exchange at world 1. usage: bash tools/r03_w21.sh <tag>
set -u
TAG=${1:-r03_w21}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for M in ring plain; do
  for X in "" "--exchange-world1"; do
    n=${M}${X:+_xchg1}
    GSGPU_FOLD_MODE=$M timeout -k 10 300 python -u bench.py --window-log2 21 --steps 3 --warmup 1 --no-cpu-baseline $X > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err"
    rc=$?; echo "$n rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$n.json'));print('%.2f G edges/s %.3f ms/step %.1f us/window'%(d['value']/1e9,d['ms_per_step'],d['ms_per_step']*1e3/d['config']['windows']))" 2>/dev/null)"
    [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$n.err"; exit 3; }
  done
done
exit 0
