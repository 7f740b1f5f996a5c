#!/bin/bash
# A/B of an experiment build against production on configs 2/4/5 and the headline (bench lines,
# alternating). usage: bash tools/r03_ygrid.sh <tag> <lib>
set -u
TAG=${1:-r03_ygrid}; LIB=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
  for w in c2 c4 c5 c3; do
    for v in prod exp; do
      if [ $v = exp ]; then E="GSGPU_LIB=$PWD/$LIB"; else E=""; fi
      env $E timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > $OUT/${w}_${v}_$rep.json 2> $OUT/${w}_${v}_$rep.err || { tail -n 5 $OUT/${w}_${v}_$rep.err; exit 3; }
      echo "$w $v $rep $(grep -o '"ms_per_step": [0-9.]*' $OUT/${w}_${v}_$rep.json)"
    done
  done
done
