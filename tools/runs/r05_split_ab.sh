#!/bin/bash
# Round 5: the young split (GSGPU_YOUNG_SPLIT=0: none) on the headline, alternated on one box.
set -u
OUT=gpurun_out/r05_split
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in default 0; do
    if [ $v = default ]; then unset GSGPU_YOUNG_SPLIT; else export GSGPU_YOUNG_SPLIT=$v; fi
    timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > "$OUT/b_$v.json" 2> "$OUT/b_$v.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_$v.err"; exit 3; }
    python -c "import json; d=json.loads([l for l in open('$OUT/b_$v.json') if l.startswith('{')][-1]); print('split=$v run $i: %.3f G edges/s %.3f ms/step' % (d['value']/1e9, d['ms_per_step']))" | tee -a "$OUT/summary.txt"
  done
done
unset GSGPU_YOUNG_SPLIT
exit 0
