#!/bin/bash
# Round 5 experiment: window 1's edges bucketed by the top K bits of src before the young fold
# (GSGPU_YOUNG_SORT=K) — parity (variant checker), then the headline alternated on one box.
set -u
OUT=gpurun_out/r05_ysort
mkdir -p "$OUT"
export TMPDIR=/tmp
GSGPU_YOUNG_SORT=8 GSGPU_RING_MIN_BITS=20 timeout -k 10 600 python -u tests/variant_check.py > "$OUT/variant.json" 2> "$OUT/variant.err"
rc=$?; echo "variant rc=$rc"; python -c "
import json; d=json.loads([l for l in open('$OUT/variant.json') if l.startswith('{')][-1]); print('ok', d['ok']); [print(c) for c in d['cases'] if not c['ok']]"
[ $rc -eq 0 ] || exit 3
for i in 1 2 3; do
  for v in 0 8 12; do
    GSGPU_YOUNG_SORT=$v timeout -k 10 300 python -u bench.py --steps 8 --no-cpu-baseline > "$OUT/b_$v.json" 2> "$OUT/b_$v.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_$v.err"; exit 3; }
    python -c "import json; d=json.loads([l for l in open('$OUT/b_$v.json') if l.startswith('{')][-1]); print('sort=$v run $i: %.3f G edges/s %.3f ms/step fixture %s' % (d['value']/1e9, d['ms_per_step'], d['final_checksum_vs_fixture']['match']))" | tee -a "$OUT/summary.txt"
  done
done
GSGPU_YOUNG_SORT=8 timeout -k 10 300 python -u tools/window_profile.py > "$OUT/wp8.txt" 2>&1; head -2 "$OUT/wp8.txt"
exit 0
