#!/bin/bash
# Round 6: the young fold's chunk counter — K blockDim-group chunks per grab (GSGPU_YOUNG_CHUNKS):
# parity at K = 4, then a same-box alternated A/B of the headline (bench --steps 5) and window 1.
set -u
TAG=${1:-r06_m}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
GSGPU_YOUNG_CHUNKS=4 timeout -k 10 600 python -u tests/variant_check.py > "$OUT/variant_k4.json" 2> "$OUT/variant_k4.err"
rc=$?; echo "variant K=4 rc=$rc $(tail -c 300 $OUT/variant_k4.json)"; [ $rc -eq 0 ] || { tail -5 "$OUT/variant_k4.err"; exit 3; }
for rep in 1 2 3; do
  for k in 1 2 4 8; do
    GSGPU_YOUNG_CHUNKS=$k timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline > "$OUT/bench_k${k}_$rep.json" 2> "$OUT/bench_k${k}_$rep.err"
    rc=$?; echo "K=$k rep=$rep rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_k${k}_$rep.json'));print('%.2f G  %.3f ms  fixture %s'%(d['value']/1e9,d['ms_per_step'],d['final_checksum_vs_fixture']['match']))")"
    [ $rc -eq 0 ] || { tail -5 "$OUT/bench_k${k}_$rep.err"; exit 3; }
  done
done
for k in 1 4 1 4; do
  GSGPU_YOUNG_CHUNKS=$k timeout -k 10 300 python -u tools/window_profile.py 16 > "$OUT/wprof_k$k.txt" 2>&1
  rc=$?; echo "wprof K=$k rc=$rc $(head -1 $OUT/wprof_k$k.txt) | $(tail -1 $OUT/wprof_k$k.txt)"; [ $rc -eq 0 ] || exit 3
done
exit 0
