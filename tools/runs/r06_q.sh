#!/bin/bash
# Round 6: the young fold's shape — workgroups per CU (GSGPU_YOUNG_BPC) x edges per thread
# (GSGPU_YOUNG_EPT), production 2 x 2: parity of two variants, then window 1 (window profiles) and the
# headline step, alternated on one box.
set -u
TAG=${1:-r06_q}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "2 1" "1 4"; do
  set -- $v
  GSGPU_YOUNG_BPC=$1 GSGPU_YOUNG_EPT=$2 timeout -k 10 600 python -u tests/variant_check.py > "$OUT/variant_$1x$2.json" 2> "$OUT/variant_$1x$2.err"
  rc=$?; echo "variant bpc=$1 ept=$2 rc=$rc ok=$(python3 -c "import json;print(json.load(open('$OUT/variant_$1x$2.json'))['ok'])")"; [ $rc -eq 0 ] || exit 3
done
for rep in 1 2; do
  for v in "2 2" "1 2" "3 2" "2 1" "4 1" "1 4"; do
    set -- $v
    GSGPU_YOUNG_BPC=$1 GSGPU_YOUNG_EPT=$2 timeout -k 10 300 python -u tools/window_profile.py 16 > "$OUT/wprof_$1x$2_$rep.txt" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "wprof $1x$2 rc=$rc"; exit 3; }
    GSGPU_YOUNG_BPC=$1 GSGPU_YOUNG_EPT=$2 timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline > "$OUT/bench_$1x$2_$rep.json" 2> "$OUT/bench_$1x$2_$rep.err"
    rc=$?; [ $rc -eq 0 ] || { echo "bench $1x$2 rc=$rc"; tail -3 "$OUT/bench_$1x$2_$rep.err"; exit 3; }
    echo "bpc=$1 ept=$2 rep=$rep $(head -1 $OUT/wprof_$1x$2_$rep.txt | grep -v amdgpu.ids) $(grep 'window   1 ' $OUT/wprof_$1x$2_$rep.txt) | $(python3 -c "import json;d=json.load(open('$OUT/bench_$1x$2_$rep.json'));print('%.2f G  %.3f ms  fixture %s'%(d['value']/1e9,d['ms_per_step'],d['final_checksum_vs_fixture']['match']))")"
  done
done
exit 0
