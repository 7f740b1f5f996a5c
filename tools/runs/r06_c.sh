#!/bin/bash
# Round 6: lazy smaller-root init (young folds) and the even-XCD ring tail — parity, then a
# same-box alternated A/B of the headline, window profiles, ring clocks.
set -u
TAG=${1:-r06_c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_variants.py -x -v --timeout 600 --timeout-method thread \
  -k "headline_config_production or c5_config_production or variant_parity" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || { tail -40 "$OUT/pytest.log"; exit 3; }
for rep in 1 2 3; do
  for cfg in "1 0" "0 0" "1 24" "1 40"; do
    set -- $cfg
    GSGPU_LAZY_LO=$1 GSGPU_RING_SKEW=$2 timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > "$OUT/bench_l$1_s$2_$rep.json" 2> "$OUT/bench_l$1_s$2_$rep.err"
    rc=$?; echo "lazy=$1 skew=$2 rep=$rep rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_l$1_s$2_$rep.json'));print('%.2f G  %.3f ms  ring %.1f us'%(d['value']/1e9,d['ms_per_step'],d['roofline']['avg_launch_ms']*1e3))")"
    [ $rc -eq 0 ] || exit 3
  done
done
for l in 0 1; do
  GSGPU_LAZY_LO=$l timeout -k 10 300 python -u tools/window_profile.py 16 > "$OUT/wprof_lazy$l.txt" 2>&1
  rc=$?; echo "wprof lazy=$l rc=$rc $(tail -1 $OUT/wprof_lazy$l.txt)"; [ $rc -eq 0 ] || exit 3
done
for sk in 0 24 40; do
  GSGPU_RING_CLOCKS=2 GSGPU_RING_SKEW=$sk timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/clocks_s$sk.json" 2> "$OUT/clocks_s$sk.err"
  rc=$?; echo "clocks skew=$sk rc=$rc"; [ $rc -eq 0 ] || exit 3
done
exit 0
