#!/bin/bash
# Round 6: k_fold_ring's per-XCD dynamic tail (GSGPU_RING_TAIL=rounds,chunk) — parity of the tail
# variants, then a same-box alternated A/B of the headline and per-XCD ring clocks.
set -u
TAG=${1:-r06_j}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_variants.py -x -v --timeout 600 --timeout-method thread \
  -k "variant_parity and (ring_tail or production)" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"; [ $rc -eq 0 ] || { tail -40 "$OUT/pytest.log"; exit 3; }
for rep in 1 2; do
  for t in 0 1,1 2,1 3,1 2,2 4,1; do
    GSGPU_RING_TAIL=$t timeout -k 10 300 python -u bench.py --steps 8 --no-cpu-baseline > "$OUT/bench_t${t}_$rep.json" 2> "$OUT/bench_t${t}_$rep.err"
    rc=$?; echo "tail=$t rep=$rep rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_t${t}_$rep.json'));print('%.2f G  %.3f ms  ring %.1f us  fixture %s'%(d['value']/1e9,d['ms_per_step'],d['roofline']['avg_launch_ms']*1e3,d['final_checksum_vs_fixture']['match']))")"
    [ $rc -eq 0 ] || { tail -5 "$OUT/bench_t${t}_$rep.err"; exit 3; }
  done
done
for t in 0 2,1; do
  GSGPU_RING_CLOCKS=2 GSGPU_RING_TAIL=$t timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/clocks_t$t.json" 2> "$OUT/clocks_t$t.err"
  rc=$?; echo "clocks tail=$t rc=$rc"; [ $rc -eq 0 ] || exit 3
  grep "ring-clocks\|ring-xcd" "$OUT/clocks_t$t.err" | tail -4
done
exit 0
