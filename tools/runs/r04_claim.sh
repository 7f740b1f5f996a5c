#!/bin/bash
# Round-4 A/B: ring claims with (GSGPU_CLAIM_MARK=1, production) and without a mark bit. Parity of
# the unmarked variant first (headline + config-5 fixtures), then alternated benches.
set -u
TAG=${1:-r04_claim}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for fx in headline c5; do
  GSGPU_CLAIM_MARK=0 timeout -k 10 300 python -u tests/headline_check.py --fixture $fx --variant --fold-windows --chunk 256 > "$OUT/fix_$fx.json" 2> "$OUT/fix_$fx.err"
  rc=$?; echo "fixture $fx (no claim mark) rc=$rc"; tail -1 "$OUT/fix_$fx.json" | cut -c1-200; [ $rc -eq 0 ] || { tail -5 "$OUT/fix_$fx.err"; exit 3; }
done
for wl in c3 c5; do
for i in 1 2; do
  for v in 1 0; do
    GSGPU_CLAIM_MARK=$v timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --no-cpu-baseline > "$OUT/b_${wl}_${v}_$i.json" 2> "$OUT/b_${wl}_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_${wl}_${v}_$i.err"; exit 3; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/b_${wl}_${v}_$i.json') if l.startswith('{')][-1]); print('$wl CLAIM_MARK=$v run $i: %.3f G edges/s, %.3f ms/step, p50 %s' % (d['value']/1e9, d['ms_per_step'], (d.get('window_latency') or {}).get('p50_us')))"
  done
done
done
exit 0
