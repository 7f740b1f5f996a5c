#!/bin/bash
# Round 5: k_fold_ring's dynamic tail (GSGPU_RING_DYN=rounds,chunk) — parity variants, then the
# headline (2^24-edge windows) and 2^21-edge windows for several settings, same box.
set -u
OUT=gpurun_out/r05_dyn
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py -k "ring_dyn or production" -x -v --timeout 500 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 3
for wl in 24 21; do
  for dyn in "" 1,1 2,1 2,2 4,2 4,4 ""; do
    GSGPU_RING_DYN=$dyn timeout -k 10 300 python -u bench.py --workload c3 --window-log2 $wl --steps 6 --warmup 1 \
        --no-cpu-baseline > "$OUT/b.json" 2> "$OUT/b.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b.err"; exit 3; }
    python -c "import json; d=json.loads([l for l in open('$OUT/b.json') if l.startswith('{')][-1]); print('w$wl dyn=[$dyn] %.3f G edges/s %.3f ms/step ring_us %.1f' % (d['value']/1e9, d['ms_per_step'], d['roofline']['avg_launch_ms']*1e3))" | tee -a "$OUT/summary.txt"
  done
done
exit 0
