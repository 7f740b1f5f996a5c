#!/bin/bash
# Round 5: per-workgroup phase clocks of k_fold_ring (GSGPU_FOLD_STATS=1) at 2^21- and 2^24-edge windows.
set -u
OUT=gpurun_out/r05_clocks
mkdir -p "$OUT"
export TMPDIR=/tmp
for wl in 21 24; do
  GSGPU_RING_CLOCKS=2 timeout -k 10 300 python -u bench.py --workload c3 --window-log2 $wl --steps 1 --warmup 0 \
      --no-cpu-baseline --no-fold-timing > "$OUT/w$wl.json" 2> "$OUT/w$wl.err"
  rc=$?; echo "w$wl rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/w$wl.err"; exit 3; }
  grep -c "ring-clocks" "$OUT/w$wl.err"
done
exit 0
