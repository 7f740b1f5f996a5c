#!/bin/bash
# Round 5: survivors of the real prefilter protocol (stale broadcast bitmaps) at P = 2, 4, 8.
set -u
OUT=gpurun_out/r05_surv
mkdir -p "$OUT"
export TMPDIR=/tmp
for p in 2 4 8; do
  GSGPU_PREFILTER_LOG=1 timeout -k 10 300 python -u tools/prefilter_survivors.py $p > "$OUT/p$p.out" 2> "$OUT/p$p.err"
  rc=$?; echo "P=$p rc=$rc $(cat $OUT/p$p.out)"; [ $rc -eq 0 ] || { tail -5 "$OUT/p$p.err"; exit 3; }
  grep -c "survivors" "$OUT/p$p.err"
  awk '/survivors/ {s += $NF} END {print "total survivors", s}' "$OUT/p$p.err"
done
exit 0
