#!/bin/bash
# A/B: workgroups of the close after the young window (a known full pass), GSGPU_FULL_GRID
set -u
TAG=${1:-r04_fullgrid}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
  for v in 0 4096 8192 16384; do
    GSGPU_FULL_GRID=$v timeout -k 10 300 python -u tools/window_profile.py > "$OUT/wp_${v}_$i.txt" 2> "$OUT/wp_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/wp_${v}_$i.err"; exit 3; }
    echo "grid $v run $i: $(head -1 $OUT/wp_${v}_$i.txt) | $(tail -1 $OUT/wp_${v}_$i.txt)"
  done
done
exit 0
