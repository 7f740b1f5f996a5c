#!/bin/bash
# Round-4 close-regression bisect: per-window profile with the round-start library, the list-close
# commit's library, the current one, and the current one without list buffers (GSGPU_NO_LISTS)
set -u
TAG=${1:-r04_bisect}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/gelly-streaming_amd/gsgpu/lib/exp
for i in 1 2; do
  for v in old 30b cur nolists; do
    unset GSGPU_LIB GSGPU_NO_LISTS
    case $v in old) export GSGPU_LIB=$L/libgsgpu_old.so;; 30b) export GSGPU_LIB=$L/libgsgpu_30b.so;; nolists) export GSGPU_NO_LISTS=1;; esac
    timeout -k 10 300 python -u tools/window_profile.py > "$OUT/wp_${v}_$i.txt" 2> "$OUT/wp_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/wp_${v}_$i.err"; exit 3; }
    echo "$v $i: $(tail -1 $OUT/wp_${v}_$i.txt)"
  done
done
exit 0
