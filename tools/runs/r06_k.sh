#!/bin/bash
# Round 6: rank-model A/B of two Merger-side tweaks: (a) the young pair fold of >= capacity/16
# survivors skips the seen bitmap as the young SoA fold does (experiment build abl/libgsgpu_AOSSKIP.so),
# (b) only close 0's filter-state broadcast synchronous (SIM_SYNC=1). P = 8 and 4 (RMAT-26, 2^24 global).
set -u
TAG=${1:-r06_k}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for P in 8 4; do
  wl=$([ $P = 8 ] && echo 21 || echo 22)
  for v in base aos sync1 aos_sync1; do
    case $v in
      base) e="X=1";; aos) e="GSGPU_LIB=$PWD/abl/libgsgpu_AOSSKIP.so";; sync1) e="SIM_SYNC=1";;
      aos_sync1) e="GSGPU_LIB=$PWD/abl/libgsgpu_AOSSKIP.so SIM_SYNC=1";;
    esac
    env $e SIM_WLOG2=$wl timeout -k 10 600 python -u tools/sim_ranks.py $P 64 prefilter > "$OUT/sim_p${P}_$v.txt" 2>&1
    rc=$?; echo "P=$P $v rc=$rc $(grep TOTAL $OUT/sim_p${P}_$v.txt)"; [ $rc -eq 0 ] || { tail -5 "$OUT/sim_p${P}_$v.txt"; exit 3; }
    grep "^w  [1-5] " "$OUT/sim_p${P}_$v.txt"
  done
done
exit 0
