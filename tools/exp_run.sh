#!/bin/bash
# A/B of experiment builds (make -C gelly-streaming_amd exp EXP=NAME) against the product library:
# the per-window profile of the headline stream per variant, alternating twice.
# usage (repo root, GPU box): bash tools/exp_run.sh <tag> [windows]
set -u
shopt -s nullglob
TAG=${1:-r02}; NW=${2:-40}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG/exp
mkdir -p "$OUT"
for rep in 1 2; do
  for L in gelly-streaming_amd/gsgpu/lib/libgsgpu.so gelly-streaming_amd/gsgpu/lib/exp/libgsgpu_*.so; do
    n=$(basename "$L" .so)
    GSGPU_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python -u tools/window_profile.py $NW > "$OUT/wp_${n}_$rep.txt" 2>&1 || { tail -5 "$OUT/wp_${n}_$rep.txt"; exit 3; }
    echo "$n rep $rep: $(grep summary "$OUT/wp_${n}_$rep.txt")"
  done
done
