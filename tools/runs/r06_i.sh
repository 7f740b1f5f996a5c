#!/bin/bash
# Round 6: config 4 A/B, same box, alternated: the product library (A), one edge per thread for
# plain folds up to 2^20 edges (B: GSGPU_SMALL_FOLD), nontemporal parent[] loads in the full-pass
# close (C: abl/libgsgpu_NTPAR.so, -DGS_EXP_NTPAR), both (D); then the headline A vs C.
set -u
TAG=${1:-r06_i}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
NT=$PWD/abl/libgsgpu_NTPAR.so
run() {  # name workload steps env...
  local name=$1 wl=$2 steps=$3; shift 3
  env "$@" timeout -k 10 300 python -u bench.py --workload $wl --steps $steps --no-cpu-baseline > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 "$OUT/$name.err"; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));k=d.get('kernels',{});print('$name: %.3f G edges/s  %.3f ms/step  close %.1f us/window' % (d['value']/1e9, d['ms_per_step'], 1000*k.get('compress_ms_per_window',0)), d.get('final_checksum_vs_fixture',''))"
}
for rep in 1 2 3; do
  run c4_A_$rep c4 5 X=1
  run c4_B_$rep c4 5 GSGPU_SMALL_FOLD=1048576
  run c4_C_$rep c4 5 GSGPU_LIB=$NT
  run c4_D_$rep c4 5 GSGPU_LIB=$NT GSGPU_SMALL_FOLD=1048576
done
for rep in 1 2; do
  run hl_A_$rep c3 3 X=1
  run hl_C_$rep c3 3 GSGPU_LIB=$NT
done
exit 0
