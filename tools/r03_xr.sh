#!/bin/bash
# XCD-sliced tail (xtail.hpp) on the GPU box, repo root: request lab (XCD-sliced lookups), headline
# parity under the forced xr fold, variant parity, then a same-box A/B of one bench step under
# rocprofv3 --kernel-trace: ring (production), xr, and the NOGBITS timing lab (wrong results on
# purpose: the ring fold without its gbits loads). Every GPU step has its own limit; a failure
# stops the script. usage: bash tools/r03_xr.sh <tag>
set -u
TAG=${1:-r03_xr}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
true

GSGPU_FOLD_MODE=xr timeout -k 10 300 python -u tests/headline_check.py --no-torch --variant > "$OUT/headline_xr.json" 2> "$OUT/headline_xr.err"
rc=$?; echo "headline xr rc=$rc"; cut -c1-600 "$OUT/headline_xr.json"; tail -3 "$OUT/headline_xr.err"
[ $rc -eq 0 ] || exit 3
GSGPU_FOLD_MODE=xr timeout -k 10 300 python -u tests/variant_check.py > "$OUT/variant_xr.json" 2> "$OUT/variant_xr.err"
rc=$?; echo "variant xr rc=$rc"; cut -c1-400 "$OUT/variant_xr.json"; tail -3 "$OUT/variant_xr.err"
[ $rc -eq 0 ] || exit 3
bash tools/r03_ab.sh "$TAG/ab" - GSGPU_FOLD_MODE=xr GSGPU_LIB=$PWD/gelly-streaming_amd/gsgpu/lib/exp/libgsgpu_NOGBITS.so
exit $?
