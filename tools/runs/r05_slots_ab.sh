#!/bin/bash
# Round 5: the slot fold (k_fold_slots) through the giant filter with claims — parity (exchange and
# prefilter tests), then rank 0's survivor-fold kernel time in the real 8-rank prefilter protocol
# (in-process, one GPU), the committed library (_var/base) alternated with the tree's.
set -u
OUT=gpurun_out/r05_slots
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_prefilter.py tests/test_gpu_comm.py tests/test_gpu_variants.py -k "prefilter or comm or ranks" -x -q \
    --timeout 850 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert" "$OUT/pytest.log" | head -20; exit 3; }
for i in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export GSGPU_LIB=$PWD/_var/base/libgsgpu.so; else unset GSGPU_LIB; fi
    timeout -k 10 300 python -u tools/prefilter_survivors.py 8 > "$OUT/p8_$v.out" 2> "$OUT/p8_$v.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/p8_$v.err"; exit 3; }
    echo "$v run $i: $(cat $OUT/p8_$v.out)" | tee -a "$OUT/summary.txt"
  done
done
unset GSGPU_LIB
exit 0
