#!/bin/bash
# Round 5, first box: (1) parity of the run-ahead filter pipeline (variant_check with the ring fold
# from 2^20 ids, on and off; the headline's gs_cc_fold_windows path vs the fixture), the list-close
# switch and torch-stream ordering tests; (2) the headline with the pipeline on/off, alternated;
# (3) the config-2 same-box A/B of the round-3 library (sources 82aa4c2d, commit 6698b9d, built into
# _ab/r03/) against HEAD, alternated, 4 runs each.
set -u
TAG=${1:-r05_run1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|137|134|139|143) return 0;; *) return 1;; esac; }
faulted() { grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault|HSA_STATUS_ERROR" "$@" 2>/dev/null; }

for v in on off; do
  if [ $v = off ]; then export GSGPU_RUN_AHEAD=0; fi
  GSGPU_RING_MIN_BITS=20 timeout -k 10 300 python -u tests/variant_check.py > "$OUT/variant_$v.json" 2> "$OUT/variant_$v.err"
  rc=$?; unset GSGPU_RUN_AHEAD; echo "variant $v rc=$rc"; tail -c 600 "$OUT/variant_$v.json"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/variant_$v.err"; exit 3; fi
done

timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  "tests/test_gpu_variants.py::test_headline_config_production[fold_windows]" tests/test_gpu_listclose.py \
  "tests/test_gpu_variants.py::test_list_close_switch" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
if fatal $rc || faulted "$OUT/pytest.log"; then exit 3; fi

for i in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export GSGPU_RUN_AHEAD=0; else unset GSGPU_RUN_AHEAD; fi
    timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > "$OUT/bench_${v}_$i.json" 2> "$OUT/bench_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_${v}_$i.err"; exit 3; }
    python -c "import json; d=json.loads([l for l in open('$OUT/bench_${v}_$i.json') if l.startswith('{')][-1]); print('head $v $i: %.3f G edges/s %.3f ms/step frac %.4f match %s' % (d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['final_checksum_vs_fixture']['match']))"
  done
done
unset GSGPU_RUN_AHEAD

OLD=$GRAFT_REPO_ROOT/_ab/r03/libgsgpu.so
for i in 1 2 3 4; do
  for v in head r03; do
    if [ $v = r03 ]; then export GSGPU_LIB=$OLD; else unset GSGPU_LIB; fi
    timeout -k 10 300 python -u bench.py --workload c2 --steps 10 --no-cpu-baseline > "$OUT/c2_${v}_$i.json" 2> "$OUT/c2_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/c2_${v}_$i.err"; exit 3; }
    python -c "import json; d=json.loads([l for l in open('$OUT/c2_${v}_$i.json') if l.startswith('{')][-1]); print('c2 $v $i: %.3f G edges/s %.4f ms/step' % (d['value']/1e9, d['ms_per_step']))"
  done
done
unset GSGPU_LIB
exit 0
