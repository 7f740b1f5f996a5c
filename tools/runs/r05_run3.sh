#!/bin/bash
# Round 5, box 3: streaming ingestion parity (tests/test_gpu_ingest.py, cc_example file mode), the
# two-level barrier lab, and a kernel trace of the 2^21-edge exchange window with the run-ahead
# filter on and off (does k_filter overlap the ordered chain?).
set -u
TAG=${1:-r05_run3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|137|134|139|143) return 0;; *) return 1;; esac; }
faulted() { grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault|HSA_STATUS_ERROR" "$@" 2>/dev/null; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ingest.py \
  "tests/test_gpu_parity.py::test_cc_example_file_input" "tests/test_gpu_parity.py::test_cc_example_builtin_stream" \
  -k "ingest or cc_example or parse" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
if fatal $rc || faulted "$OUT/pytest.log"; then exit 3; fi
timeout -k 10 120 ./tools/barrier_lab 2000 > "$OUT/barrier_lab.json" 2> "$OUT/barrier_lab.err"
rc=$?; echo "barrier rc=$rc"; cat "$OUT/barrier_lab.json"; [ $rc -eq 0 ] || { tail -3 "$OUT/barrier_lab.err"; exit 3; }
cd /tmp
for v in 1 0; do
  GSGPU_RUN_AHEAD=$v timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/trace_$v" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --window-log2 21 --exchange-world1 --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/trace_$v.log" 2>&1
  rc=$?; echo "trace $v rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$GRAFT_REPO_ROOT/$OUT/trace_$v.log"; exit 3; }
done
exit 0
