#!/bin/bash
# Round 5, box 5: the whole GPU suite on the current sources, smoke, the headline and config-4 lines
# (the full-pass close's rename shortcut), and the barrier lab with leaders-only fences.
set -u
TAG=${1:-r05_run5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|137|134|139|143) return 0;; *) return 1;; esac; }
faulted() { grep -qE "illegal memory access|hipErrorIllegalAddress|Memory access fault|HSA_STATUS_ERROR" "$@" 2>/dev/null; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
if fatal $rc || faulted "$OUT/pytest_gpu.log"; then exit 3; fi
[ $rc -eq 0 ] || { grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head; exit 3; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit 3
for wl in c3 c4; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --no-cpu-baseline > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err"
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$wl.err"; exit 3; }
  python -c "import json; d=json.loads([l for l in open('$OUT/bench_$wl.json') if l.startswith('{')][-1]); print('$wl: %.3f G edges/s %.3f ms/step compress_ms/window %.4f' % (d['value']/1e9, d['ms_per_step'], d['kernels']['compress_ms_per_window']))"
done
timeout -k 10 300 python -u tools/window_profile.py > "$OUT/wp.txt" 2> "$OUT/wp.err"; echo "wp rc=$?"; head -6 "$OUT/wp.txt"; tail -1 "$OUT/wp.txt"
timeout -k 10 120 ./tools/barrier_lab 2000 > "$OUT/barrier_lab.json" 2> "$OUT/barrier_lab.err"
echo "barrier rc=$?"; cat "$OUT/barrier_lab.json"
exit 0
