#!/bin/bash
# Close A/B (GPU box): headline parity (64 windows, 2 passes), the GPU tests that exercise closes
# (parity configs, variants, comm), the headline bench and its per-window profile, and the 2^21-edge
# window with the exchange. usage: bash tools/r03_close.sh <tag>
set -u
TAG=${1:-r03_close}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { case "$1" in 0) return 1;; *) return 0;; esac; }
timeout -k 10 300 python -u tests/headline_check.py --steps 2 > "$OUT/headline.json" 2> "$OUT/headline.err"
rc=$?; echo "headline rc=$rc"; cut -c1-300 "$OUT/headline.json"; tail -2 "$OUT/headline.err"
if stop $rc; then exit 3; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_variants.py tests/test_gpu_comm.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"
if stop $rc; then exit 3; fi
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc $(grep -o '"value": [0-9.e+]*' "$OUT/bench.json") $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench.json")"
if stop $rc; then exit 3; fi
timeout -k 10 300 python -u tools/window_profile.py > "$OUT/window_profile.txt" 2>&1
rc=$?; tail -1 "$OUT/window_profile.txt"; if stop $rc; then exit 3; fi
timeout -k 10 300 python -u bench.py --window-log2 21 --exchange-world1 --steps 3 --no-cpu-baseline > "$OUT/bench_xchg1_w21.json" 2> "$OUT/bench_xchg1_w21.err"
rc=$?; echo "xchg1 w21 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_xchg1_w21.json")"
if stop $rc; then exit 3; fi
timeout -k 10 300 python -u bench.py --window-log2 21 --steps 3 --no-cpu-baseline > "$OUT/bench_w21.json" 2> "$OUT/bench_w21.err"
rc=$?; echo "w21 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_w21.json")"
if stop $rc; then exit 3; fi
for w in c4 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  rc=$?; echo "$w rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_$w.json")"; if stop $rc; then exit 3; fi
done
exit 0
