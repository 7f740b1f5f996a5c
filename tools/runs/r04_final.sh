#!/bin/bash
# Round-4 evidence for the library as committed (GPU box, repo root). Part "tests": the whole GPU
# suite and smoke. Part "evidence": the default bench line (as the driver runs it), a rocprofv3
# kernel-stats run of the same command, the PMC passes of the headline (fold_traffic.json for these
# sources), the per-window profile, and the config lines. Every GPU step has its own limit; a failure
# stops the script. usage: bash tools/r04_final.sh <tag> tests|evidence
set -u
TAG=${1:-r04_final}; PART=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$PART" = tests ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"; [ $rc -eq 0 ] || { tail -30 "$OUT/pytest_gpu.log"; exit 3; }
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc $(tail -1 $OUT/smoke.log)"; [ $rc -eq 0 ] || exit 3
  exit 0
fi
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc $(cut -c1-300 $OUT/bench.json)"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit 3; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/prof.log"; exit 3; }
bash tools/pmc_traffic.sh "$TAG" > "$OUT/pmc.out" 2>&1 || { echo "pmc failed"; tail -5 "$OUT/pmc.out"; exit 3; }
echo "pmc ok"
timeout -k 10 300 python -u tools/window_profile.py > "$OUT/window_profile.txt" 2> "$OUT/window_profile.err"
rc=$?; echo "wprof rc=$rc $(tail -1 $OUT/window_profile.txt)"; [ $rc -eq 0 ] || exit 3
for w in c2 c4 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  rc=$?; echo "bench $w rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$w.err"; exit 3; }
done
timeout -k 10 300 python -u bench.py --id-bits 64 --steps 3 --no-cpu-baseline > "$OUT/bench_int64.json" 2> "$OUT/bench_int64.err"
rc=$?; echo "bench int64 rc=$rc"; [ $rc -eq 0 ] || exit 3
exit 0
