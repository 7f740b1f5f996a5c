#!/bin/bash
# Round-6 fresh-box baseline of the committed library: the default bench line, the per-window
# profile and the config-5 line. usage (repo root, GPU box): bash tools/runs/r06_base.sh <tag>
set -u
TAG=${1:-r06_base}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc $(cut -c1-200 $OUT/bench.json)"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit 3; }
timeout -k 10 300 python -u tools/window_profile.py > "$OUT/window_profile.txt" 2> "$OUT/window_profile.err"
rc=$?; echo "wprof rc=$rc"; [ $rc -eq 0 ] || exit 3
for i in 1 2; do
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --no-cpu-baseline > "$OUT/bench_c5_$i.json" 2> "$OUT/bench_c5_$i.err"
rc=$?; echo "bench c5 rc=$rc $(cut -c1-200 $OUT/bench_c5_$i.json)"; [ $rc -eq 0 ] || exit 3
done
exit 0
