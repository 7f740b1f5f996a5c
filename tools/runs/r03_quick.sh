#!/bin/bash
# Round-3 quick look (GPU box, repo root): headline parity vs the 64-window fixture, variant
# parity (production), a short bench and a kernel trace. Every GPU step has its own limit; a fault,
# abort or timeout stops the script. usage: bash tools/r03_quick.sh <tag>
set -u
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { case "$1" in 0) return 1;; *) return 0;; esac; }
timeout -k 10 300 python -u tests/headline_check.py --steps 2 > "$OUT/headline.json" 2> "$OUT/headline.err"
rc=$?; echo "headline rc=$rc"; cat "$OUT/headline.json"; tail -4 "$OUT/headline.err"
if stop $rc; then exit 3; fi
timeout -k 10 300 python -u tests/variant_check.py > "$OUT/variant.json" 2> "$OUT/variant.err"
rc=$?; echo "variant rc=$rc"; cut -c1-400 "$OUT/variant.json"; tail -3 "$OUT/variant.err"
if stop $rc; then exit 3; fi
timeout -k 10 300 python -u bench.py --steps 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cut -c1-600 "$OUT/bench.json"; tail -3 "$OUT/bench.err"
if stop $rc; then exit 3; fi
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 "$GRAFT_REPO_ROOT/$OUT/prof.log"
f=$(find "$GRAFT_REPO_ROOT/$OUT/prof" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -16
exit 0
