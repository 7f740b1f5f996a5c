#!/bin/bash
# Is the per-window exchange loop (2^21-edge windows, allgather at world 1) host-bound? Kernel trace
# plus HIP API trace of a short run: the API call that enqueues each kernel vs the previous
# kernel's end on the GPU (tools/hosttrace.py reads the CSVs).
set -u
TAG=${1:-r04_hosttrace}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --window-log2 21 --exchange-world1 --steps 2 --warmup 1 --no-cpu-baseline \
  --no-fold-timing > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof rc=$rc"; tail -2 "$OUT/prof.log"; [ $rc -eq 0 ] || exit 3
timeout -k 10 120 python3 tools/hosttrace.py "$OUT/prof" 2500 > "$OUT/analysis.txt" 2>&1; echo "analysis rc=$?"
head -60 "$OUT/analysis.txt"
find "$OUT/prof" -name "*hip_api_trace.csv" -exec gzip {} \;
exit 0
