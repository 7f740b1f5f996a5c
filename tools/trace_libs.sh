#!/bin/bash
# rocprofv3 kernel trace of window_profile.py (8 windows) for the product library and every
# experiment build; prints the first young-window dispatches of the last rep per library.
# usage (repo root, GPU box): bash tools/trace_libs.sh <tag>
set -u
TAG=${1:-r02}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG/trace
mkdir -p "$OUT"
export TMPDIR=/tmp
for L in gelly-streaming_amd/gsgpu/lib/libgsgpu.so gelly-streaming_amd/gsgpu/lib/exp/libgsgpu_*.so; do
  n=$(basename "$L" .so)
  cd /tmp && GSGPU_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/$n" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/window_profile.py" 8 > "$OUT/$n.log" 2>&1 || { tail -5 "$OUT/$n.log"; exit 3; }
  cd "$GRAFT_REPO_ROOT"
  f=$(find "$OUT/$n" -name "*kernel_trace.csv" | head -1)
  echo "== $n"; python3 tools/trace_seq.py "$f" 40 | head -14
done
