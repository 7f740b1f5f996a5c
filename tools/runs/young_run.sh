#!/bin/bash
# Young-window analysis on the GPU box: memory-operation throughputs (atomic_lab), per-window fold
# counters (GSGPU_FOLD_STATS) and the dispatch sequence of one 16-window step under rocprofv3.
# usage (repo root, GPU box): bash tools/young_run.sh <tag>
set -u
TAG=${1:-r02}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG/young
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 ./tools/atomic_lab > "$OUT/atomic_lab.json" 2>&1 || { cat "$OUT/atomic_lab.json"; exit 3; }
cat "$OUT/atomic_lab.json"
GSGPU_FOLD_STATS=1 timeout -k 10 300 python -u tools/window_profile.py 16 > "$OUT/stats.txt" 2>&1 || { tail -5 "$OUT/stats.txt"; exit 3; }
grep -c fold-stats "$OUT/stats.txt"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/window_profile.py" 16 > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 3; }
cd "$GRAFT_REPO_ROOT" && python3 tools/trace_seq.py $(ls "$OUT"/prof/*/run_kernel_trace.csv "$OUT"/prof/run_kernel_trace.csv 2>/dev/null | head -1) 120 > "$OUT/seq.txt" && head -60 "$OUT/seq.txt"
# experiment builds (make -C gelly-streaming_amd exp EXP=...): the same profile per variant
for L in gelly-streaming_amd/gsgpu/lib/exp/libgsgpu_*.so; do
  [ -e "$L" ] || continue
  n=$(basename "$L" .so)
  GSGPU_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python -u tools/window_profile.py 16 > "$OUT/wp_$n.txt" 2>&1 || { tail -5 "$OUT/wp_$n.txt"; exit 3; }
  echo "== $n"; head -14 "$OUT/wp_$n.txt"
done
