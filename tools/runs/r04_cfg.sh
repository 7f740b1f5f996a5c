#!/bin/bash
# Round-4 config lines (GPU box, repo root): bench of configs 2, 4, 5 and the headline, then a
# kernel trace of config 4. usage: bash tools/r04_cfg.sh <tag>
set -u
TAG=${1:-r04_cfg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in c4 c2 c5 c3; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$w.err"; exit 3; }
  python -c "import json; d=json.loads([l for l in open('$OUT/bench_$w.json') if l.startswith('{')][-1]); print('$w: %.3f G edges/s, %.3f ms/step, close %.1f us/window, fixture %s' % (d['value']/1e9, d['ms_per_step'], d['kernels']['compress_ms_per_window']*1e3, (d.get('final_checksum_vs_fixture') or {}).get('match')))"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_c4" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof_c4.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof c4 rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/prof_c4.log"; exit 3; }
exit 0
