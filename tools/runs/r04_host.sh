#!/bin/bash
# A/B: gs_cc_fold_windows checking the buffers once per call (current) vs once per window (libgsgpu_pre)
set -u
TAG=${1:-r04_host}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/gelly-streaming_amd/gsgpu/lib/exp
for i in 1 2 3; do
  for v in cur pre; do
    unset GSGPU_LIB; [ $v = pre ] && export GSGPU_LIB=$L/libgsgpu_pre.so
    timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --no-cpu-baseline > "$OUT/b_${v}_$i.json" 2> "$OUT/b_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_${v}_$i.err"; exit 3; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/b_${v}_$i.json') if l.startswith('{')][-1]); print('c5 $v run $i: %.3f G edges/s, %.3f ms/step, p50 %.1f' % (d['value']/1e9, d['ms_per_step'], (d.get('window_latency') or {}).get('p50_us')))"
  done
done
unset GSGPU_LIB
exit 0
