#!/bin/bash
# full GPU check + PMC + per-window sweep + parity-config bench lines (GPU box): bash tools/v11_run.sh <tag>
set -u
TAG=${1:-r01}
export TMPDIR=/tmp
bash tools/gpu_check.sh $TAG || exit 3
cd "$GRAFT_REPO_ROOT" && bash tools/pmc_traffic.sh $TAG || exit 3
cd "$GRAFT_REPO_ROOT" && bash tools/sweep_env.sh "GSGPU_RING_GFLAG=1" || exit 3
mkdir -p gpurun_out/$TAG/cfg
for w in c4 c5 c2; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 > gpurun_out/$TAG/cfg/bench_$w.json 2> gpurun_out/$TAG/cfg/bench_$w.err || { tail -5 gpurun_out/$TAG/cfg/bench_$w.err; exit 3; }
  cut -c1-200 gpurun_out/$TAG/cfg/bench_$w.json
done
