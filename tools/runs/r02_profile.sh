#!/bin/bash
# Round-2 measurement batch (repo root, GPU box): PMC passes of the headline bench (per-launch HBM
# traffic of k_fold_ring) and the fold/close costs at the per-rank window of an 8-GPU strong run
# (2^21-edge windows on one GPU). usage: bash tools/r02_profile.sh <tag>
set -u
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 3; }
bash tools/pmc_traffic.sh "$TAG" || exit 3
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --window-log2 21 --no-cpu-baseline > "$OUT/bench_w21.json" 2> "$OUT/bench_w21.err" || { tail -5 "$OUT/bench_w21.err"; exit 3; }
cut -c1-200 "$OUT/bench_w21.json"; python3 -c "import json;d=json.load(open('$OUT/bench_w21.json'));print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernels'])"
