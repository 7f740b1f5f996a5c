#!/bin/bash
# Bench lines of the parity configs (c2, c4, c5) + the 8-rank one-GPU exchange simulator + a
# measured HBM copy peak (GPU box): bash tools/configs_run.sh <tag>
set -u
TAG=${1:-r01}
OUT=gpurun_out/$TAG/cfg
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/hbm_peak.py > "$OUT/hbm_peak.json" 2> "$OUT/hbm_peak.err" || { tail -5 "$OUT/hbm_peak.err"; exit 3; }
cat "$OUT/hbm_peak.json"
for w in c2 c4 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -5 "$OUT/bench_$w.err"; exit 3; }
  cut -c1-400 "$OUT/bench_$w.json"
done
timeout -k 10 400 python -u tools/sim_ranks.py 8 64 allgather > "$OUT/sim8_allgather.txt" 2>&1 || { tail -5 "$OUT/sim8_allgather.txt"; exit 3; }
tail -12 "$OUT/sim8_allgather.txt"
