#!/bin/bash
# PMC passes (FETCH/WRITE, L2 hit/miss, memory-side atomics) of BASELINE configs 2, 4 and 5,
# per-kernel totals in <tag>_cN/pmc/traffic.json. usage: bash tools/r03_pmc_cfg.sh <tag>
set -u
TAG=${1:-r03_pmc}
for w in c2 c4 c5; do
  bash tools/pmc_traffic.sh "${TAG}_$w" --workload $w > /dev/null || { echo "pmc $w failed"; exit 3; }
  echo "pmc $w ok"
done
exit 0
