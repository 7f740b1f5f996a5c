#!/bin/bash
# Final round-3 evidence (GPU box, repo root): the four PMC passes of the headline bench (refreshes
# profiles/fold_traffic.json for this library), then the extra bench lines and the per-window
# profile (tools/r03_lines.sh). usage: bash tools/r03_evidence.sh <tag>
set -u
TAG=${1:-r03_ev}
bash tools/pmc_traffic.sh "$TAG" || exit 3
bash tools/r03_lines.sh "$TAG/lines" || exit 3
exit 0
