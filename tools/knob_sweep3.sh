#!/bin/bash
# hot-set budget / sample and young chunk A/B on the headline bench (GPU box): bash tools/knob_sweep3.sh
set -u
export TMPDIR=/tmp
bash tools/ab_env.sh GSGPU_HOT_BUDGET "8 4 16" --steps 5 || exit 3
bash tools/ab_env.sh GSGPU_HOT_SAMPLE "262144 524288" --steps 5 || exit 3
bash tools/ab_env.sh GSGPU_YOUNG_CHUNK "262144 524288 131072" --steps 5 || exit 3
