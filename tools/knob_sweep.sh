#!/bin/bash
# A/B of several fold knobs on the headline bench (GPU box): bash tools/knob_sweep.sh
set -u
export TMPDIR=/tmp
bash tools/ab_env.sh GSGPU_WARM_BUCKETS "18 19" --steps 5 || exit 3
bash tools/ab_env.sh GSGPU_HOT_THRESH "3 4" --steps 5 || exit 3
bash tools/ab_env.sh GSGPU_WARM_SAMPLE "8388608 16777216" --steps 5 || exit 3
bash tools/ab_env.sh GSGPU_YOUNG_BPC "2 4" --steps 5 || exit 3
bash tools/ab_env.sh GSGPU_COMPRESS_GRID "2048 1024" --steps 5 || exit 3
bash tools/ab_env.sh GSGPU_HOT_ADMIT_EVERY "16 32" --steps 5 || exit 3
