#!/bin/bash
# admission cadence + close grid A/B on the headline bench (GPU box): bash tools/knob_sweep2.sh
set -u
export TMPDIR=/tmp
bash tools/ab_env.sh GSGPU_HOT_ADMIT_EVERY "16 32 64 1000000" --steps 5 || exit 3
bash tools/ab_env.sh GSGPU_COMPRESS_GRID "2048 4096" --steps 5 || exit 3
