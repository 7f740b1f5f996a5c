#!/bin/bash
# warm band passes A/B on the headline bench (GPU box): bash tools/bands_ab.sh
set -u
export TMPDIR=/tmp
bash tools/ab_env.sh GSGPU_WARM_BANDS "4 5 6" --steps 5 || exit 3
