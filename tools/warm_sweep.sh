# warm-set / admission cadence sweep on the headline stream (GPU box): bash tools/warm_sweep.sh
set -u
export TMPDIR=/tmp
bash tools/sweep_env.sh "GSGPU_WARM=1" "GSGPU_WARM_SAMPLE=4194304" "GSGPU_WARM_SAMPLE=2097152" "GSGPU_WARM_AT=5" "GSGPU_WARM_AT=2" "GSGPU_HOT_ADMIT_EVERY=1000000" "GSGPU_WARM_AT=5 GSGPU_WARM_SAMPLE=4194304" || exit 3
