#!/bin/bash
# giant-flag survivors: GPU parity suite, then A/B against parent reads (GPU box): bash tools/gflag_check.sh
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/gflag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gflag/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/gflag/pytest.log; if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/gflag/pytest.log | head; exit 3; fi
bash tools/ab_env.sh GSGPU_RING_GFLAG "1 0" --steps 5 || exit 3
bash tools/sweep_env.sh "GSGPU_RING_GFLAG=1" "GSGPU_RING_GFLAG=0" || exit 3
