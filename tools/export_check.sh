# export change: multi-rank GPU parity tests, then the simulator's kernel stats (GPU box)
set -u
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "exchange or two_ranks or export or mark" > gpurun_out/exp_tests.log 2>&1 || { tail -30 gpurun_out/exp_tests.log; exit 3; }
tail -2 gpurun_out/exp_tests.log
bash tools/sim_prof.sh 16 | grep -E "k_export|k_fold<unsigned int, true|Name" || exit 3
grep TOTAL gpurun_out/simprof/log.txt
