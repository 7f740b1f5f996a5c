set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_y
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_y/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r06_y/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r06_y/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_y/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r06_y/smoke.log; exit 1; }
tail -2 gpurun_out/r06_y/smoke.log
for c in 1 0; do
  SIM_WLOG2=21 GSGPU_PAIR_COMBINE=$c timeout -k 10 300 python -u tools/sim_ranks.py 8 64 allgather > gpurun_out/r06_y/ag21_64_c$c.txt 2>&1 || { echo SIM_FAIL; exit 1; }
  grep -E "^w  [15] |TOTAL" gpurun_out/r06_y/ag21_64_c$c.txt
done
