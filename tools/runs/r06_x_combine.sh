set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_x
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_prefilter.py tests/test_gpu_parity.py -p no:cacheprovider > gpurun_out/r06_x/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r06_x/pytest.log; exit 1; }
tail -2 gpurun_out/r06_x/pytest.log
for c in 1 0; do
  GSGPU_PAIR_COMBINE=$c timeout -k 10 300 python -u tools/sim_ranks.py 8 16 allgather > gpurun_out/r06_x/ag16_c$c.txt 2>&1 || { echo SIM_FAIL $c; tail -5 gpurun_out/r06_x/ag16_c$c.txt; exit 1; }
done
grep -E "^w  [15] |total|step" gpurun_out/r06_x/ag16_c1.txt | head; echo ---; grep -E "^w  [15] |total|step" gpurun_out/r06_x/ag16_c0.txt | head
