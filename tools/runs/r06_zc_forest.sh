set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_zc
SIM_WLOG2=21 timeout -k 10 600 python -u tools/sim_ranks.py 8 64 prefilter_forest prefilter > gpurun_out/r06_zc/sim_p8.txt 2>&1 || { echo SIM_FAIL; tail -5 gpurun_out/r06_zc/sim_p8.txt; exit 1; }
grep -E "^==|^w  [1-9] |TOTAL" gpurun_out/r06_zc/sim_p8.txt
