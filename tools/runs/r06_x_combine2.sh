set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_x
for rep in 1 2; do
for c in 1 0; do
  SIM_WLOG2=21 GSGPU_PAIR_COMBINE=$c timeout -k 10 300 python -u tools/sim_ranks.py 8 16 allgather > gpurun_out/r06_x/ag21_c${c}_$rep.txt 2>&1 || { echo SIM_FAIL $c; tail -5 gpurun_out/r06_x/ag21_c${c}_$rep.txt; exit 1; }
  grep -E "^w  [1-5] |TOTAL" gpurun_out/r06_x/ag21_c${c}_$rep.txt
done
done
