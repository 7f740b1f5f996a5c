set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_x
for cfg in "1 0" "1 1" "0 1"; do
  set -- $cfg
  SIM_WLOG2=21 GSGPU_PAIR_COMBINE=$1 GSGPU_PAIR_HALVE=$2 timeout -k 10 300 python -u tools/sim_ranks.py 8 16 allgather > gpurun_out/r06_x/ag21_c$1_h$2.txt 2>&1 || { echo SIM_FAIL; tail -5 gpurun_out/r06_x/ag21_c$1_h$2.txt; exit 1; }
  echo "== allgather combine=$1 halve=$2"; grep -E "^w  [15] |TOTAL" gpurun_out/r06_x/ag21_c$1_h$2.txt
done
for cfg in "1 0" "1 1" "0 1"; do
  set -- $cfg
  SIM_WLOG2=21 GSGPU_PAIR_COMBINE=$1 GSGPU_PAIR_HALVE=$2 timeout -k 10 400 python -u tools/sim_ranks.py 8 64 prefilter > gpurun_out/r06_x/pf21_c$1_h$2.txt 2>&1 || { echo SIM_FAIL; tail -5 gpurun_out/r06_x/pf21_c$1_h$2.txt; exit 1; }
  echo "== prefilter combine=$1 halve=$2"; grep -E "^w  [15] |TOTAL" gpurun_out/r06_x/pf21_c$1_h$2.txt
done
