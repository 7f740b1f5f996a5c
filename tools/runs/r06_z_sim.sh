set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_z
for cfg in "2 23 prefilter" "4 22 prefilter" "8 21 prefilter" "8 21 gather" "8 21 tree"; do
  set -- $cfg
  SIM_WLOG2=$2 timeout -k 10 400 python -u tools/sim_ranks.py $1 64 $3 > gpurun_out/r06_z/sim_$3_p$1.txt 2>&1 || { echo SIM_FAIL $cfg; tail -5 gpurun_out/r06_z/sim_$3_p$1.txt; exit 1; }
  echo "P=$1 $3: $(grep TOTAL gpurun_out/r06_z/sim_$3_p$1.txt)"
done
