# kernel stats of the one-GPU 8-rank simulator (GPU box): bash tools/sim_prof.sh [windows]
set -u
export TMPDIR=/tmp
NW=${1:-16}
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/simprof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/simprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/sim_ranks.py 8 $NW allgather > $GRAFT_REPO_ROOT/gpurun_out/simprof/log.txt 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/simprof/log.txt; exit 3; }
cut -c1-200 $GRAFT_REPO_ROOT/gpurun_out/simprof/run_kernel_stats.csv
