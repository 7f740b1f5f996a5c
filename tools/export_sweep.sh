# export grid sweep with the one-GPU multi-rank simulator (GPU box): bash tools/export_sweep.sh
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
for b in 1024 256 128; do
  GSGPU_EXPORT_BLOCKS=$b timeout -k 10 300 python -u tools/sim_ranks.py 8 16 allgather > gpurun_out/exp/blocks_$b.txt 2>&1 || { tail -5 gpurun_out/exp/blocks_$b.txt; exit 3; }
  echo "== blocks $b"; tail -6 gpurun_out/exp/blocks_$b.txt
done
