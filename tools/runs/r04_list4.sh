set -u
bash tools/r04_list.sh r04_list4 || exit 3
bash tools/pmc_traffic.sh r04_pmc_c5_list4 --workload c5 > gpurun_out/pmc_c5_list4.log 2>&1
python3 tools/pmc_dist.py gpurun_out/r04_pmc_c5_list4/pmc/p1 k_compress > gpurun_out/r04_pmc_c5_list4/dist_fetch.txt
rm -rf gpurun_out/r04_pmc_c5_list4/pmc/p[0-9]
cat gpurun_out/r04_pmc_c5_list4/dist_fetch.txt
