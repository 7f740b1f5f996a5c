set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_zb
BASE=$GRAFT_REPO_ROOT/gelly-streaming_amd/gsgpu/lib/ab/base/libgsgpu.so
for rep in 1 2; do
  for v in new base; do
    if [ $v = base ]; then L=$BASE; else L=$GRAFT_REPO_ROOT/gelly-streaming_amd/gsgpu/lib/libgsgpu.so; fi
    GSGPU_LIB=$L SIM_WLOG2=21 timeout -k 10 400 python -u tools/sim_ranks.py 8 64 prefilter > gpurun_out/r06_zb/pf_${v}_$rep.txt 2>&1 || { echo SIM_FAIL; tail -5 gpurun_out/r06_zb/pf_${v}_$rep.txt; exit 1; }
    echo "$v $rep: $(grep -E '^w  1 ' gpurun_out/r06_zb/pf_${v}_$rep.txt | cut -c1-150)"; grep TOTAL gpurun_out/r06_zb/pf_${v}_$rep.txt
  done
done
timeout -k 10 700 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_prefilter.py -p no:cacheprovider > gpurun_out/r06_zb/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -20 gpurun_out/r06_zb/pytest.log; exit 1; }
tail -1 gpurun_out/r06_zb/pytest.log
