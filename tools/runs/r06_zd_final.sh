set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_zd
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_zd/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r06_zd/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r06_zd/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_zd/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r06_zd/smoke.log; exit 1; }
tail -1 gpurun_out/r06_zd/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r06_zd/bench.json 2> gpurun_out/r06_zd/bench.err || { echo BENCH_FAIL; tail -5 gpurun_out/r06_zd/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r06_zd/bench.json'));r=d['roofline'];print(d['value']/1e9, d['ms_per_step'], r['frac'], r['traffic_source'], r['requests']['frac'], d['final_checksum_vs_fixture']['match'])"
