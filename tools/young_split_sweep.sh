set -u
export TMPDIR=/tmp
GSGPU_YOUNG_SPLIT=65536 GSGPU_YOUNG_SPLITS=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "baseline_config or c5_small or full_size" > gpurun_out/ys_tests.log 2>&1 || { tail -20 gpurun_out/ys_tests.log; exit 3; }
tail -2 gpurun_out/ys_tests.log
bash tools/sweep_env.sh "GSGPU_YOUNG_SPLIT=0" "GSGPU_YOUNG_SPLIT=2097152" "GSGPU_YOUNG_SPLIT=4194304" "GSGPU_YOUNG_SPLIT=8388608" "GSGPU_YOUNG_SPLIT=1048576 GSGPU_YOUNG_SPLITS=3" "GSGPU_YOUNG_SPLIT=2097152 GSGPU_YOUNG_SPLITS=2" "GSGPU_YOUNG_SPLIT=524288 GSGPU_YOUNG_SPLITS=5" || exit 3
GSGPU_YOUNG_SPLIT=2097152 GSGPU_YOUNG_SPLITS=2 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --verify --no-cpu-baseline > gpurun_out/ys_bench.json 2> gpurun_out/ys_bench.err || exit 3
cat gpurun_out/ys_bench.json | python -c "import json,sys; b=json.loads(sys.stdin.read()); print(b['value']/1e9, b.get('verify'))"
