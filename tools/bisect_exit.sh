set -u
mkdir -p gpurun_out/r02_f
export PYTHONFAULTHANDLER=1
for f in tests/test_gpu_parity.py tests/test_gpu_variants.py; do
  n=$(basename $f .py)
  timeout -k 10 600 python -u -m pytest $f -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_f/$n.log 2>&1
  rc=$?
  echo "$n rc=$rc"; tail -25 gpurun_out/r02_f/$n.log | grep -v "^\.\.\."
  case $rc in 124|137|139) exit 3;; esac
done
