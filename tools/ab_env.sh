#!/bin/bash
# A/B an env-var knob over bench.py (interleaved runs). usage: bash tools/ab_env.sh VAR "valA valB" [bench args]
VAR=$1; VALS=$2; shift 2
mkdir -p gpurun_out/ab
for rep in 1 2; do for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/ab/$VAR-$v-$rep.json 2>/dev/null
  rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi
  python -c "import json; b=json.load(open('gpurun_out/ab/$VAR-$v-$rep.json')); print('$VAR=$v rep $rep: %.2f Ge/s  %.2f ms/step  fold/win %.3f ms  close/win %.4f ms' % (b['value']/1e9, b['ms_per_step'], b['roofline']['fold_ms_per_window'], b['kernels']['compress_ms_per_window']))"
done; done
