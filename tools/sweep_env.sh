#!/bin/bash
# Per-window fold times of the headline stream (64 windows) under env-var configurations (GPU box).
# usage: bash tools/sweep_env.sh "ENV=a ENV2=b" "ENV=c" ...
mkdir -p gpurun_out/sweep
for cfg in "$@"; do
  tag=$(echo "$cfg" | tr ' =' '_-')
  env $cfg timeout -k 10 120 python -u tools/window_profile.py 64 > gpurun_out/sweep/$tag.txt 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "$cfg rc=$rc"; tail -3 gpurun_out/sweep/$tag.txt; exit $rc; fi
  python - "$cfg" gpurun_out/sweep/$tag.txt <<'PY'
import sys
rows = [l.split() for l in open(sys.argv[2]) if l.startswith("window")]
f = [float(r[3]) for r in rows]; c = [float(r[6]) for r in rows]
print("%-44s w1 %6.0f w2-12 %6.0f  w13-32 avg %5.1f  w33-64 avg %5.1f | fold %6.0f close %5.0f us" % (
    sys.argv[1], f[0], sum(f[1:12]), sum(f[12:32]) / 20, sum(f[32:]) / 32, sum(f), sum(c)))
PY
done
