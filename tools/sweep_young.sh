#!/bin/bash
# Sweep the young-forest knobs over the first 12 windows of the headline stream (GPU box).
# usage: bash tools/sweep_young.sh "ENV=a ENV2=b" "ENV=c" ...
mkdir -p gpurun_out/sweep
for cfg in "$@"; do
  tag=$(echo "$cfg" | tr ' =' '_-')
  env $cfg timeout -k 10 120 python -u tools/window_profile.py 12 > gpurun_out/sweep/$tag.txt 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "$cfg rc=$rc"; tail -3 gpurun_out/sweep/$tag.txt; exit $rc; fi
  python - "$cfg" gpurun_out/sweep/$tag.txt <<'PY'
import sys
rows = [l.split() for l in open(sys.argv[2]) if l.startswith("window")]
f = [float(r[3]) for r in rows]; c = [float(r[6]) for r in rows]
print("%-50s w1 %7.1f w2 %6.1f w3 %6.1f w4-12 %7.1f | fold sum %8.1f close sum %6.1f" % (sys.argv[1], f[0], f[1], f[2], sum(f[3:]), sum(f), sum(c)))
PY
done
