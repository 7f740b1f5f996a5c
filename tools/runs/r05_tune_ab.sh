#!/bin/bash
# Round 5: tuning constants re-measured on the current code, same box, alternated (GSGPU_LIB).
set -u
OUT=gpurun_out/r05_tune
mkdir -p "$OUT"
export TMPDIR=/tmp
LIBS="${LIBS:-base admit8 admit2 warmat1 pick32 thresh2 cgrid4096 cgrid1024}"
for i in ${ROUNDS:-1 2}; do
  for v in $LIBS; do
    if [ $v = base ]; then unset GSGPU_LIB; else export GSGPU_LIB=$PWD/_var/$v/libgsgpu.so; fi
    timeout -k 10 300 python -u bench.py --steps 8 --no-cpu-baseline > "$OUT/b_$v.json" 2> "$OUT/b_$v.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_$v.err"; exit 3; }
    python -c "import json; d=json.loads([l for l in open('$OUT/b_$v.json') if l.startswith('{')][-1]); print('%-10s run $i: %.3f G edges/s %.3f ms/step %s' % ('$v', d['value']/1e9, d['ms_per_step'], d['library']))" | tee -a "$OUT/summary.txt"
  done
done
unset GSGPU_LIB
exit 0
