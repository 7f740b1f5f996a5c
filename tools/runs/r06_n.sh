#!/bin/bash
# Round 6: run-to-run spread of the streaming file-ingestion line (bench.py --workload parse_file), 4 runs.
set -u
TAG=${1:-r06_n}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py --workload parse_file --steps 3 > "$OUT/parse_file_$i.json" 2> "$OUT/parse_file_$i.err"
  rc=$?; echo "parse_file $i rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/parse_file_$i.json'));r=d['roofline'];print('%.3f G edges/s  %.1f of %.1f GB/s (%.2f)'%(d['value']/1e9,r['achieved'],r['peak'],r['frac']))")"
  [ $rc -eq 0 ] || { tail -5 "$OUT/parse_file_$i.err"; exit 3; }
done
exit 0
