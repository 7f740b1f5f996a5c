#!/bin/bash
# Round-6 evidence for the library as committed (GPU box, repo root). Parts:
#   evidence  the default bench line (as the driver runs it), a rocprofv3 kernel-stats run of the same
#             command, the headline's PMC passes (fold_traffic.json for these sources), the per-window
#             profile, the config lines (c2 / c4 / c5 x2 / int64) and the PMC passes of configs 2, 4, 5
#   rows      the SURVEY 8(f) rows' lines (parse, parse_file, bip) and the host-input / emit-host /
#             exchange-at-world-1 lines
# Every GPU step has its own limit; a failure stops the script. usage: bash tools/runs/r06_final.sh <tag> <part>
set -u
TAG=${1:-r06_final}; PART=${2:-evidence}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$PART" = evidence ]; then
# the PMC passes first: their traffic.json becomes this tree's profiles/fold_traffic.json, so the bench
# line below carries roofline.traffic of these very sources (copy it into the repo afterwards)
bash tools/pmc_traffic.sh "$TAG" > "$OUT/pmc.out" 2>&1 || { echo "pmc failed"; tail -5 "$OUT/pmc.out"; exit 3; }
cp "$OUT/pmc/traffic.json" profiles/fold_traffic.json
echo "pmc ok"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc $(cut -c1-200 $OUT/bench.json)"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit 3; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/prof.log"; exit 3; }
timeout -k 10 300 python -u tools/window_profile.py > "$OUT/window_profile.txt" 2> "$OUT/window_profile.err"
rc=$?; echo "wprof rc=$rc $(tail -1 $OUT/window_profile.txt)"; [ $rc -eq 0 ] || exit 3
for w in c2 c4 c5 c5; do
  n=$w; [ -e "$OUT/bench_$w.json" ] && n=${w}_2
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --no-cpu-baseline > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err"
  rc=$?; echo "bench $n rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$n.json'));print('%.3f G'%(d['value']/1e9), d.get('window_latency',''))")"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$n.err"; exit 3; }
done
timeout -k 10 300 python -u bench.py --id-bits 64 --steps 3 --no-cpu-baseline > "$OUT/bench_int64.json" 2> "$OUT/bench_int64.err"
rc=$?; echo "bench int64 rc=$rc"; [ $rc -eq 0 ] || exit 3
for w in c2 c4 c5; do
  bash tools/pmc_traffic.sh "${TAG}_$w" --workload $w > "$OUT/pmc_$w.out" 2>&1 || { echo "pmc $w failed"; tail -5 "$OUT/pmc_$w.out"; exit 3; }
  echo "pmc $w ok"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_c4" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof_c4.log" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; echo "rocprof c4 rc=$rc"; [ $rc -eq 0 ] || exit 3
exit 0
fi
if [ "$PART" = rows ]; then
for w in parse parse_file bip; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  rc=$?; echo "bench $w rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$w.err"; exit 3; }
done
timeout -k 10 300 python -u bench.py --host-input --steps 3 --no-cpu-baseline > "$OUT/bench_host.json" 2> "$OUT/bench_host.err"
rc=$?; echo "bench host rc=$rc"; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -u bench.py --emit-host --steps 3 --no-cpu-baseline > "$OUT/bench_emit_host.json" 2> "$OUT/bench_emit_host.err"
rc=$?; echo "bench emit-host rc=$rc"; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -u bench.py --window-log2 21 --exchange-world1 --merge prefilter --steps 3 --no-cpu-baseline > "$OUT/bench_w21_xchg.json" 2> "$OUT/bench_w21_xchg.err"
rc=$?; echo "bench w21 exchange rc=$rc"; [ $rc -eq 0 ] || exit 3
exit 0
fi
exit 0
