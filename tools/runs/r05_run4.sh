#!/bin/bash
# Round 5, box 4: the young windows' union work as a separate kernel with CAS-free claims (k_filter
# CLAIM, GSGPU_RUN_AHEAD=3) against the fused ring fold (0) and the plain serialised split (2):
# parity first (variant_check, ring from 2^20 ids), then headline bench lines and kernel traces per
# window; the atomic lab with the relaxed atomic store; the barrier lab.
set -u
TAG=${1:-r05_run4}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_comm.py \
  -k "overflow or mismatched or rccl_world1" > "$OUT/pytest_comm.log" 2>&1
rc=$?; echo "pytest comm rc=$rc"; tail -3 "$OUT/pytest_comm.log"; [ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -u bench.py --workload parse_file --steps 5 > "$OUT/bench_parse_file.json" 2> "$OUT/bench_parse_file.err"
rc=$?; echo "parse_file rc=$rc"; cat "$OUT/bench_parse_file.json"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_parse_file.err"; exit 3; }
GSGPU_RUN_AHEAD=3 GSGPU_RING_MIN_BITS=20 timeout -k 10 300 python -u tests/variant_check.py > "$OUT/variant3.json" 2> "$OUT/variant3.err"
rc=$?; echo "variant3 rc=$rc"; python -c "import json; d=json.loads(open('$OUT/variant3.json').read().splitlines()[-1]); print('variant ok', d['ok'], [c for c in d['cases'] if not c['ok']])"
[ $rc -eq 0 ] || { tail -5 "$OUT/variant3.err"; exit 3; }
GSGPU_RUN_AHEAD=3 timeout -k 10 600 python -u tests/headline_check.py --fold-windows --no-torch --variant > "$OUT/headline3.json" 2> "$OUT/headline3.err"
rc=$?; echo "headline3 rc=$rc"; tail -c 300 "$OUT/headline3.json"; [ $rc -eq 0 ] || { tail -5 "$OUT/headline3.err"; exit 3; }
for v in 3 0 2; do
  GSGPU_RUN_AHEAD=$v timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"
  rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_$v.err"; exit 3; }
  python -c "import json; d=json.loads([l for l in open('$OUT/bench_$v.json') if l.startswith('{')][-1]); print('head run_ahead=$v: %.3f G edges/s %.3f ms/step match %s' % (d['value']/1e9, d['ms_per_step'], d['final_checksum_vs_fixture']['match']))"
done
cd /tmp
for v in 3 0; do
  GSGPU_RUN_AHEAD=$v timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/trace_$v" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-fold-timing > "$GRAFT_REPO_ROOT/$OUT/trace_$v.log" 2>&1
  rc=$?; echo "trace $v rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$GRAFT_REPO_ROOT/$OUT/trace_$v.log"; exit 3; }
  python3 "$GRAFT_REPO_ROOT/tools/trace_steps.py" "$(ls $GRAFT_REPO_ROOT/$OUT/trace_$v/*kernel_trace.csv)" 1 > "$GRAFT_REPO_ROOT/$OUT/windows_$v.txt" 2>&1
  head -20 "$GRAFT_REPO_ROOT/$OUT/windows_$v.txt"; tail -1 "$GRAFT_REPO_ROOT/$OUT/windows_$v.txt"
done
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 ./tools/atomic_lab > "$OUT/atomic_lab.json" 2>&1; echo "atomic rc=$?"; cat "$OUT/atomic_lab.json"
exit 0
