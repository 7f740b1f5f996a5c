#!/bin/bash
# Round-4 regression check: parity subset, then the per-window profile and the headline bench with
# the current library and with the round's starting library (gsgpu/lib/exp/libgsgpu_old.so, built
# from commit 010a0e2), alternated on one box
set -u
TAG=${1:-r04_cmp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_listclose.py \
  tests/test_gpu_parity.py -k "listclose or list_close or c5 or random_streams or baseline_config or emit_delta or streams_golden" \
  > "$OUT/pytest.log" 2>&1
rc=$?; tail -1 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -20; exit 3; }
OLD=$GRAFT_REPO_ROOT/gelly-streaming_amd/gsgpu/lib/exp/libgsgpu_old.so
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export GSGPU_LIB=$OLD; else unset GSGPU_LIB; fi
    timeout -k 10 300 python -u tools/window_profile.py > "$OUT/wp_${v}_$i.txt" 2> "$OUT/wp_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/wp_${v}_$i.err"; exit 3; }
    echo "$v $i: $(tail -1 $OUT/wp_${v}_$i.txt)"
    timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > "$OUT/b_${v}_$i.json" 2> "$OUT/b_${v}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/b_${v}_$i.err"; exit 3; }
    python -c "import json; d=json.loads([l for l in open('$OUT/b_${v}_$i.json') if l.startswith('{')][-1]); print('$v $i bench: %.3f G edges/s %.3f ms/step' % (d['value']/1e9, d['ms_per_step']))"
  done
done
unset GSGPU_LIB
exit 0
