#!/bin/bash
# Parity of an experiment build before adopting it: tests/variant_check.py (production env and the
# ring fold from 2^20 ids) and tests/headline_check.py (RMAT-26) against the C oracle.
# usage (repo root, GPU box): bash tools/exp_parity.sh <tag> <lib path>
set -u
TAG=$1; L=$2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG/parity
mkdir -p "$OUT"
n=$(basename "$L" .so)
GSGPU_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python -u tests/variant_check.py > "$OUT/${n}_prod.json" 2>&1 || { tail -5 "$OUT/${n}_prod.json"; exit 3; }
echo "$n prod: $(grep -o '"ok": [a-z]*' "$OUT/${n}_prod.json" | head -1)"
GSGPU_RING_MIN_BITS=20 GSGPU_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python -u tests/variant_check.py > "$OUT/${n}_ring20.json" 2>&1 || { tail -5 "$OUT/${n}_ring20.json"; exit 3; }
echo "$n ring20: $(grep -o '"ok": [a-z]*' "$OUT/${n}_ring20.json" | head -1)"
GSGPU_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 600 python -u tests/headline_check.py > "$OUT/${n}_headline.json" 2>&1 || { tail -5 "$OUT/${n}_headline.json"; exit 3; }
echo "$n headline: $(tail -1 "$OUT/${n}_headline.json" | cut -c1-400)"
