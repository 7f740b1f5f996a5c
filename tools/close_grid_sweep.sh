#!/bin/bash
# young-close grid sweep, per-window fold/close sums over 64 windows (GPU box): bash tools/close_grid_sweep.sh
set -u
export TMPDIR=/tmp
bash tools/sweep_env.sh "GSGPU_COMPRESS_GRID_YOUNG=2048" "GSGPU_COMPRESS_GRID_YOUNG=8192" "GSGPU_COMPRESS_GRID_YOUNG=65536" "GSGPU_COMPRESS_GRID_YOUNG=2048" "GSGPU_COMPRESS_GRID_YOUNG=16384" || exit 3
