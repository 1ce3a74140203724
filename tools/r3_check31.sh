#!/bin/bash
# Session 31: SCK grid sweep (microbench, alternating) and driver-form headline bench with RICRC_SCK_GRID (alternating processes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3s31}; mkdir -p "$OUT"
GRID_SWEEP=1 timeout -k 10 120 ./tools/microbench/half_line > "$OUT/grid_sweep.txt" 2>&1 || exit 2
cat "$OUT/grid_sweep.txt"
TAG=${TAG:-r3s31}_env MODES="base RICRC_SCK_GRID=240 RICRC_SCK_GRID=224 RICRC_SCK_GRID=192" ARGS=" " bash tools/ab_env.sh || exit 3
