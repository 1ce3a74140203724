#!/bin/bash
# Session 32: SCK grid sweeps (4 KiB, 1 KiB) and the ragged fold grid (RICRC_RSCK_GRID) on the C4 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3s32}; mkdir -p "$OUT"
GRID_SWEEP=1 timeout -k 10 150 ./tools/microbench/half_line > "$OUT/grid_sweep.txt" 2>&1 || exit 2
cat "$OUT/grid_sweep.txt"
TAG=${TAG:-r3s32}_env MODES="base RICRC_RSCK_GRID=240 RICRC_RSCK_GRID=224" ARGS="--mix" bash tools/ab_env.sh || exit 3
