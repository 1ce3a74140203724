#!/bin/bash
# Session 8: GPU suite; C4 A/B of the working tree (first loads before the table fill) against tools/ab/prev
# (half-line commit); pass / gather grid study by environment knobs; rocprof C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r3h}
OUT=gpurun_out/$T; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "[gpu tests] rc=$rc"; tail -3 "$OUT/gpu_tests.log"
[ $rc -ne 0 ] && exit 3
TAG=${T}_prev ARGS="--mix" RUNS=3 bash tools/ab_bench.sh || exit 4
TAG=${T}_env MODES="base RICRC_RS_PASS_GRID=256 RICRC_RS_PASS_GRID=128 RICRC_RS_GATHER_GRID=2048 RICRC_RS_GATHER_GRID=1024" ARGS="--mix" bash tools/ab_env.sh || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --mix > "$OUT/prof_c4.log" 2>&1 || exit 6
python3 tools/prof_summary.py --last 20 "$OUT/prof_c4/run_kernel_trace.csv" | grep -A1 "rsck\|rsmall\|gather\|count\|scatter"
