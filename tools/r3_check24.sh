#!/bin/bash
# Session 24: cheap last-line edge path in the ragged fold: GPU suite, fold attribution microbench (random data),
# C4 A/B against tools/ab/prev (HEAD), rocprof C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3s24}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "[gpu tests] rc=$rc"; tail -2 "$OUT/gpu_tests.log"
[ $rc -ne 0 ] && exit 3
timeout -k 10 200 ./tools/microbench/bucket_abl > "$OUT/bucket_abl.txt" 2>&1 || exit 4
grep "^fold" "$OUT/bucket_abl.txt" | tail -7
TAG=${TAG:-r3s24}_prev ARGS="--mix" RUNS=3 bash tools/ab_bench.sh || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --mix > "$OUT/prof_c4.log" 2>&1 || exit 6
python3 tools/prof_summary.py --last 20 "$OUT/prof_c4/run_kernel_trace.csv" | grep -A1 "rsck\|rsmall\|gather\|bucket"
