#!/bin/bash
# Session 10: block-local bucket pass (count pass + plan removed): GPU suite, C4 A/B against tools/ab/prev
# (half-line commit, count + plan + scatter), rocprof C4, PMC mix traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r3j}
OUT=gpurun_out/$T; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "[gpu tests] rc=$rc"; tail -5 "$OUT/gpu_tests.log"
[ $rc -ne 0 ] && exit 3
TAG=${T}_prev ARGS="--mix" RUNS=3 bash tools/ab_bench.sh || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --mix > "$OUT/prof_c4.log" 2>&1 || exit 6
python3 tools/prof_summary.py --last 20 "$OUT/prof_c4/run_kernel_trace.csv" | grep -A1 "rsck\|rsmall\|gather\|bucket"
timeout -k 10 600 python3 tools/pmc_traffic.py --mix --out "$OUT/pmc_traffic_mix.json" --scratch "$OUT/pmc" > "$OUT/pmc_mix.log" 2>&1 || exit 8
python3 -c "import json; d=json.load(open('$OUT/pmc_traffic_mix.json')); print('mix traffic', d['traffic_over_algorithmic'], list(d['kernels']))"
