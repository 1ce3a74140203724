#!/bin/bash
# Session 6: GPU suite, C4 A/B (fold quiet blocks whose loads cross groups vs previous commit), rocprof C4, PMC mix traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3f}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "[gpu tests] rc=$rc"; tail -3 "$OUT/gpu_tests.log"
[ $rc -ne 0 ] && exit 3
TAG=${TAG:-r3f} ARGS="--mix" RUNS=3 bash tools/ab_bench.sh || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --mix > "$OUT/prof_c4.log" 2>&1 || exit 6
python3 tools/prof_summary.py --last 20 "$OUT/prof_c4/run_kernel_trace.csv" | grep -A1 "rsck\|rsmall\|gather\|count\|scatter"
timeout -k 10 600 python3 tools/pmc_traffic.py --mix --out "$OUT/pmc_traffic_mix.json" --scratch "$OUT/pmc" > "$OUT/pmc_mix.log" 2>&1 || exit 8
python3 -c "import json; print('mix traffic', json.load(open('$OUT/pmc_traffic_mix.json'))['traffic_over_algorithmic'])"
