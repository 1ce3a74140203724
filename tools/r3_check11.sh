#!/bin/bash
# Session 11: bucket pass on 256 blocks x 16 packets per thread (all resident), non-bucketed packets in the gather:
# GPU suite, C4 A/B against tools/ab/prev (half-line commit), rocprof C4 of both builds on the same box, PMC mix.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r3k}
OUT=gpurun_out/$T; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "[gpu tests] rc=$rc"; tail -5 "$OUT/gpu_tests.log"
[ $rc -ne 0 ] && exit 3
TAG=${T}_prev ARGS="--mix" RUNS=3 bash tools/ab_bench.sh || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --mix > "$OUT/prof_c4.log" 2>&1 || exit 6
(cd tools/ab/prev && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "../../../$OUT/prof_c4_prev" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --mix > "../../../$OUT/prof_c4_prev.log" 2>&1) || exit 7
for p in prof_c4 prof_c4_prev; do echo $p; python3 tools/prof_summary.py --last 20 "$OUT/$p/run_kernel_trace.csv" | grep -A1 "rsck\|rsmall\|gather\|bucket"; done
timeout -k 10 600 python3 tools/pmc_traffic.py --mix --out "$OUT/pmc_traffic_mix.json" --scratch "$OUT/pmc" > "$OUT/pmc_mix.log" 2>&1 || exit 8
python3 -c "import json; d=json.load(open('$OUT/pmc_traffic_mix.json')); print('mix traffic', d['traffic_over_algorithmic'], {k: round(2*v['FETCH_SIZE_KiB']/1024+v['WRITE_SIZE_KiB']/1024,1) for k,v in d['kernels'].items()})"
