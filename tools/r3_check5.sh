#!/bin/bash
# Session 5: GPU suite, C4 A/B (one-line half-line path vs previous commit), C1 bench x3 (quad in place), rocprof C1 + C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3e}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "[gpu tests] rc=$rc"; tail -3 "$OUT/gpu_tests.log"
[ $rc -ne 0 ] && exit 3
TAG=${TAG:-r3e} ARGS="--mix" RUNS=3 bash tools/ab_bench.sh || exit 4
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --size 64 > "$OUT/bench_c1_$r.json" 2> "$OUT/bench_c1_$r.err" || exit 5
  python3 -c "import json; d=json.load(open('$OUT/bench_c1_$r.json')); print('c1', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
for cfg in "c1:--size 64" "c4:--mix"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu $args > "$OUT/prof_$name.log" 2>&1 || exit 6
  python3 tools/prof_summary.py --last 20 "$OUT/prof_$name/run_kernel_trace.csv" | grep -A1 "quad\|rsck\|rsmall\|gather\|count\|scatter"
done
timeout -k 10 600 python3 tools/pmc_traffic.py --out "$OUT/pmc_traffic.json" --scratch "$OUT/pmc" > "$OUT/pmc.log" 2>&1 || exit 7
timeout -k 10 600 python3 tools/pmc_traffic.py --mix --out "$OUT/pmc_traffic_mix.json" --scratch "$OUT/pmc" > "$OUT/pmc_mix.log" 2>&1 || exit 8
python3 -c "import json; [print(f, json.load(open('$OUT/'+f))['traffic_over_algorithmic']) for f in ('pmc_traffic.json','pmc_traffic_mix.json')]"
