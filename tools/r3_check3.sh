#!/bin/bash
# Quad kernel (C1) session: GPU suite, C1 bench (driver form) + rocprof, C4 A/B, fold instruction profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3c}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "[gpu tests] rc=$rc"; tail -3 "$OUT/gpu_tests.log"
[ $rc -ne 0 ] && exit 3
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --size 64 > "$OUT/bench_c1_$r.json" 2> "$OUT/bench_c1_$r.err" || exit 4
  python3 -c "import json; d=json.load(open('$OUT/bench_c1_$r.json')); print('c1', d['metric'][:60], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c1" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --size 64 > "$OUT/prof_c1.log" 2>&1 || exit 5
python3 tools/prof_summary.py --last 20 "$OUT/prof_c1/run_kernel_trace.csv" | grep -A1 quad
TAG=${TAG:-r3c}_insts bash tools/pmc_insts.sh || exit 6
timeout -k 10 600 python3 tools/pmc_traffic.py --out "$OUT/pmc_traffic.json" --scratch "$OUT/pmc" > "$OUT/pmc.log" 2>&1 || exit 7
timeout -k 10 600 python3 tools/pmc_traffic.py --mix --out "$OUT/pmc_traffic_mix.json" --scratch "$OUT/pmc" > "$OUT/pmc_mix.log" 2>&1 || exit 8
python3 -c "import json; [print(f, json.load(open('$OUT/'+f))['traffic_over_algorithmic']) for f in ('pmc_traffic.json','pmc_traffic_mix.json')]"
TAG=${TAG:-r3c}_modes RUNS=6 bash tools/c4_modes.sh
