#!/bin/bash
# Session 40: PMC traffic for C4 at the current ragged sources, C4 driver-form bench, rocprof C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3s40}; mkdir -p "$OUT"
timeout -k 10 600 python3 tools/pmc_traffic.py --mix --out "$OUT/pmc_traffic_mix.json" --scratch "$OUT/pmc_mix" > "$OUT/pmc_mix.log" 2>&1 || exit 2
python3 -c "import json; d=json.load(open('$OUT/pmc_traffic_mix.json')); print('mix traffic', d['kernel_src'], d['traffic_over_algorithmic'])"
cp "$OUT/pmc_traffic_mix.json" profiles/pmc_traffic_mix.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mix > "$OUT/bench_mix_c4.json" 2> "$OUT/bench_mix.err" || exit 3
python3 -c "import json; d=json.load(open('$OUT/bench_mix_c4.json')); r=d['roofline']; print('c4', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('traffic'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --mix > "$OUT/prof_c4.log" 2>&1 || exit 4
python3 tools/prof_summary.py --last 20 "$OUT/prof_c4/run_kernel_trace.csv" | grep -A1 "rsck\|rsmall\|gather\|bucket"
