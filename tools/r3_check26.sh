#!/bin/bash
# Session 26: full check at the current sources (tools/r3_check17.sh's steps) + PMC traffic for every kept record.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r3s26}
TAG=$T bash tools/gpu_check.sh || exit $?
OUT=gpurun_out/$T
timeout -k 10 600 python3 tools/pmc_traffic.py --mix --out "$OUT/pmc_traffic_mix.json" --scratch "$OUT/pmc_mix" > "$OUT/pmc_mix.log" 2>&1 || exit 8
timeout -k 10 280 python3 tools/pmc_traffic.py --size 1024 --out "$OUT/pmc_traffic_1024.json" --scratch "$OUT/pmc" > "$OUT/pmc1024.log" 2>&1 || exit 9
timeout -k 10 280 python3 tools/pmc_traffic.py --size 64 --out "$OUT/pmc_traffic_64.json" --scratch "$OUT/pmc" > "$OUT/pmc64.log" 2>&1 || exit 10
for f in "$OUT"/pmc_traffic*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['kernel_src'], round(d['traffic_over_algorithmic'], 5))"; done
for cfg in headline c1 c2 c4; do echo "== $cfg"; python3 tools/prof_summary.py --last 20 "$OUT/prof_$cfg/run_kernel_trace.csv" | grep -v "copyBuffer\|synth\|prime" | grep -A1 "icrc\|rsck\|gather\|bucket"; done
for f in bench bench_mix_c4 bench_c1 bench_c2 bench_c3_16GiB; do python3 -c "import json; d=json.load(open('$OUT/$f.json')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('traffic'))"; done
