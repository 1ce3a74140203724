#!/bin/bash
# Session 22: PMC traffic refresh at the current SCK source (headline + C2), smoke, GPU suite, driver-form headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3s22}; mkdir -p "$OUT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || exit 3
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 280 python3 tools/pmc_traffic.py --out "$OUT/pmc_traffic.json" --scratch "$OUT/pmc" > "$OUT/pmc.log" 2>&1 || exit 4
timeout -k 10 280 python3 tools/pmc_traffic.py --size 1024 --out "$OUT/pmc_traffic_1024.json" --scratch "$OUT/pmc" > "$OUT/pmc1024.log" 2>&1 || exit 5
for f in "$OUT"/pmc_traffic*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['kernel_src'], d['traffic_over_algorithmic'])"; done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 6
cat "$OUT/bench.json"
