#!/bin/bash
# Session 17: full check at the current sources (smoke, GPU suite, driver-form benches of every config,
# rocprof per config, PMC traffic for the headline and for the C4 mix) + the ragged attribution microbench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r3q}
TAG=$T bash tools/gpu_check.sh || exit $?
OUT=gpurun_out/$T
timeout -k 10 600 python3 tools/pmc_traffic.py --mix --out "$OUT/pmc_traffic_mix.json" --scratch "$OUT/pmc_mix" > "$OUT/pmc_mix.log" 2>&1 || exit 8
python3 -c "import json; d=json.load(open('$OUT/pmc_traffic_mix.json')); print('mix traffic', d['traffic_over_algorithmic'], {k: round(2*v['FETCH_SIZE_KiB']/1024+v['WRITE_SIZE_KiB']/1024,1) for k,v in d['kernels'].items()})"
timeout -k 10 200 ./tools/microbench/bucket_abl > "$OUT/bucket_abl.txt" 2>&1 || exit 9
for cfg in headline c1 c2 c4; do echo "== $cfg"; python3 tools/prof_summary.py --last 20 "$OUT/prof_$cfg/run_kernel_trace.csv" | grep -v "copyBuffer\|synth\|prime" | grep -A1 "icrc\|rsck\|gather\|bucket"; done
