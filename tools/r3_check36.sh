#!/bin/bash
# Session 36: end-of-session check at HEAD (smoke, GPU suite, driver-form benches of every config, rocprof per config).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r3s36}
SKIP_PMC=1 TAG=$T bash tools/gpu_check.sh || exit $?
OUT=gpurun_out/$T
for cfg in headline c1 c2 c4; do echo "== $cfg"; python3 tools/prof_summary.py --last 20 "$OUT/prof_$cfg/run_kernel_trace.csv" | grep -v "copyBuffer\|synth\|prime" | grep -A1 "icrc\|rsck\|gather\|bucket"; done
for f in bench bench_mix_c4 bench_c1 bench_c2 bench_c3_16GiB; do python3 -c "import json; d=json.load(open('$OUT/$f.json')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('traffic'))"; done
