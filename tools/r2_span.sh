#!/bin/bash
# Headline after the one-copy finish tables: PMC traffic at HEAD, rocprof of
# the driver's form, and a same-box A/B of span vs per-step events.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-span}; mkdir -p $O
timeout -k 10 400 python3 tools/pmc_traffic.py --out $O/pmc_traffic.json --scratch $O/pmc_scratch > $O/pmc.log 2>&1 || exit 3
cat $O/pmc_traffic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_head -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/prof_head.log 2>&1 || exit 3
python3 tools/prof_summary.py --last 20 $(find $O/prof_head -name '*kernel_trace.csv' | head -1) | grep -A1 sck
for r in 1 2 3; do
  for m in span step; do
    if [ $m = step ]; then x=--step-events; else x=; fi
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu $x > $O/${m}_$r.json 2>$O/${m}_$r.err || exit 3
    python3 -c "import json; d=json.load(open('$O/${m}_$r.json')); print('$m $r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  done
done
