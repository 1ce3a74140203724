#!/bin/bash
# Same-box A/B of several library snapshots (tools/ab/<name>/, each a copy of
# roce-test_amd + bench.py + oracle + include [+ tools/ring_bench.py] built in
# place), alternating processes:
#   VARS="prev va vb" ARGS="--mix --count 524288" RUNS=3 bash tools/ab_multi.sh
#   VARS="prev va" RING="1024:64-1010,2048:64-2034" RUNS=2 bash tools/ab_multi.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab_multi}; mkdir -p $O
for r in $(seq 1 ${RUNS:-3}); do
  for v in ${VARS}; do
    d=tools/ab/$v
    if [ -n "${RING:-}" ]; then
      (cd $d && timeout -k 10 200 python tools/ring_bench.py --cases "$RING" --reps 20) > $O/${v}_$r.jsonl 2>$O/${v}_$r.err || exit 3
      python3 -c "
import json
for l in open('$O/${v}_$r.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print('$v $r', d['slot'], d['lengths'], d['ms'], d['frac'])"
    else
      (cd $d && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-side ${ARGS}) > $O/${v}_$r.json 2>$O/${v}_$r.err || exit 3
      python3 -c "import json; d=json.load(open('$O/${v}_$r.json')); print('$v $r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
    fi
  done
done
