#!/bin/bash
# Same-box A/B of bench configurations that differ only in environment
# knobs, alternating runs:  MODES="base RICRC_NO_GATHER_SPLIT=1" ARGS="--mix --count 524288" bash tools/ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab_env}; mkdir -p $O
for r in 1 2 3; do
  for m in ${MODES:-base}; do
    if [ "$m" = base ]; then e=""; else e="$m"; fi
    env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-side ${ARGS:---mix} > $O/${m//=/_}_$r.json 2>$O/${m//=/_}_$r.err || exit 3
    python3 -c "import json; d=json.load(open('$O/${m//=/_}_$r.json')); print('$m $r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
