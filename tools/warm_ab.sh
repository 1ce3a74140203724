#!/bin/bash
# Driver-form bench (K = 20, W = 5) with the workload's own untimed steps run
# for --warm-ms before the warmup, alternating processes; then the default
# K = 100, W = 40 form for comparison.
#   RUNS=2 TAG=name bash tools/warm_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-warm_ab}; mkdir -p $O
for r in $(seq 1 ${RUNS:-2}); do
  for cfg in head mix; do
    a=$([ $cfg = mix ] && echo "--mix" || echo "")
    for wm in 0 100 300 1000; do
      timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --warm-ms $wm $a > $O/${cfg}_w${wm}_$r.json 2> $O/${cfg}_w${wm}_$r.err || exit 3
      python3 -c "import json; d=json.load(open('$O/${cfg}_w${wm}_$r.json')); print('$cfg warm $wm ms run $r:', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
    timeout -k 10 200 python bench.py --steps 100 --warmup 40 --no-cpu $a > $O/${cfg}_k100_$r.json 2> $O/${cfg}_k100_$r.err || exit 3
    python3 -c "import json; d=json.load(open('$O/${cfg}_k100_$r.json')); print('$cfg K=100 W=40 run $r:', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
