#!/bin/bash
# The driver-form bench (K = 20 timed steps) with the default 25 ms primer
# against a 200 ms primer, alternating processes, for C4 and the headline.
#   RUNS=3 TAG=name bash tools/prime_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-prime_ab}; mkdir -p $O
for r in $(seq 1 ${RUNS:-3}); do
  for cfg in mix head; do
    for pm in 25 200; do
      a=$([ $cfg = mix ] && echo "--mix" || echo "")
      timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --prime-ms $pm $a > $O/${cfg}_${pm}_$r.json 2> $O/${cfg}_${pm}_$r.err || exit 3
      python3 -c "import json; d=json.load(open('$O/${cfg}_${pm}_$r.json')); print('$cfg prime $pm ms run $r:', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
    done
  done
done
