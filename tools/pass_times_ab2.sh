#!/bin/bash
# Follow-up of tools/pass_times_ab.sh: how long does an amd-smi reading slow
# the C4 pipeline?  --pass-times with the reading right before 20 or 200
# timed steps, with a 2 s wait after the reading, and without the reading.
#   RUNS=2 TAG=name bash tools/pass_times_ab2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-pass_times_ab2}; mkdir -p $O
for r in $(seq 1 ${RUNS:-2}); do
  for v in smi20 smi200 smi20_wait2s nosmi200; do
    case $v in
      smi20) a="--steps 20" ;;
      smi200) a="--steps 200" ;;
      smi20_wait2s) a="--steps 20 --gpu-state-delay 2" ;;
      nosmi200) a="--steps 200 --no-gpu-state" ;;
    esac
    timeout -k 10 200 python bench.py --warmup 5 --no-cpu --mix --pass-times $a > $O/${v}_$r.json 2> $O/${v}_$r.err || exit 3
    echo -n "$v $r: "; python3 tools/c4_modes_summary.py "$O/${v}_$r.json"
  done
done
