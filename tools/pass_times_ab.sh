#!/bin/bash
# Does the --pass-times diagnostic perturb C4?  Alternating bench processes:
# plain --mix, --mix --pass-times, --mix --pass-times --no-gpu-state (no
# amd-smi readings), RUNS rounds; one summary line per process.
#   RUNS=3 TAG=name bash tools/pass_times_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-pass_times_ab}; mkdir -p $O
for r in $(seq 1 ${RUNS:-3}); do
  for v in plain pt pt_nosmi; do
    case $v in
      plain) a="" ;;
      pt) a="--pass-times" ;;
      pt_nosmi) a="--pass-times --no-gpu-state" ;;
    esac
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --mix $a > $O/${v}_$r.json 2> $O/${v}_$r.err || exit 3
    echo -n "$v $r: "; python3 tools/c4_modes_summary.py "$O/${v}_$r.json"
  done
done
