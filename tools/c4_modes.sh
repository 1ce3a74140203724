#!/bin/bash
# C4's per-process step-time modes: N separate bench
# processes on one box, each timing the ragged pipeline's passes inside its
# own timed steps (--pass-times: HIP events between bucket / fold / one-line /
# gather) and reading the GPU's clocks, power and temperature right before and
# after them, in the same process; one summary line per process.
#   RUNS=6 TAG=name bash tools/c4_modes.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-c4_modes}; mkdir -p $O
for r in $(seq 1 ${RUNS:-6}); do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --mix --pass-times ${ARGS:-} > $O/run_$r.json 2> $O/run_$r.err || exit 3
  python3 tools/c4_modes_summary.py "$O/run_$r.json"
done
