#!/bin/bash
# Same-box A/B of a bench configuration (tools/ab_bench.sh), then a rocprofv3
# kernel trace of each side: per-kernel means of the timed steps.
#   ARGS="--mix" bash tools/ab_prof.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd); O=gpurun_out/${TAG:-ab_prof}; mkdir -p $O
ARGS="${ARGS:---mix}" bash tools/ab_bench.sh || exit 3
for v in new prev; do
  d=$R; [ $v = prev ] && d=$R/tools/ab/prev
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/$v -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu ${ARGS:---mix} > $R/$O/$v.log 2>&1) || exit 3
  echo "== $v"; python3 tools/prof_summary.py --last 20 $(find $O/$v -name '*kernel_trace.csv' | head -1) | grep -A1 "rsck\|rsmall\|icrc_sck\|stream_kernel" | grep -v "^--"
done
