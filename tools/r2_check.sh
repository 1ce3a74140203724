#!/bin/bash
# Quick GPU check after a kernel change: microbench, GPU tests, benches.
#   TESTS="tests/test_gpu_parity.py ..." BENCHES="--size 1024|" bash tools/r2_check.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-check}; mkdir -p $O
if [ -n "${MB:-}" ]; then timeout -k 10 200 $MB > $O/mb.txt 2>&1 || exit 3; cat $O/mb.txt; fi
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ge 2 ] && exit $rc
IFS='|' read -ra BS <<< "${BENCHES:-}"
n=0
for r in 1 2; do for b in "${BS[@]}"; do n=$((n+1))
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu $b > $O/b$n.json 2>$O/b$n.err || exit 3
  python3 -c "import json; d=json.load(open('$O/b$n.json')); print('[$b]', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done; done
exit $rc
