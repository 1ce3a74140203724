#!/bin/bash
# Same-box A/B of a bench configuration: the current library against
# tools/ab/libroceicrc_prev.so (a build of an earlier commit), alternating runs.
#   ARGS="--mix" bash tools/ab_bench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_bench; mkdir -p $O
rm -rf /tmp/prevrepo && mkdir -p /tmp/prevrepo && cp -r bench.py __graft_entry__.py oracle roce-test_amd /tmp/prevrepo/ && cp tools/ab/libroceicrc_prev.so /tmp/prevrepo/roce-test_amd/roce_icrc/libroceicrc.so || exit 3
for r in 1 2 3; do
  (cd /tmp/prevrepo && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu ${ARGS:---mix}) > $O/prev_$r.json 2>$O/prev_$r.err || exit 3
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu ${ARGS:---mix} > $O/new_$r.json 2>$O/new_$r.err || exit 3
done
for r in 1 2 3; do for v in prev new; do python3 -c "import json; d=json.load(open('$O/${v}_$r.json')); print('$v $r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; done; done
