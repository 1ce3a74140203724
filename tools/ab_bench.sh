#!/bin/bash
# Same-box A/B of a bench configuration: the working tree against
# tools/ab/prev/ (a snapshot of an earlier commit with its own built library:
#   mkdir -p tools/ab/prev && git archive <rev> roce-test_amd bench.py \
#     __graft_entry__.py oracle include | tar -x -C tools/ab/prev && \
#   make -C tools/ab/prev/roce-test_amd/csrc && make -C tools/ab/prev/oracle),
# alternating runs.   ARGS="--mix" RUNS=3 [PREV=tools/ab/other] bash tools/ab_bench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_bench${TAG:+_$TAG}; mkdir -p $O
PREV=${PREV:-tools/ab/prev}
[ -d $PREV ] || { echo "no $PREV snapshot"; exit 3; }
R=${RUNS:-3}
for r in $(seq 1 $R); do
  (cd $PREV && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-side ${ARGS:---mix}) > $O/prev_$r.json 2>$O/prev_$r.err || exit 3
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-side ${ARGS:---mix} > $O/new_$r.json 2>$O/new_$r.err || exit 3
done
for r in $(seq 1 $R); do for v in prev new; do python3 -c "import json; d=json.load(open('$O/${v}_$r.json')); print('$v $r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; done; done
