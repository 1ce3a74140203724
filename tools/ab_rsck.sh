#!/bin/bash
# Same-box A/B of the ragged fold microbench (mix): the current build against
# tools/microbench/rsck_abl_prev (built from an earlier commit), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab; mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 ./tools/microbench/rsck_abl_prev ${MODE:-mix} > $O/prev_$r.txt 2>&1 || exit 3
  timeout -k 10 120 ./tools/microbench/rsck_abl ${MODE:-mix} > $O/new_$r.txt 2>&1 || exit 3
done
for r in 1 2; do for v in prev new; do echo "$v $r: $(grep 'inside' $O/${v}_$r.txt | awk '{print $(NF-3)}' | tr '\n' ' ') full: $(grep 'rsck full ' $O/${v}_$r.txt | tail -1 | awk '{print $(NF-3)}') no-finish: $(grep 'rsck no finish  ' $O/${v}_$r.txt | tail -1 | awk '{print $(NF-3)}') small: $(grep 'small kernel' $O/${v}_$r.txt | tail -1 | awk '{print $(NF-3)}')"; done; done
