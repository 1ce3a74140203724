#!/bin/bash
# Dead-slot clamp of the ragged fold: parity, same-box bench A/B against the
# previous commit, microbench, and the fold's FETCH_SIZE on both builds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/clamp; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_sim_stream.py tests/test_gpu_dist.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
ARGS="--mix" bash tools/ab_bench.sh || exit 3
SYNTH=1 timeout -k 10 200 ./tools/microbench/rsck_abl mix > $O/rsck_abl_mix.txt 2>&1 || exit 3
grep -E "rsck full|clamp|memory path" $O/rsck_abl_mix.txt
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_new -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --mix > $O/pmc_new.log 2>&1 || exit 3
(cd /tmp/prevrepo && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_prev -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --mix > $GRAFT_REPO_ROOT/$O/pmc_prev.log 2>&1) || exit 3
for v in prev new; do echo "== $v"; python3 tools/pmc_summary.py $O/pmc_$v | grep -A1 "rsck_kernel\|rsmall" | grep -v "^--"; done
