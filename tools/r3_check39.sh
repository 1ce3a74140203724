#!/bin/bash
# Session 39: 17 packets per thread in the bucket / gather passes above 4 M packets: GPU suite, A/B (tools/ab/prev = HEAD)
# on the largest C4 shard of an 8-GPU weak-scaling run (4,197,912 packets) and on C4 (4 M), 2 KiB SCK A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3s39}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "[gpu tests] rc=$rc"; tail -2 "$OUT/gpu_tests.log"
[ $rc -ne 0 ] && exit 3
TAG=r3s39_big ARGS="--mix --count 4197912" RUNS=3 bash tools/ab_bench.sh || exit 4
TAG=r3s39_c4 ARGS="--mix" RUNS=2 bash tools/ab_bench.sh || exit 5
