#!/bin/bash
# Session 33: SCK grid on 15/16 of the CUs: GPU suite, same-box A/B against tools/ab/prev (HEAD, all CUs)
# for the headline, C2 and C3 (alternating processes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3s33}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "[gpu tests] rc=$rc"; tail -2 "$OUT/gpu_tests.log"
[ $rc -ne 0 ] && exit 3
TAG=r3s33_head ARGS=" " RUNS=3 bash tools/ab_bench.sh || exit 4
TAG=r3s33_c2 ARGS="--size 1024" RUNS=3 bash tools/ab_bench.sh || exit 5
TAG=r3s33_c3 ARGS="--global-count 4194304" RUNS=2 bash tools/ab_bench.sh || exit 6
