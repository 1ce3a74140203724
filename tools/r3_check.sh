#!/bin/bash
# Round-3 GPU session: new tests first (no -x: see every failure), then the
# standard check (smoke, whole GPU suite, benches, rocprof, PMC), then the
# same-box C4 A/B against the previous commit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest ${NEWTESTS:-tests/test_gpu_fixtures.py tests/test_gpu_status.py} -m gpu -v --timeout 120 --timeout-method thread > "$OUT/new_tests.log" 2>&1
rc=$?; echo "[new tests] rc=$rc"; tail -5 "$OUT/new_tests.log"
[ $rc -ge 2 ] && [ $rc -ne 1 ] && exit $rc
TAG=${TAG:-r3} bash tools/gpu_check.sh || exit $?
[ "${SKIP_AB:-0}" = 1 ] || TAG=${TAG:-r3} ARGS="--mix" bash tools/ab_bench.sh
