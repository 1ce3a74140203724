#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprofv3 kernel stats.
# Stops at the first step that crashes, aborts or times out (exit >= 2 or
# signal): a plain test failure (rc 1) still lets the bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ge 2 ]; then echo "stopping after $what"; exit "$rc"; fi; }

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; ok $? smoke
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > "$OUT/gpu_tests.log" 2>&1; ok $? gpu_tests
  tail -5 "$OUT/gpu_tests.log"
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"; ok $? bench
cat "$OUT/bench.json"
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu > "$OUT/prof.log" 2>&1; ok $? rocprof
  find "$OUT/prof" -name '*kernel_stats.csv' -exec cat {} \;
fi
if [ "${SKIP_PMC:-0}" != 1 ]; then
  timeout -k 10 600 python3 tools/pmc_traffic.py --out "$OUT/pmc_traffic.json" --scratch "$OUT/pmc_scratch" > "$OUT/pmc.log" 2>&1; ok $? pmc
  cat "$OUT/pmc_traffic.json"
fi
