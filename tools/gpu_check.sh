#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> benches -> rocprofv3 kernel stats -> PMC traffic.
# Stops at the first step that crashes, aborts or times out (exit >= 2 or
# signal): a plain test failure (rc 1) still lets the benches run.
#   TAG=name  SKIP_TESTS=1 SKIP_PROF=1 SKIP_PMC=1 SKIP_EXTRA=1  PYTEST_ARGS=...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ge 2 ]; then echo "stopping after $what"; exit "$rc"; fi; }

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; ok $? smoke
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/gpu_tests.log" 2>&1; ok $? gpu_tests
  tail -3 "$OUT/gpu_tests.log"
fi
# the driver's form
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"; ok $? bench
cat "$OUT/bench.json"
if [ "${SKIP_EXTRA:-0}" != 1 ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --global-count 4194304 > "$OUT/bench_c3_16GiB.json" 2> "$OUT/bench_c3.err"; ok $? bench_c3
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mix > "$OUT/bench_mix_c4.json" 2> "$OUT/bench_mix.err"; ok $? bench_mix
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --size 1024 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"; ok $? bench_c2
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --size 64 > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err"; ok $? bench_c1
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  for cfg in "headline:" "c1:--size 64" "c2:--size 1024" "c4:--mix"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu $args > "$OUT/prof_$name.log" 2>&1; ok $? "rocprof $name"
  done
fi
if [ "${SKIP_PMC:-0}" != 1 ]; then
  timeout -k 10 600 python3 tools/pmc_traffic.py --out "$OUT/pmc_traffic.json" --scratch "$OUT/pmc_scratch" > "$OUT/pmc.log" 2>&1; ok $? pmc
  cat "$OUT/pmc_traffic.json"
fi
