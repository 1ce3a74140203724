#!/bin/bash
# One GPU-box session from one commit: the only launcher (replaces round 2-3's
# one-off tools/r2*.sh / r3_check*.sh scripts).  STEPS picks what runs, in order:
#   smoke                 __graft_entry__.smoke()
#   tests                 pytest -m gpu (PYTEST_K="expr" selects with -k)
#   bench:<cfg>           driver-form bench line   -> $OUT/bench_<cfg>.json
#   prof:<cfg>            rocprofv3 --kernel-trace --stats of the bench, per-kernel
#                         summary of the timed launches -> $OUT/prof_<cfg>.txt
#   pmc:<cfg>             FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.py)
#                         -> $OUT/pmc_<cfg>.json (copy into profiles/ by hand)
#   microbench:<name>     build + run tools/microbench/<name>.hip -> $OUT/mb_<name>.txt
# configs (BASELINE.json configs + the 8-GPU shard stand-ins of SURVEY 8(e)):
#   headline  1 M x 4096 B          c1  1 M x 64 B       c2  1 M x 1024 B
#   c3        4 M x 4096 B (16 GiB)  c4  4 M mixed 64/256/1024/4096 B
#   c3s       512 K x 4096 B (C3's shard at N = 8)
#   c4s       512 K mixed (C4's shard at N = 8: 4 M mixed over 8 GPUs)
#   ring      1 M x 4096 B Ethernet-framed NIC ring slots, the L3 packet at 14
#   ring_len  1 M x 1024 B ring slots, L3 at 14, a length per slot of 64..1010 B
#   ringbench tools/ring_bench.py (every ring row)   pathbench tools/path_bench.py
# Every GPU step runs under its own timeout; the session stops at the first
# step that crashes, aborts or times out (rc >= 2); a plain test failure
# (rc 1) lets the rest run.
#   gpurun -- 'STEPS="smoke tests bench:headline prof:c4" TAG=r4s1 bash tools/gpu_session.sh'
# (variables go inside the command: the box does not see this shell's environment)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-session}
mkdir -p "$OUT"
K=${BENCH_STEPS:-20}
W=${BENCH_WARMUP:-5}
git_rev() { cat .git_rev 2>/dev/null || echo unknown; }
echo "session $OUT at $(git_rev), $(date -u +%FT%TZ)" | tee "$OUT/session.txt"

cfg_args() {
  case "$1" in
    headline) echo "" ;;
    c1) echo "--size 64" ;;
    c2) echo "--size 1024" ;;
    c3) echo "--global-count 4194304" ;;
    c4) echo "--mix" ;;
    c3s) echo "--count 524288" ;;
    c4s) echo "--mix --count 524288" ;;
    ring) echo "--l3-offset 14 --stride 4096" ;;
    ring_len) echo "--l3-offset 14 --stride 1024 --slot-lengths 64:1010" ;;
    *) echo "BAD" ;;
  esac
}
pmc_args() {
  case "$1" in
    headline) echo "" ;;
    c1) echo "--size 64" ;;
    c2) echo "--size 1024" ;;
    c3) echo "--count 4194304" ;;
    c4) echo "--mix" ;;
    c3s) echo "--count 524288" ;;
    c4s) echo "--mix --count 524288" ;;
    ring) echo "--l3-offset 14 --stride 4096" ;;
    ring_len) echo "--l3-offset 14 --stride 1024 --slot-lengths 64:1010" ;;
    *) echo "BAD" ;;
  esac
}
ok() {
  local rc=$1 what=$2
  echo "[$what] rc=$rc" | tee -a "$OUT/session.txt"
  if [ "$rc" -ge 2 ]; then echo "stopping after $what" | tee -a "$OUT/session.txt"; exit "$rc"; fi
}

for step in ${STEPS:-smoke tests bench:headline}; do
  kind=${step%%:*}
  cfg=${step#*:}
  case "$kind" in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      ok $? smoke ;;
    tests)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/gpu_tests.log" 2>&1
      ok $? tests
      tail -3 "$OUT/gpu_tests.log" ;;
    bench)
      a=$(cfg_args "$cfg")
      t0=$SECONDS
      timeout -k 10 300 python bench.py --steps "$K" --warmup "$W" $a ${BENCH_ARGS:-} > "$OUT/bench_$cfg.json" \
        2> "$OUT/bench_$cfg.err"
      ok $? "bench $cfg"
      echo "bench $cfg: $((SECONDS - t0)) s wall (the process, side configs included)" | tee -a "$OUT/session.txt"
      python3 -c "import json; d=json.load(open('$OUT/bench_$cfg.json')); r=d['roofline']; \
print('$cfg', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('traffic'), d.get('pass_ms'))" \
        | tee -a "$OUT/session.txt" ;;
    prof)
      a=$(cfg_args "$cfg")
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$cfg" -o run -- \
        python3 bench.py --steps "$K" --warmup "$W" --no-cpu --no-side $a > "$OUT/prof_$cfg.log" 2>&1
      ok $? "rocprof $cfg"
      python3 tools/prof_summary.py --last "$K" "$OUT/prof_$cfg/run_kernel_trace.csv" > "$OUT/prof_$cfg.txt"
      grep -v "copyBuffer\|synth\|prime\|fill" "$OUT/prof_$cfg.txt" | grep -A1 "icrc\|rsck\|gather\|bucket\|rs_" \
        | tee -a "$OUT/session.txt" ;;
    pmc)
      a=$(pmc_args "$cfg")
      timeout -k 10 600 python3 tools/pmc_traffic.py $a --out "$OUT/pmc_$cfg.json" --scratch "$OUT/pmc_scratch" \
        > "$OUT/pmc_$cfg.log" 2>&1
      ok $? "pmc $cfg"
      python3 -c "import json; d=json.load(open('$OUT/pmc_$cfg.json')); print('pmc $cfg', d['kernel_src'], \
round(d['traffic_over_algorithmic'], 5))" | tee -a "$OUT/session.txt" ;;
    ringbench)
      timeout -k 10 300 python tools/ring_bench.py > "$OUT/ring_bench.jsonl" 2> "$OUT/ring_bench.err"
      ok $? ringbench
      cut -c1-160 "$OUT/ring_bench.jsonl" | tee -a "$OUT/session.txt" ;;
    pathbench)
      timeout -k 10 600 python tools/path_bench.py ${PATH_ARGS:-} > "$OUT/path_bench.jsonl" 2> "$OUT/path_bench.err"
      ok $? pathbench
      cut -c1-200 "$OUT/path_bench.jsonl" | tee -a "$OUT/session.txt" ;;
    microbench)
      (cd tools/microbench && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 "$cfg.hip" -o "$cfg" \
        > "../../$OUT/mb_${cfg}_build.log" 2>&1)
      rc=$?; [ $rc -ne 0 ] && rc=2  # a failed build must not run a stale binary
      ok $rc "build $cfg"
      timeout -k 10 300 "tools/microbench/$cfg" ${MB_ARGS:-} > "$OUT/mb_$cfg.txt" 2>&1
      ok $? "microbench $cfg"
      tail -40 "$OUT/mb_$cfg.txt" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session done" | tee -a "$OUT/session.txt"
