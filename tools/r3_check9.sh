#!/bin/bash
# Session 9: C2 (1 M x 1 KiB) and headline against the round-2 final build (tools/ab/r2: rocprof showed C2
# 168 -> 176 us between the rounds); C4 pass grid 512 vs 256 (5 alternating runs); PMC mix traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r3i}
OUT=gpurun_out/$T; mkdir -p "$OUT"
TAG=${T}_c2 PREV=tools/ab/r2 ARGS="--size 1024" RUNS=3 bash tools/ab_bench.sh || exit 4
TAG=${T}_hl PREV=tools/ab/r2 ARGS="--size 4096" RUNS=3 bash tools/ab_bench.sh || exit 5
for r in 1 2 3 4 5; do
  for m in base RICRC_RS_PASS_GRID=256; do
    if [ "$m" = base ]; then e=""; else e="$m"; fi
    env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --mix > $OUT/pg_${m//=/_}_$r.json 2>$OUT/pg_${m//=/_}_$r.err || exit 6
    python3 -c "import json; d=json.load(open('$OUT/pg_${m//=/_}_$r.json')); print('$m $r', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --size 1024 > "$OUT/prof_c2.log" 2>&1 || exit 7
(cd tools/ab/r2 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "../../../$OUT/prof_c2_r2" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --size 1024 > "../../../$OUT/prof_c2_r2.log" 2>&1) || exit 8
for p in prof_c2 prof_c2_r2; do echo $p; python3 tools/prof_summary.py --last 20 "$OUT/$p/run_kernel_trace.csv" | grep -A1 "sck_kernel"; done
timeout -k 10 600 python3 tools/pmc_traffic.py --mix --out "$OUT/pmc_traffic_mix.json" --scratch "$OUT/pmc" > "$OUT/pmc_mix.log" 2>&1 || exit 9
python3 -c "import json; print('mix traffic', json.load(open('$OUT/pmc_traffic_mix.json'))['traffic_over_algorithmic'])"
