#!/bin/bash
# Two extra PMC passes over the C4 bench for the ragged fold's issue profile
# (branches, instruction fetch, icache); one rocprofv3 --pmc run per pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/pmc_fold
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in \
  "SQ_INSTS_BRANCH SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
  "SQC_ICACHE_HITS SQC_ICACHE_MISSES" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --mix > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_summary.py "$OUT" | tee "$OUT/summary.txt"
