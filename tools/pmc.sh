#!/bin/bash
# PMC passes over the bench (one rocprofv3 --pmc run per counter group, as
# /opt/skills/guides/MI355X_MICROARCH.md prescribes).
# Usage: TAG=x [PROG=tools/path_bench.py] tools/pmc.sh [program args]   (PROG defaults to bench.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/pmc_${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
PROG="${PROG:-bench.py}"
if [ "$PROG" = bench.py ]; then ARGS="${*:---steps 5 --warmup 1 --no-cpu}"; else ARGS="$*"; fi
i=0
for grp in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
  "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_WAVES SQ_LEVEL_WAVES SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 $PROG $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_summary.py "$OUT" | tee "$OUT/summary.txt"
