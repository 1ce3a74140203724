#!/bin/bash
# PMC passes over the ragged fold on uniform 1 KiB, with and without its
# result stores (tools/microbench/rsck_abl s1k).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/pmc_stores; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for grp in \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
  "TA_BUSY_avr TA_TA_BUSY_sum" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- ./tools/microbench/rsck_abl s1k > "$OUT/p$i.log" 2>&1
  echo "pass $i rc=$?"
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1; grep -A20 "rsck_kernel" "$OUT/summary.txt" | head -60
