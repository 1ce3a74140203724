#!/bin/bash
# Instruction profile of the ragged fold (C4 --mix, icrc_rsck_kernel) against
# the strided-chain kernel (headline, icrc_sck_kernel): two rocprofv3 --pmc
# passes per workload (<= 8 SQ counters each), then tools/pmc_insts.py
# normalises per wave step (one 16-byte-per-lane load = 8 lines of 128 B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/${TAG:-pmc_insts}
mkdir -p "$OUT"
export TMPDIR=/tmp
for wl in mix headline; do
  args=""; [ $wl = mix ] && args="--mix"
  i=0
  for grp in \
    "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
    "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAVES" ; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/${wl}_p$i" -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu $args > "$OUT/${wl}_p$i.log" 2>&1
    rc=$?; echo "$wl pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/${wl}_p$i.log"; exit $rc; }
  done
done
python3 tools/pmc_insts.py "$OUT" | tee "$OUT/summary.txt"
