export TMPDIR=/tmp; O=gpurun_out/r2h; mkdir -p $O
timeout -k 10 120 ./tools/microbench/mb_scatter | grep COLD
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/pmc1 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --mix --prime-ms 0 > $O/pmc1.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/pmc2 -o run -- ./tools/microbench/mb_scatter > $O/pmc2.log 2>&1 || exit 3
python3 tools/pmc_summary.py $O/pmc1 | grep -A9 rsmall
python3 tools/pmc_summary.py $O/pmc2 | grep -A9 "fold_allILi16ELb1"
