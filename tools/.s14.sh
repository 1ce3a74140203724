STEPS="microbench:sck_skew" TAG=r4s14 bash tools/gpu_session.sh || exit $?
timeout -k 10 300 tools/microbench/sck_skew 32 256 > gpurun_out/r4s14/mb_sck_skew_4k_256cu.txt 2>&1; cat gpurun_out/r4s14/mb_sck_skew_4k_256cu.txt
