STEPS="microbench:sck_skew" TAG=r4s13 bash tools/gpu_session.sh || exit $?
timeout -k 10 300 tools/microbench/sck_skew 8 > gpurun_out/r4s13/mb_sck_skew_1k.txt 2>&1; cat gpurun_out/r4s13/mb_sck_skew_1k.txt
