STEPS="microbench:placement" TAG=r4s8 bash tools/gpu_session.sh || exit $?
RUNS=4 TAG=r4s8/c4_modes timeout -k 10 600 bash tools/c4_modes.sh > gpurun_out/r4s8/c4_modes.txt 2>&1; cat gpurun_out/r4s8/c4_modes.txt
