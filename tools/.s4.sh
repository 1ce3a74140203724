STEPS="microbench:class_rates microbench:c1_probe" TAG=r4s4 bash tools/gpu_session.sh || exit $?
RUNS=6 TAG=r4s4/c4_modes timeout -k 10 600 bash tools/c4_modes.sh > gpurun_out/r4s4/c4_modes.txt 2>&1; cat gpurun_out/r4s4/c4_modes.txt
