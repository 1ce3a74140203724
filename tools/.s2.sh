STEPS="smoke microbench:fold_var tests bench:c4 bench:headline" TAG=r4s2 bash tools/gpu_session.sh || exit $?
ARGS="--mix" RUNS=3 TAG=r4s2 timeout -k 10 400 bash tools/ab_bench.sh > gpurun_out/r4s2/ab.txt 2>&1; tail -6 gpurun_out/r4s2/ab.txt
STEPS="prof:c4 microbench:aos_probe" TAG=r4s2b bash tools/gpu_session.sh || exit $?
RUNS=4 TAG=r4s2/c4_modes timeout -k 10 600 bash tools/c4_modes.sh > gpurun_out/r4s2/c4_modes.txt 2>&1; tail -4 gpurun_out/r4s2/c4_modes.txt
timeout -k 10 500 python tools/path_bench.py --quick > gpurun_out/r4s2/path_bench.jsonl 2> gpurun_out/r4s2/path_bench.err; tail -12 gpurun_out/r4s2/path_bench.jsonl
