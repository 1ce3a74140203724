STEPS="tests" TAG=r4s16 bash tools/gpu_session.sh || exit $?
PREV=tools/ab/head ARGS=" " RUNS=3 TAG=r4s16h timeout -k 10 400 bash tools/ab_bench.sh > gpurun_out/r4s16/ab_head_headline.txt 2>&1; tail -6 gpurun_out/r4s16/ab_head_headline.txt
PREV=tools/ab/head ARGS="--mix" RUNS=3 TAG=r4s16m timeout -k 10 400 bash tools/ab_bench.sh > gpurun_out/r4s16/ab_head_mix.txt 2>&1; tail -6 gpurun_out/r4s16/ab_head_mix.txt
PREV=tools/ab/head ARGS="--global-count 4194304" RUNS=2 TAG=r4s16c3 timeout -k 10 400 bash tools/ab_bench.sh > gpurun_out/r4s16/ab_head_c3.txt 2>&1; tail -4 gpurun_out/r4s16/ab_head_c3.txt
