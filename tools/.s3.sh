STEPS="smoke tests microbench:fold_var" TAG=r4s3 bash tools/gpu_session.sh || exit $?
ARGS="--mix" RUNS=3 TAG=r4s3 timeout -k 10 400 bash tools/ab_bench.sh > gpurun_out/r4s3/ab_prev.txt 2>&1; tail -6 gpurun_out/r4s3/ab_prev.txt
PREV=tools/ab/sl0 ARGS="--mix" RUNS=3 TAG=r4s3sl0 timeout -k 10 400 bash tools/ab_bench.sh > gpurun_out/r4s3/ab_sl0.txt 2>&1; tail -6 gpurun_out/r4s3/ab_sl0.txt
STEPS="prof:c4" TAG=r4s3 bash tools/gpu_session.sh
