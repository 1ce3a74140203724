STEPS="tests" TAG=r4s7 bash tools/gpu_session.sh || exit $?
timeout -k 10 300 python tools/path_bench.py --only-ring > gpurun_out/r4s7/path_ring.jsonl 2> gpurun_out/r4s7/path_ring.err; echo "ring rc=$?"; cat gpurun_out/r4s7/path_ring.jsonl
PREV=tools/ab/head ARGS="--mix" RUNS=4 TAG=r4s7 timeout -k 10 500 bash tools/ab_bench.sh > gpurun_out/r4s7/ab_head.txt 2>&1; tail -8 gpurun_out/r4s7/ab_head.txt
