STEPS="tests microbench:class_rates" TAG=r4s6 bash tools/gpu_session.sh || exit $?
PREV=tools/ab/head ARGS="--mix" RUNS=3 TAG=r4s6 timeout -k 10 400 bash tools/ab_bench.sh > gpurun_out/r4s6/ab_head.txt 2>&1; tail -6 gpurun_out/r4s6/ab_head.txt
STEPS="bench:c3s bench:c4s prof:c3s prof:c4s" TAG=r4s6 bash tools/gpu_session.sh || exit $?
timeout -k 10 900 python tools/path_bench.py > gpurun_out/r4s6/path_bench.jsonl 2> gpurun_out/r4s6/path_bench.err; echo "path_bench rc=$?"; cat gpurun_out/r4s6/path_bench.jsonl
