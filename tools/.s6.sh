STEPS="bench:c3s bench:c4s prof:c3s prof:c4s" TAG=r4s6 bash tools/gpu_session.sh || exit $?
timeout -k 10 900 python tools/path_bench.py > gpurun_out/r4s6/path_bench.jsonl 2> gpurun_out/r4s6/path_bench.err; echo "path_bench rc=$?"; cat gpurun_out/r4s6/path_bench.jsonl
