RUNS=3 TAG=r4s10 timeout -k 10 900 bash tools/pass_times_ab.sh > gpurun_out/r4s10_pass_times_ab.txt 2>&1; cat gpurun_out/r4s10_pass_times_ab.txt
