RUNS=2 TAG=r4s11 timeout -k 10 900 bash tools/pass_times_ab2.sh > gpurun_out/r4s11_pass_times_ab2.txt 2>&1; cat gpurun_out/r4s11_pass_times_ab2.txt
