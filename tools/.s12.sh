RUNS=3 TAG=r4s12 timeout -k 10 900 bash tools/prime_ab.sh > gpurun_out/r4s12_prime_ab.txt 2>&1; cat gpurun_out/r4s12_prime_ab.txt
