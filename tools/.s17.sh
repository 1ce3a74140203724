cd tools/microbench && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 sck_skew.hip -o sck_skew && cd ../.. && mkdir -p gpurun_out/r4s17 || exit 2
for g in 224 232 240; do timeout -k 10 200 tools/microbench/sck_skew 32 $g 1048576 0,15,20,25,30 > gpurun_out/r4s17/sck_4k_$g.txt 2>&1 || exit 3; grep round gpurun_out/r4s17/sck_4k_$g.txt | tail -2; done
for g in 224 240 256; do timeout -k 10 200 tools/microbench/sck_skew 8 $g 1048576 0,10,20,30,40,50 > gpurun_out/r4s17/sck_1k_$g.txt 2>&1 || exit 3; grep round gpurun_out/r4s17/sck_1k_$g.txt | tail -2; done
