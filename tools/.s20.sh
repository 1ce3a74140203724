STEPS="microbench:tailfill" TAG=r4s20 bash tools/gpu_session.sh
