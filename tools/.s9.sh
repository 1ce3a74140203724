STEPS="microbench:placement" TAG=r4s9 bash tools/gpu_session.sh
