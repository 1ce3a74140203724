STEPS="microbench:class_rates" TAG=r4s5 bash tools/gpu_session.sh
