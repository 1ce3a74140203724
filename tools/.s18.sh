STEPS="smoke tests pmc:headline pmc:c1 pmc:c2 pmc:c3 pmc:c4 pmc:c3s pmc:c4s" TAG=r4s18 bash tools/gpu_session.sh
