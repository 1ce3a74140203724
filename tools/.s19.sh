STEPS="bench:headline bench:c1 bench:c2 bench:c3 bench:c4 bench:c3s bench:c4s prof:headline prof:c1 prof:c2 prof:c3 prof:c4 prof:c3s prof:c4s" TAG=r4s19 bash tools/gpu_session.sh
