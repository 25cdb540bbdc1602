# C5 (12 Gbp plant-like, minlen 50, 64-bit builder) bench on one GPU.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c5
mkdir -p $O
free -g > $O/free.txt
GT_SMAX_VERBOSE=1 timeout -k 10 1000 python -u bench.py --config c5 --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err
