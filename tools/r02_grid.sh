# K1 grid sweep: 8-way shard and whole C3.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/grid
mkdir -p $O
GT_SMAX_VERBOSE=1 timeout -k 10 400 python -u tools/k1_grid_sweep.py human 3e9 20 3/8 768 1024 1536 2048 3072 4096 6144 8192 12288 > $O/s3of8.txt 2> $O/s3of8.err
timeout -k 10 400 python -u tools/k1_grid_sweep.py human 3e9 20 0/1 3072 6144 12288 24576 49152 > $O/c3.txt 2>&1
