# K1b per-tile cycle profile (workgroup kernel) at C3, whole and one 8-way shard.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/k1b
mkdir -p $O
timeout -k 10 300 python -u tools/k1b_cycles.py human 3e9 20 0 0/1 > $O/c3.txt 2>&1
timeout -k 10 300 python -u tools/k1b_cycles.py human 3e9 20 0 3/8 > $O/c3_s3of8.txt 2>&1
