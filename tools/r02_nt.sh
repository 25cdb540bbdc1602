# K1 window DMA with the nt policy (A, in-tree) vs default policy (B = ab/libB.so), interleaved.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/nt
mkdir -p $O
timeout -k 10 300 python -u tools/ab_interleave.py human 3e9 20 ab/libB.so 6 0/1 > $O/ab_c3.txt 2>&1
timeout -k 10 300 python -u tools/ab_interleave.py human 3e9 20 ab/libB.so 6 3/8 > $O/ab_s3of8.txt 2>&1
timeout -k 10 300 python -u tools/ab_interleave.py uniform 1e8 20 ab/libB.so 6 0/1 > $O/ab_c2.txt 2>&1
