# K1b workgroup kernel variants, interleaved A/B with K1 event times:
# A in-tree, B = previous build (ab/libB.so), C = ab/libC.so.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/k1bab2
mkdir -p $O
timeout -k 10 300 python -u tools/ab_interleave.py human 3e9 20 ab/libB.so 6 0/1 > $O/ab_c3_B.txt 2>&1
timeout -k 10 300 python -u tools/ab_interleave.py human 3e9 20 ab/libC.so 6 0/1 > $O/ab_c3_C.txt 2>&1
timeout -k 10 300 python -u tools/ab_interleave.py human 3e9 20 ab/libB.so 6 3/8 > $O/ab_s3of8_B.txt 2>&1
timeout -k 10 300 python -u tools/ab_interleave.py human 3e9 20 ab/libC.so 6 3/8 > $O/ab_s3of8_C.txt 2>&1
