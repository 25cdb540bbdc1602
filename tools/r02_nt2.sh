# nt policy A/B on the 2- and 4-way splits and two more 8-way shards.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/nt2
mkdir -p $O
for S in 1/2 2/4 0/8 5/8; do
  timeout -k 10 300 python -u tools/ab_interleave.py human 3e9 20 ab/libB.so 6 $S > $O/ab_${S/\//of}.txt 2>&1
done
