cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 16384 16512; do
GT_SMAX_DEBUG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/k1b_$v -o p -- python3 $R/tools/k1_once.py human 3e9 4 > $R/gpurun_out/k1b_$v.log 2>&1 || exit 1
done
