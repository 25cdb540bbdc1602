# Block sums fused into K1b (no K2): GPU tests, then A (fused) vs B (K2) interleaved.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fsum
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
for S in 0/1 3/8 2/4; do
  timeout -k 10 300 python -u tools/ab_interleave.py human 3e9 20 ab/libH.so 6 $S > $O/ab_${S/\//of}.txt 2>&1
done
timeout -k 10 300 python -u tools/ab_interleave.py uniform 1e8 20 ab/libH.so 6 0/1 > $O/ab_c2.txt 2>&1
