# K1b window loads non-temporal (A) vs default (B = ab/libH.so), interleaved; smax tests.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/k1bnt
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_smax_gpu.py tests/test_runtime_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for S in 0/1 3/8; do
  timeout -k 10 300 python -u tools/ab_interleave.py human 3e9 20 ab/libH.so 6 $S > $O/ab_${S/\//of}.txt 2>&1
done
timeout -k 10 300 python -u tools/ab_interleave.py uniform 1e8 20 ab/libH.so 6 0/1 > $O/ab_c2.txt 2>&1
