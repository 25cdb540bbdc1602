# Partial nt: LCP-only (L) or packed-BWT-only (P) non-temporal window loads, forced on
# (A, GT_SMAX_NT=1 for plan A only), vs the current build with the default policy (B).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ntpart
mkdir -p $O
for V in L P; do
  cp ab/lib$V.so genometools_smax_amd/lib/libgtsmax_hip.so
  for S in 0/1 3/8; do
    AB_ENV_A=GT_SMAX_NT=1 timeout -k 10 300 python -u tools/ab_interleave.py human 3e9 20 ab/libH.so 6 $S > $O/ab_${V}_${S/\//of}.txt 2>&1
  done
done
