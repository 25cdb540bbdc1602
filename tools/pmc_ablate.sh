# SQ instruction counters of K1 under ablation bits (GT_SMAX_DEBUG), 3 Gbp human-like
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"
for v in ${VARIANTS:-0 2 8 4 4096}; do
  GT_SMAX_DEBUG=$v timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex smax_scan -d $R/gpurun_out/pmca_$v -o p -- python3 $R/tools/k1_once.py human ${BASES:-3e9} 2 > $R/gpurun_out/pmca_$v.log 2>&1 || exit 1
done
