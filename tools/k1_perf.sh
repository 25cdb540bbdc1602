# K1 iteration loop on the GPU box: parity tests, K1 time (3 Gbp human-like),
# SQ instruction counters of K1.  Usage: bash tools/k1_perf.sh [variants]
set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python tools/k1_ablate.py human 3e9 ${1:-0} > $R/gpurun_out/ablate.log 2>&1
cd /tmp && export TMPDIR=/tmp
P="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"
timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex smax_scan -d $R/gpurun_out/pmcp -o p -- python3 $R/tools/k1_once.py human 3e9 2 > $R/gpurun_out/pmcp.log 2>&1
