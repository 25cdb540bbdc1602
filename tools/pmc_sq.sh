cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-include-regex smax_scan -d $R/gpurun_out/pmc1 -o p -- python3 $R/tools/k1_once.py human 3e9 2 > $R/gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-include-regex smax_scan -d $R/gpurun_out/pmc2 -o p -- python3 $R/tools/k1_once.py human 3e9 2 > $R/gpurun_out/pmc2.log 2>&1
