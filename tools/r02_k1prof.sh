# K1 ablation timings + SQ counters at C3 (current build)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/k1
timeout -k 10 300 python tools/k1_ablate.py human 3e9 0,2,8,4,4096,1 > $R/gpurun_out/k1/ablate.txt 2>&1
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-include-regex smax_scan -d $R/gpurun_out/k1/pmc1 -o p -- python3 $R/tools/k1_once.py human 3e9 2 > $R/gpurun_out/k1/pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-include-regex smax_scan -d $R/gpurun_out/k1/pmc2 -o p -- python3 $R/tools/k1_once.py human 3e9 2 > $R/gpurun_out/k1/pmc2.log 2>&1
cd $R
python3 tools/pmc_table.py smax_scan gpurun_out/k1/pmc1/p_results.db gpurun_out/k1/pmc2/p_results.db > gpurun_out/k1/pmc.txt
