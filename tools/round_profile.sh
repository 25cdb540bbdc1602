# Round-end evidence on the GPU box: GPU tests, the default bench line, the
# rocprofv3 kernel-trace summary of the same bench, and K1's HBM traffic
# (FETCH_SIZE / WRITE_SIZE in separate --pmc passes).  Outputs under
# gpurun_out/round/.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end > $O/bench_prof.json 2> $O/bench_prof.err
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex smax_scan_kernel -d $O/pmc_$C -o p -- python3 $R/tools/k1_once.py human 3e9 5 > $O/pmc_$C.log 2>&1
done
cd $R
python3 tools/rocpd_summary.py stats $O/prof/p_results.db $O/kernel_stats.csv
python3 tools/rocpd_summary.py pmc $O/pmc.json smax_scan_kernel $O/pmc_FETCH_SIZE/p_results.db $O/pmc_WRITE_SIZE/p_results.db
