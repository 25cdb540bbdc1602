# Round evidence on the GPU box: K1 HBM traffic (FETCH_SIZE / WRITE_SIZE in
# separate --pmc passes, used by the bench line's roofline), all GPU tests,
# the default bench line (C3), C2 and C5 bench lines, and the rocprofv3
# kernel-trace summary of the C3 bench.  Outputs under gpurun_out/round/.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex smax_scan_kernel -d $O/pmc_$C -o p -- python3 $R/tools/k1_once.py human 3e9 5 > $O/pmc_$C.log 2>&1
done
cd $R
python3 tools/rocpd_summary.py pmc $O/pmc.json smax_scan_kernel $O/pmc_FETCH_SIZE/p_results.db $O/pmc_WRITE_SIZE/p_results.db
cp $O/pmc.json profiles/pmc_c3_n1.json
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --config c2 > $O/bench_c2.json 2> $O/bench_c2.err
GT_SMAX_VERBOSE=1 timeout -k 10 600 python -u bench.py --config c5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end > $O/bench_prof.json 2> $O/bench_prof.err
cd $R
python3 tools/rocpd_summary.py stats $O/prof/p_results.db $O/kernel_stats.csv
