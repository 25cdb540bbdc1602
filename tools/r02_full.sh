# Full GPU check: all GPU tests, C3 bench, C5 bench, rocprofv3 kernel stats of both.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/full
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err
GT_SMAX_VERBOSE=1 timeout -k 10 600 python -u bench.py --config c5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof3 -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end > $O/prof_c3.json 2> $O/prof_c3.err
cd $R
python3 tools/rocpd_summary.py stats $O/prof3/p_results.db $O/kernel_stats_c3.csv
