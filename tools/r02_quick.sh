# Quick GPU check: smax GPU tests, bench, rocprofv3 kernel stats of the bench.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_smax_gpu.py tests/test_configs_gpu.py tests/test_runtime_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py --no-end-to-end > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end > $O/bench_prof.json 2> $O/bench_prof.err
cd $R
python3 tools/rocpd_summary.py stats $O/prof/p_results.db $O/kernel_stats.csv
