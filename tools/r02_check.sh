# Round-2 check on the GPU box: GPU tests, default bench, e2e phases over
# repeated calls, .llv window statistics at C3 (K1b static list sizing).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python tools/e2e_breakdown.py > $O/e2e.txt 2>&1
timeout -k 10 300 python tools/defer_stats.py human 3e9 > $O/defer_stats.txt 2>&1
