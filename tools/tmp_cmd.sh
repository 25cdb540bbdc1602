# GPU tests, C3 bench (end-to-end leg through the staged H2D), C5-profile
# bench with the CPU oracle over all rows.  Outputs under gpurun_out/h/.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 400 python bench.py --config c5p > $O/bench_c5p.json 2> $O/bench_c5p.err
