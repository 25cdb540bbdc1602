# Pipelined passes: runtime GPU tests, the default bench line (pipelined + serial), C2.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pipe
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_runtime_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python bench.py --no-end-to-end > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --config c2 --no-end-to-end > $O/bench_c2.json 2> $O/bench_c2.err
