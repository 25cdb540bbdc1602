# Timing-stride check: runtime GPU tests and the default bench line.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/stride
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_runtime_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python bench.py --no-end-to-end > $O/bench.json 2> $O/bench.err
timeout -k 10 400 python bench.py --no-end-to-end > $O/bench2.json 2> $O/bench2.err
