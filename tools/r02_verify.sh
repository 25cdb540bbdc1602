# Re-entry check on the GPU box: all GPU tests and the default bench line (C3).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/verify
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
