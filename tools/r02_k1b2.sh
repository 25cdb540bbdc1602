# K1b per-tile cycle stages incl. inside the window load (C3), plus the smax GPU tests.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/k1b2
mkdir -p $O
timeout -k 10 300 python -u tools/k1b_cycles.py human 3e9 20 0 0/1 > $O/c3.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_smax_gpu.py tests/test_runtime_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
