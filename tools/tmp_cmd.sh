set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/gpu_tests.log 2>&1
ROUNDS=5 timeout -k 10 400 python tools/k1_env.py human 3e9 '|GT_SMAX_DEBUG=1' > $R/gpurun_out/env.log 2>&1
VARIANTS="0 2" bash tools/pmc_ablate.sh
