set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-end-to-end > $R/gpurun_out/bench.json 2> $R/gpurun_out/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_nt -o p -- python3 $R/tools/k1_once.py human 3e9 6 > $R/gpurun_out/once.log 2>&1
