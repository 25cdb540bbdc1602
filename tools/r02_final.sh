# Final check: all GPU tests, smoke, default bench, K1 event overhead.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -u tools/timing_overhead.py human 3e9 20 3/8 > $O/ev_s3of8.txt 2>&1
timeout -k 10 300 python -u tools/timing_overhead.py human 3e9 20 0/1 > $O/ev_c3.txt 2>&1
