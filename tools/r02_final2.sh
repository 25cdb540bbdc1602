# Final check after the nt policy: all GPU tests, smoke, default bench, 3-rank C3 rehearsal (nt shards) with parity.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
GT_SMAX_VERBOSE=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 3 --one-gpu --dist-backend gloo --steps 10 --warmup 2 > $O/w3.json 2> $O/w3.err
