# Zero-copy boundary send: runtime tests, 2-rank gloo rehearsal with parity.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/zc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_runtime_gpu.py tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --one-gpu --dist-backend gloo --bases 300000000 --steps 10 --warmup 2 > $O/w2.json 2> $O/w2.err
