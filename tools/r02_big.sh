# >2^32-row GPU tests and a 2-rank (gloo, one GPU) rehearsal of the sharded bench.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/big
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_big_gpu.py -x -v --timeout 400 --timeout-method thread > $O/big_tests.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --one-gpu --dist-backend gloo --bases 300000000 --steps 10 --warmup 2 > $O/rehearsal_w2.json 2> $O/rehearsal_w2.err
