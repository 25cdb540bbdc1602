set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/smoke.log 2>&1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo --one-gpu > $R/gpurun_out/bench_2r.json 2> $R/gpurun_out/bench_2r.err
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 3 --steps 5 --warmup 1 --dist-backend gloo --one-gpu --config c2 > $R/gpurun_out/bench_3r.json 2> $R/gpurun_out/bench_3r.err
