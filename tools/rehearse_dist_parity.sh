set -e
O=gpurun_out/reh; mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --one-gpu --dist-backend gloo --bases 300000000 --steps 10 --warmup 2 > $O/w2.json 2> $O/w2.err
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 3 --one-gpu --dist-backend gloo --steps 10 --warmup 2 > $O/w3.json 2> $O/w3.err
