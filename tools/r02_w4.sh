# 4-rank C3 rehearsal on one GPU (gloo staging; nt window stream on 362K-tile shards) with whole-table parity.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/w4
mkdir -p $O
GT_SMAX_VERBOSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 4 --one-gpu --dist-backend gloo --steps 10 --warmup 2 > $O/w4.json 2> $O/w4.err
