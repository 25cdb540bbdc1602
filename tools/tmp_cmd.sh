# C5-profile bench (plant-like 4.2 Gbp, minlen 50), C3 bench with the all-core
# CPU figure, rocprof kernel stats of the C5-profile bench, and a 2-rank gloo
# rehearsal of the sharded path on one GPU.  Outputs under gpurun_out/g/.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/g
mkdir -p $O
timeout -k 10 400 python bench.py --config c5p > $O/bench_c5p.json 2> $O/bench_c5p.err
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o p -- python3 $R/bench.py --config c5p --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end > $O/bench_c5p_prof.json 2> $O/bench_c5p_prof.err
cd $R
python3 tools/rocpd_summary.py stats $O/prof/p_results.db $O/c5p_kernel_stats.csv
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --one-gpu --bases 1000000000 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_rehearsal_w2.json 2> $O/bench_rehearsal_w2.err
