# rehearsal of bench.py's multi-rank path (shards, graph replay, stats all_reduce every 300 steps,
# barrier, max over ranks) with 2 ranks sharing the box's one GPU over gloo
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FUTBOL_SHARE_DEVICE=1 FUTBOL_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 600 --warmup 20 \
    --envs 32768 > gpurun_out/bench_2rank.log 2>&1
