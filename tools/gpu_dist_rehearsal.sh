# 2-rank rehearsal of bench.py's multi-GPU path on ONE GPU (gloo all-reduce, both ranks on cuda:0):
# graph capture + all-reduce hook between the replays + max-over-ranks timing (no RCCL here; the
# driver's 8-GPU node runs the nccl backend)
set -o pipefail
mkdir -p gpurun_out
NERF_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 6 --warmup 4 \
    > gpurun_out/bench_dist2.json 2> gpurun_out/bench_dist2.err || exit 1
