# 2-rank rehearsals of bench.py's multi-GPU path on ONE GPU (both ranks on cuda:0): gloo collectives
# (weak scaling with the ZeRO-1 sharded optimizer, weak with one all-reduce, strong), then the same
# with the nccl backend (RCCL) as the last step. Graph capture + hook between the replays +
# max-over-ranks timing. Outputs: gpurun_out/dist/.
set -o pipefail
mkdir -p gpurun_out/dist
run() {  # name backend args...
  local name=$1 be=$2; shift 2
  NERF_DIST_BACKEND=$be timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) bench.py --gpus 2 --steps 8 --warmup 4 \
      --no-cpu-baseline "$@" > gpurun_out/dist/$name.json 2> gpurun_out/dist/$name.err
}
run gloo_weak_zero gloo --zero 1 || exit 1
run gloo_weak_allreduce gloo --zero 0 || exit 2
run gloo_strong_zero gloo --zero 1 --scaling strong || exit 3
# RCCL refuses two ranks on one GPU ("Duplicate GPU detected", profiles/r02u_dist2_rccl_refused.txt):
# on a 1-GPU box this last step documents the refusal; on a multi-GPU box it runs the real path
run rccl_weak_zero nccl --zero 1 || { grep -m1 "Duplicate GPU" gpurun_out/dist/rccl_weak_zero.err; exit 4; }
