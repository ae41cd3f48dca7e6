# On the GPU box: HIP replays of every F19c/F19d seed (default library, K=2), the same with fp32 owner
# sums (build/variants/acc32) and in deterministic mode (K=1, runs are identical), then the GPU suite.
# usage: bash tools/gpu_converge_final.sh SEEDS   (comma list; outputs under gpurun_out/conv_final/)
set -o pipefail
SEEDS=$1
OUT=gpurun_out/conv_final
mkdir -p $OUT
timeout -k 10 400 python -u tools/converge_hip.py --runs 2 --iters 300 --batch-seeds $SEEDS --out $OUT/hip.npz > $OUT/hip.log 2>&1 || exit 1
NERF_HIP_LIB=build/variants/acc32/libnerfhip.so timeout -k 10 400 python -u tools/converge_hip.py --runs 2 --iters 300 --batch-seeds $SEEDS --out $OUT/hip_acc32.npz > $OUT/hip_acc32.log 2>&1 || exit 2
timeout -k 10 400 python -u tools/converge_hip.py --runs 1 --iters 300 --deterministic --batch-seeds $SEEDS --out $OUT/hip_det.npz > $OUT/hip_det.log 2>&1 || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 4
