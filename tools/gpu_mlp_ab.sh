# On the GPU box: tools/mlp_ab.py against each library variant under build/variants/, alternating,
# three rounds; JSON lines in gpurun_out/mlp_ab/results.jsonl.
# usage: tools/gpu_mlp_ab.sh VARIANT...
set -o pipefail
mkdir -p gpurun_out/mlp_ab
for r in 1 2 3; do
  for v in "$@"; do
    NERF_HIP_LIB=build/variants/$v/libnerfhip.so timeout -k 10 120 python tools/mlp_ab.py >> gpurun_out/mlp_ab/results.jsonl 2>> gpurun_out/mlp_ab/err.log || exit 1
    echo "round $r $v done"
  done
done
