set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
for i in 1 2; do
NERF_HASH_FWD=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ab_old_$i.json 2>/dev/null || exit 2
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ab_new_$i.json 2>/dev/null || exit 3
done
