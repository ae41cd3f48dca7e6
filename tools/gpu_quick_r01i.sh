# GPU suite + lego bench + A/B of the previous reduction cost (outputs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ab/red_new.json 2> gpurun_out/ab/red_new.err || exit 2
timeout -k 10 200 env NERF_X6CG_FLUSH=2 python -u bench.py --no-cpu-baseline > gpurun_out/ab/red_skip.json 2> gpurun_out/ab/red_skip.err || exit 3
