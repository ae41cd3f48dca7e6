# x6 MLP check: accuracy tests first, then the whole GPU suite, then A/B benches (outputs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp_x6.py tests/test_gpu_parity.py -k "mlp or x6" -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gpu_x6_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_x6.json 2> gpurun_out/bench_x6.err || exit 2
NERF_MLP=3 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_f32.json 2> gpurun_out/bench_f32.err || exit 3
NERF_MLP=3 timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 4
