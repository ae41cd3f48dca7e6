set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "hash or train" -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/hash_t.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_o12.json 2> gpurun_out/bench_o12.err || exit 2
NERF_HASH_OWNER=13 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_o13.json 2> gpurun_out/bench_o13.err || exit 3
