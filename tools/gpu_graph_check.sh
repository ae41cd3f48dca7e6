# graph-mode check: graph parity tests, then eager vs graph bench lines (outputs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_graph_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --graph 0 > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err || exit 2
timeout -k 10 200 python -u bench.py --no-cpu-baseline --graph 1 > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err || exit 3
timeout -k 10 200 python -u bench.py --no-cpu-baseline --graph 1 --profile-kernels 0 > gpurun_out/bench_graph_np.json 2> gpurun_out/bench_graph_np.err || exit 4
