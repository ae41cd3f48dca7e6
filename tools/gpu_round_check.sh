# full GPU suite, then the workload bench lines (outputs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 2
for wl in ${WORKLOADS:-fern acaq scannet}; do
  timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > gpurun_out/bench_${wl}.json 2> gpurun_out/bench_${wl}.err || exit 3
done
