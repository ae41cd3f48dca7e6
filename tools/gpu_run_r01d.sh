# round-1 GPU check: parity tests, then the workload benches (outputs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
for wl in ${WORKLOADS:-lego fern acaq}; do
  timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > gpurun_out/bench_${wl}.json 2> gpurun_out/bench_${wl}.err || exit 2
done
for wl in ${RENDER_WORKLOADS:-lego acaq}; do
  timeout -k 10 200 python -u bench.py --workload $wl --mode render --no-cpu-baseline > gpurun_out/bench_${wl}_render.json 2> gpurun_out/bench_${wl}_render.err || exit 3
done
