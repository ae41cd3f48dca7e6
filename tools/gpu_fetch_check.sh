set -o pipefail
mkdir -p gpurun_out/r04zd
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_graphs.py tests/test_gpu_scalars_fetch.py > gpurun_out/r04zd/graphs.log 2>&1 || { tail -30 gpurun_out/r04zd/graphs.log; exit 1; }
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline 2> gpurun_out/r04zd/bench_$r.err | tail -1 >> gpurun_out/r04zd/results.jsonl || exit 1
done
