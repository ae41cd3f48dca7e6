# GPU suite of this tree, then the lego bench of this tree and of an older tree built under
# build/ab_old (same box, alternating), outputs under gpurun_out/ab3/.
set -o pipefail
mkdir -p gpurun_out/ab3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/ab3/bench_new_$r.json 2> gpurun_out/ab3/bench_new_$r.err || exit 2
  (cd build/ab_old && timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline > ../../gpurun_out/ab3/bench_old_$r.json 2> ../../gpurun_out/ab3/bench_old_$r.err) || exit 3
done
