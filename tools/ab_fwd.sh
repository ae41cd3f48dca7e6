# A/B of library builds (build/variants/<name>) on the lego bench: per-kernel times per build,
# then the hash parity tests against each build named in PARITY. Usage: bash tools/ab_fwd.sh OUT v1 v2 ...
set -o pipefail
out=$1; shift
mkdir -p gpurun_out/$out
for v in "$@"; do
  L=build/variants/$v/libnerfhip.so
  NERF_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/$out/bench_$v.json 2> gpurun_out/$out/bench_$v.err || exit 1
done
for v in $PARITY; do
  NERF_HIP_LIB=build/variants/$v/libnerfhip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "hash or train_step or render" > gpurun_out/$out/parity_$v.log 2>&1 || exit 2
done
