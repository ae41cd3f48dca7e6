# A/B of library builds (build/variants/<name>, "default" = the in-tree library) on the lego bench,
# alternating over two rounds; outputs gpurun_out/<OUT>/bench_<name>_<round>.json.
set -o pipefail
out=$1; shift
mkdir -p gpurun_out/$out
for r in 1 2; do
  for v in "$@"; do
    if [ $v = default ]; then L=indoor-nerf_amd/libnerfhip.so; else L=build/variants/$v/libnerfhip.so; fi
    NERF_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/$out/bench_${v}_$r.json 2> gpurun_out/$out/bench_${v}_$r.err || exit 1
  done
done
