# A/B of library builds on the lego step: owner_ab (bin / owner launch times, plain and deterministic)
# and a short bench per build. Usage: bash tools/ab_chunks.sh OUTDIR default c512 ... (build/variants/<name>)
set -e
out=$1; shift
mkdir -p gpurun_out/$out
for v in "$@"; do
  if [ $v = default ]; then L=indoor-nerf_amd/libnerfhip.so; else L=build/variants/$v/libnerfhip.so; fi
  NERF_HIP_LIB=$L timeout -k 10 120 python tools/owner_ab.py > gpurun_out/$out/ab_$v.json
  NERF_DET=1 NERF_HIP_LIB=$L timeout -k 10 120 python tools/owner_ab.py > gpurun_out/$out/ab_${v}_det.json
  NERF_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/$out/bench_$v.json
done
