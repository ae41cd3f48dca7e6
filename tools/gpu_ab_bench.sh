# On the GPU box: the lego bench (or BENCH_ARGS) of library variants, alternating, three rounds;
# "default" = the in-tree library, else build/variants/<name>/libnerfhip.so.
# usage: tools/gpu_ab_bench.sh OUT VARIANT...   (JSON lines in gpurun_out/OUT/results.jsonl)
set -o pipefail
out=$1; shift
mkdir -p gpurun_out/$out
for r in 1 2 3; do
  for v in "$@"; do
    if [ $v = default ]; then L=indoor-nerf_amd/libnerfhip.so; else L=build/variants/$v/libnerfhip.so; fi
    echo -n "{\"variant\": \"$v\", \"round\": $r, \"result\": " >> gpurun_out/$out/results.jsonl
    NERF_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline $BENCH_ARGS 2> gpurun_out/$out/$v_$r.err | tail -1 | tr -d '\n' >> gpurun_out/$out/results.jsonl || exit 1
    echo "}" >> gpurun_out/$out/results.jsonl
  done
done
