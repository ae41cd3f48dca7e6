set -o pipefail
out=${1:-r04ze}
mkdir -p gpurun_out/$out
for r in 1 2 3; do
  for v in ${VARIANTS:-copy spin}; do
    export NERF_DIAG_UPLOAD=$v
    echo -n "{\"variant\": \"$v\", \"round\": $r, \"result\": " >> gpurun_out/$out/results.jsonl
    timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline 2> gpurun_out/$out/${v}_$r.err | tail -1 | tr -d '\n' >> gpurun_out/$out/results.jsonl || exit 1
    echo "}" >> gpurun_out/$out/results.jsonl
  done
done
