# Round 4's A/B of the captured step's scalar upload (profiles/r04zc_diag_constant_jitter.jsonl,
# profiles/r04zf_ab_upload.jsonl). The NERF_DIAG_UPLOAD modes it selects (copy / event / spin / none)
# were a temporary switch in graphs.StepScalars, removed once "spin" (the in-graph fetch) was adopted:
# re-running it needs that switch patched back in. usage: bash tools/gpu_ab_upload.sh OUT
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
