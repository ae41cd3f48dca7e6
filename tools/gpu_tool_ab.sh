# On the GPU box: a timing tool (python script printing one JSON line) against library variants
# (build/variants/<name>/libnerfhip.so; "default" = the in-tree library), alternating, three rounds.
# usage: tools/gpu_tool_ab.sh OUT SCRIPT VARIANT...   (JSON lines in gpurun_out/OUT/results.jsonl)
set -o pipefail
out=$1; script=$2; shift 2
mkdir -p gpurun_out/$out
for r in 1 2 3; do
  for v in "$@"; do
    if [ $v = default ]; then L=indoor-nerf_amd/libnerfhip.so; else L=build/variants/$v/libnerfhip.so; fi
    echo -n "{\"variant\": \"$v\", \"round\": $r, \"result\": " >> gpurun_out/$out/results.jsonl
    NERF_HIP_LIB=$L timeout -k 10 120 python $script | tail -1 | tr -d '\n' >> gpurun_out/$out/results.jsonl || exit 1
    echo "}" >> gpurun_out/$out/results.jsonl
    echo "round $r $v done"
  done
done
