# On the GPU box: the bench with different argument sets, alternating, ROUNDS rounds (default 3), one
# library (the in-tree one). usage: tools/gpu_ab_args.sh OUT "name=ARGS" "name=ARGS" ...
# (JSON lines in gpurun_out/OUT/results.jsonl)
set -o pipefail
out=$1; shift
mkdir -p gpurun_out/$out
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in "$@"; do
    name=${v%%=*}; args=${v#*=}
    echo -n "{\"variant\": \"$name\", \"args\": \"$args\", \"round\": $r, \"result\": " >> gpurun_out/$out/results.jsonl
    timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline $args 2> gpurun_out/$out/${name}_$r.err | tail -1 | tr -d '\n' >> gpurun_out/$out/results.jsonl || exit 1
    echo "}" >> gpurun_out/$out/results.jsonl
  done
done
