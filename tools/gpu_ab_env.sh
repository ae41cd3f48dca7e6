# Same box, alternating: this tree's bench under environment variants, JSON lines in
# gpurun_out/OUT/results.jsonl. usage: tools/gpu_ab_env.sh OUT ROUNDS WORKLOAD "ENV=.." "ENV=.." ...
set -o pipefail
out=gpurun_out/$1; rounds=$2; wl=$3; shift 3
mkdir -p $out
for r in $(seq $rounds); do
  for v in "$@"; do
    echo -n "{\"variant\": \"${wl}_$v\", \"round\": $r, \"result\": " >> $out/results.jsonl
    env $v timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline $BENCH_ARGS 2> /dev/null | tail -1 | tr -d '\n' >> $out/results.jsonl || exit 1
    echo "}" >> $out/results.jsonl
  done
done
