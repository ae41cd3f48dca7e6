# Same box, alternating: bench variants given as DIR:ENV (DIR = a tree with its own built library, "."
# for this one; ENV = one VAR=VALUE or "-"), JSON lines in gpurun_out/OUT/results.jsonl.
# usage: tools/gpu_ab_mix.sh OUT ROUNDS WORKLOAD DIR:ENV ...
set -o pipefail
out=$PWD/gpurun_out/$1; rounds=$2; wl=$3; shift 3
mkdir -p $out
for r in $(seq $rounds); do
  for v in "$@"; do
    d=${v%%:*}; e=${v#*:}; [ "$e" = "-" ] && e="NERF_AB_NONE=1"
    echo -n "{\"variant\": \"${wl}_$v\", \"round\": $r, \"result\": " >> $out/results.jsonl
    (cd $d && env $e timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline $BENCH_ARGS 2> /dev/null | tail -1 | tr -d '\n') >> $out/results.jsonl || exit 1
    echo "}" >> $out/results.jsonl
  done
done
