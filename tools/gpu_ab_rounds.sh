# Same box, alternating: this tree's bench against round 5's final tree built under build/ab_old
# (lego three times, then the ScanNet workload twice), JSON lines in gpurun_out/OUT/results.jsonl.
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
run() {  # tree wl round
  if [ $1 = new ]; then d=.; else d=build/ab_old; fi
  echo -n "{\"variant\": \"$1_$2\", \"round\": $3, \"result\": " >> $out/results.jsonl
  (cd $d && timeout -k 10 200 python bench.py --workload $2 --no-cpu-baseline 2> /dev/null | tail -1 | tr -d '\n') >> $out/results.jsonl || exit 1
  echo "}" >> $out/results.jsonl
}
for r in 1 2 3; do run new lego $r && run old lego $r || exit 1; done
for r in 1 2; do run new scannet $r && run old scannet $r || exit 1; done
