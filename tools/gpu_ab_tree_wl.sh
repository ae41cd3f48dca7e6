# this tree vs build/ab_old on one workload (WL), alternating, two rounds: gpurun_out/ab6/
set -o pipefail
mkdir -p gpurun_out/ab6
for r in 1 2; do
  timeout -k 10 200 python bench.py --workload $WL --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/ab6/new_$r.json 2> gpurun_out/ab6/new_$r.err || exit 2
  (cd build/ab_old && timeout -k 10 200 python bench.py --workload $WL --steps 40 --warmup 10 --no-cpu-baseline > ../../gpurun_out/ab6/old_$r.json 2> ../../gpurun_out/ab6/old_$r.err) || exit 3
done
