# GPU milestone, part B: the default bench line (with the CPU baseline), rocprofv3 kernel stats + PMC
# traffic + SQ counters of it, and the A-CAQ render workload (int-packed gather) with its own profile.
# usage: bash tools/gpu_milestone_b.sh TAG
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 900 bash tools/profile_bench.sh $TAG > $OUT/profile.log 2>&1 || exit 2
timeout -k 10 400 bash tools/pmc_sq.sh $TAG > $OUT/sq.log 2>&1 || exit 3
timeout -k 10 200 python -u bench.py --workload acaq --mode render --no-cpu-baseline > $OUT/bench_acaq_render.json 2> $OUT/bench_acaq_render.err || exit 4
timeout -k 10 900 bash tools/profile_bench.sh ${TAG}_acaq_render --workload acaq --mode render > $OUT/profile_acaq.log 2>&1 || exit 5
for wl in fern acaq scannet; do
  timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || exit 6
done
timeout -k 10 200 python -u bench.py --deterministic 1 --no-cpu-baseline > $OUT/bench_det.json 2> $OUT/bench_det.err || exit 7
echo "milestone B $TAG done"
