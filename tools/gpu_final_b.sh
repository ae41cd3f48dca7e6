# Final GPU pass, measurement half (the suite, smoke() and the convergence replays run in
# tools/gpu_milestone_a.sh): the default bench line (with the CPU baseline and the fresh-ray leg), the
# other workloads and the deterministic lego line, rocprofv3 kernel stats + PMC traffic + SQ counters.
# usage: bash tools/gpu_final_b.sh TAG   (outputs under gpurun_out/TAG/, prof_TAG/, sq_TAG/)
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
for wl in fern acaq scannet; do
  timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || exit 4
done
timeout -k 10 200 python -u bench.py --deterministic 1 --no-cpu-baseline > $OUT/bench_det.json 2> $OUT/bench_det.err || exit 5
timeout -k 10 900 bash tools/profile_bench.sh $TAG --fresh-rays 0 > $OUT/profile.log 2>&1 || exit 6
timeout -k 10 400 bash tools/pmc_sq.sh $TAG --fresh-rays 0 > $OUT/sq.log 2>&1 || exit 7
echo "final $TAG done"
