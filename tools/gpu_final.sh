# Final GPU pass of a round: GPU suite, smoke(), the default bench line (with the CPU baseline), the
# other workloads and the deterministic lego line, rocprofv3 kernel stats + PMC traffic + SQ counters.
# usage: bash tools/gpu_final.sh TAG   (outputs under gpurun_out/TAG/, prof_TAG/, sq_TAG/)
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
for wl in fern acaq scannet; do
  timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || exit 4
done
timeout -k 10 200 python -u bench.py --deterministic 1 --no-cpu-baseline > $OUT/bench_det.json 2> $OUT/bench_det.err || exit 5
timeout -k 10 900 bash tools/profile_bench.sh $TAG > $OUT/profile.log 2>&1 || exit 6
timeout -k 10 400 bash tools/pmc_sq.sh $TAG > $OUT/sq.log 2>&1 || exit 7
echo "final $TAG done"
