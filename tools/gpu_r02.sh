#!/bin/bash
# Round-2 GPU pass: GPU suite, default bench line, rocprofv3 kernel stats + PMC traffic + SQ counters.
# usage: tools/gpu_r02.sh TAG   (everything under gpurun_out/r02_TAG/ and gpurun_out/{prof,sq}_TAG/)
set -eo pipefail
TAG=${1:-r02a}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -3 "$OUT/gpu_tests.log"
fi
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json" | cut -c1-400
bash tools/profile_bench.sh "$TAG"
bash tools/pmc_sq.sh "$TAG" > /dev/null
for wl in ${WORKLOADS:-}; do
  timeout -k 10 200 python -u bench.py --workload $wl --no-cpu-baseline > "$OUT/bench_${wl}.json" 2> "$OUT/bench_${wl}.err"
done
echo "gpu_r02 $TAG done"
