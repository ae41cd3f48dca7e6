#!/bin/bash
# On the GPU box: rocprofv3 kernel-trace stats and the two PMC traffic passes of a short bench run.
# usage: tools/profile_bench.sh TAG [BENCH ARGS...]   (outputs under gpurun_out/prof_TAG/)
set -euo pipefail
TAG=${1:-r01}
shift || true
EXTRA=("$@")
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o trace -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --profile-kernels 0 "${EXTRA[@]}" > "$OUT/trace_bench.json" 2> "$OUT/trace.log"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT" -o fetch -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --profile-kernels 0 --steps 5 --warmup 3 "${EXTRA[@]}" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT" -o write -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --profile-kernels 0 --steps 5 --warmup 3 "${EXTRA[@]}" > "$OUT/write.log" 2>&1
python3 "$ROOT/tools/pmc_traffic.py" "$OUT/fetch_counter_collection.csv" "$OUT/write_counter_collection.csv" \
    "$OUT/traffic.json" > /dev/null
python3 "$ROOT/tools/prof_summary.py" "$OUT/trace_kernel_stats.csv" > "$OUT/kernel_stats.md"
echo "profile $TAG done"
