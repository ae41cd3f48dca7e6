#!/bin/bash
# On the GPU box: FETCH_SIZE / WRITE_SIZE calibration per access width (tools/fetch_calib.hip), one PMC
# counter per pass. usage: tools/pmc_calib.sh TAG   (outputs under gpurun_out/calib_TAG/)
set -euo pipefail
TAG=${1:-r03}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/calib_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT" -o fetch -- "$ROOT/build/fetch_calib" > "$OUT/calib.json" 2> "$OUT/fetch.log"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT" -o write -- "$ROOT/build/fetch_calib" > /dev/null 2> "$OUT/write.log"
python3 "$ROOT/tools/fetch_calib.py" "$OUT/fetch_counter_collection.csv" "$OUT/write_counter_collection.csv" "$OUT/calib.json" > "$OUT/ratios.json"
echo "calib $TAG done"
