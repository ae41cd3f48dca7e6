#!/bin/bash
# One SQ-counter PMC pass aimed at LDS / memory waits (8 SQ counters), per-kernel averages.
# usage: tools/pmc_lds.sh TAG
set -euo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS \
    SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY \
    --output-format csv -d "$OUT" -o sq -- python3 "$ROOT/bench.py" --no-cpu-baseline --profile-kernels 0 \
    --steps 3 --warmup 2 "$@" > "$OUT/sq.log" 2>&1
python3 - "$OUT/sq_counter_collection.csv" <<'PY' > "$OUT/sq_summary.txt"
import collections, csv, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "nerf::" not in k:
        continue
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
cat "$OUT/sq_summary.txt"
