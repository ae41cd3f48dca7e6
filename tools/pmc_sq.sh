#!/bin/bash
# SQ counters of the bench's kernels in two PMC passes (at most 8 SQ counters per pass):
# A = cycles / waits / busy, B = instruction mix + LDS bank conflicts. Per-kernel averages per launch.
# usage: tools/pmc_sq.sh TAG [bench args...]   (outputs under gpurun_out/sq_TAG/)
set -euo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    --output-format csv -d "$OUT" -o a -- python3 "$ROOT/bench.py" --no-cpu-baseline --profile-kernels 0 \
    --steps 3 --warmup 2 "$@" > "$OUT/a.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM \
    SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAVES \
    --output-format csv -d "$OUT" -o b -- python3 "$ROOT/bench.py" --no-cpu-baseline --profile-kernels 0 \
    --steps 3 --warmup 2 "$@" > "$OUT/b.log" 2>&1
python3 - "$OUT/a_counter_collection.csv" "$OUT/b_counter_collection.csv" <<'PY' > "$OUT/sq_summary.txt"
import collections, csv, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "nerf::" not in k:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
print("per-launch averages (rocprofv3 --pmc, two passes over bench.py --steps 3 --warmup 2)")
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
cat "$OUT/sq_summary.txt"
