#!/bin/bash
# SQ counters of the MLP kernels (tools/mlp_one.py), two passes; usage: tools/pmc_mlp.sh TAG
set -euo pipefail
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/mlp_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    --output-format csv -d "$OUT" -o a -- python3 "$ROOT/tools/mlp_one.py" > "$OUT/a.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM \
    SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAVES \
    --output-format csv -d "$OUT" -o b -- python3 "$ROOT/tools/mlp_one.py" > "$OUT/b.log" 2>&1
python3 - "$OUT/a_counter_collection.csv" "$OUT/b_counter_collection.csv" <<'PY' > "$OUT/summary.txt"
import collections, csv, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "mlp" not in k:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
cat "$OUT/summary.txt"
