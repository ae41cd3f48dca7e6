#!/bin/bash
# L2 (TCC) counters per launch of the bench's kernels, split by grid size (the coarse and the fine
# pass's hash_encode_fwd_pair_kernel launches share a symbol but not a grid): hits, misses and the
# read / write requests L2 sends to memory (EA = the Infinity Cache / HBM side). One PMC pass
# (4 TCC counters, the per-pass limit).
# usage: tools/pmc_tcc.sh TAG [bench args...]   (outputs under gpurun_out/tcc_TAG/)
set -euo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/tcc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum \
    --output-format csv -d "$OUT" -o t -- python3 "$ROOT/bench.py" --no-cpu-baseline --profile-kernels 0 \
    --fresh-rays 0 --steps 6 --warmup 3 "$@" > "$OUT/t.log" 2>&1
python3 - "$OUT/t_counter_collection.csv" <<'PY' > "$OUT/tcc_summary.txt"
import collections, csv, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "nerf::" not in k:
        continue
    grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
    acc[(k, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
print("per-launch averages (rocprofv3 --pmc TCC_HIT/MISS/EA0_RDREQ/EA0_WRREQ, bench.py --steps 6 --warmup 3)")
for (k, grid), d in sorted(acc.items()):
    hit, miss = d.get("TCC_HIT_sum", [0]), d.get("TCC_MISS_sum", [0])
    h, m = sum(hit) / len(hit), sum(miss) / len(miss)
    row = {c: round(sum(v) / len(v)) for c, v in sorted(d.items())}
    row["hit_rate"] = round(h / (h + m), 4) if h + m else None
    row["launches"] = max(len(v) for v in d.values())
    print(k, "grid", grid, row)
PY
cat "$OUT/tcc_summary.txt"
