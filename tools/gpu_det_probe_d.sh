#!/bin/bash
# Bin launch reproducibility in the two-rank rehearsal (tools/det_repro_d.py): ranks whose device
# buffers sit at the same virtual addresses (the default: both processes allocate alike) vs ranks
# whose allocations are shifted apart (rank 1 first reserves DET_SHIFT_GIB GiB).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
K=${1:-10}
run() {   # tag, extra args...
  local tag=$1; shift
  timeout -k 10 300 python -u tools/det_repro_d.py gpurun_out/r06_det_d_$tag.json --runs $K --reps 3 "$@" > gpurun_out/r06_det_d_$tag.log 2>&1 || { echo "$tag failed rc=$?"; tail -30 gpurun_out/r06_det_d_$tag.log; exit 1; }
  echo "== $tag: $(grep -c '^run' gpurun_out/r06_det_d_$tag.log) rank-runs, $(grep '^run' gpurun_out/r06_det_d_$tag.log | grep -vc ' 0 reruns differ') with a rerun mismatch"
  grep "^streams" gpurun_out/r06_det_d_$tag.log | cut -c1-300
  grep "^run" gpurun_out/r06_det_d_$tag.log | grep -v " 0 reruns differ" | cut -c1-300
}
DET_CU_SPLIT=1 run w2cusplit --world 2
run w2shared --world 2
