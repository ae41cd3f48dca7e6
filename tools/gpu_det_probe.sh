#!/bin/bash
# Deterministic two-rank rehearsal (test_gpu_dist.py's _dp_worker, ZeRO-1 + overlap + gated all-gather,
# 7 steps) run K times with stream-ordered buffer checksums, each run compared with the first
# (tools/det_repro_c.py); $2: library variants to repeat it with (build/variants/<name>/libnerfhip.so).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
K=${1:-10}
for v in base $2; do
  if [ "$v" = base ]; then unset NERF_HIP_LIB; else export NERF_HIP_LIB=$PWD/build/variants/$v/libnerfhip.so; fi
  timeout -k 10 300 python -u tools/det_repro_c.py gpurun_out/r06_det_c_$v.json --runs $K > gpurun_out/r06_det_c_$v.log 2>&1 || { echo "$v failed rc=$?"; tail -30 gpurun_out/r06_det_c_$v.log; exit 1; }
  echo "== $v"; grep "^run [1-9]\|distinct" gpurun_out/r06_det_c_$v.log | cut -c1-300
done
