#!/bin/bash
# The DP equivalence test's measurements (tools/dp_equiv_stats.py) and the deterministic two-rank
# rehearsal run K times (tools/det_repro.py --runs), each rank on its own half of the CUs.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dp_equiv_stats.py gpurun_out/r06_dp_equiv_stats.json > gpurun_out/r06_dp_equiv_stats.log 2>&1 || { echo "stats failed rc=$?"; tail -30 gpurun_out/r06_dp_equiv_stats.log; exit 1; }
grep "^default\|^deterministic" gpurun_out/r06_dp_equiv_stats.log
timeout -k 10 400 python -u tools/det_repro.py gpurun_out/r06_det_dp2_cusplit.json --runs ${1:-8} > gpurun_out/r06_det_dp2_cusplit.log 2>&1 || { echo "repro failed rc=$?"; tail -30 gpurun_out/r06_det_dp2_cusplit.log; exit 1; }
grep "^run" gpurun_out/r06_det_dp2_cusplit.log | cut -c1-300
