# GPU milestone, part C: the whole GPU suite and smoke (no convergence replays: for changes that keep
# the gradients bit for bit), then part B (bench, profiles, workloads). usage: bash tools/gpu_milestone_c.sh TAG
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 2
bash tools/gpu_milestone_b.sh $TAG || exit 3
echo "milestone C $TAG done"
