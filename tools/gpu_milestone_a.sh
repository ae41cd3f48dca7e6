# GPU milestone, part A: the whole GPU suite, then the convergence replays of every F19c/F19d seed
# (K=2) and their summary (profiles/<tag>_psnr_vs_reference.json). usage: bash tools/gpu_milestone_a.sh TAG
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 2
SEEDS=$(python -c "print(','.join(str(s) for s in list(range(100, 148)) + list(range(200, 304))))")
timeout -k 10 600 python -u tools/converge_hip.py --runs 2 --iters 300 --batch-seeds $SEEDS --out $OUT/hip.npz > $OUT/hip.log 2>&1 || exit 3
python tools/converge_seed_stats.py $OUT/hip.npz --json $OUT/psnr_vs_reference.json --commit "$(cat build/COMMIT)" > $OUT/stats.log 2>&1 || exit 4
echo "milestone A $TAG done"
