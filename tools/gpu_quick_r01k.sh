# GPU suite + lego bench + rocprofv3 kernel trace of the bench (outputs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out/k
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/k/bench.json 2> gpurun_out/k/bench.err || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/k" -o trace -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --profile-kernels 0 > "$GRAFT_REPO_ROOT/gpurun_out/k/trace_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/k/trace.log" || exit 3
