# split-role MLP backward (NERF_MLP=4): x6 accuracy tests under it, then A/B against v3 and the lego bench
set -o pipefail
mkdir -p gpurun_out
NERF_MLP=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp_x6.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpu_cg_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/mlp_ab.py 786432 3,4 > gpurun_out/mlp_ab_cg.json 2> gpurun_out/mlp_ab_cg.err || exit 2
NERF_MLP=4 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_cg.json 2> gpurun_out/bench_cg.err || exit 3
NERF_HIP_LIB=build/prof/libnerfhip_prof.so timeout -k 10 200 python -u tools/mlp_ab.py 786432 4 > gpurun_out/cgprof.json 2> gpurun_out/cgprof.err || exit 4
