# GPU suite + default bench, the point-major forward A/B (time + FETCH_SIZE), then the default tree's
# rocprofv3 profile. Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out/ab2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 2
NERF_HIP_LIB=build/variants/pointmajor/libnerfhip.so timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/ab2/bench_pointmajor.json 2> gpurun_out/ab2/bench_pointmajor.err || exit 3
timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/ab2/bench_default.json 2> gpurun_out/ab2/bench_default.err || exit 4
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
NERF_HIP_LIB=$ROOT/build/variants/pointmajor/libnerfhip.so timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/gpurun_out/ab2 -o pm_fetch -- python3 $ROOT/bench.py --no-cpu-baseline --profile-kernels 0 --steps 5 --warmup 3 > $ROOT/gpurun_out/ab2/pm_fetch.log 2>&1 || exit 5
cd $ROOT
timeout -k 10 900 bash tools/profile_bench.sh r02s || exit 6
