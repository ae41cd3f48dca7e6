# A/B on the GPU box: owner level order, MLP backward weight-gradient flush cost (outputs under gpurun_out/ab/)
set -o pipefail
mkdir -p gpurun_out/ab
run() { timeout -k 10 200 env "$@" python -u bench.py --no-cpu-baseline > "gpurun_out/ab/${1//=/_}.json" 2> "gpurun_out/ab/${1//=/_}.err"; }
run NERF_AB=base || exit 1
run NERF_OWNER_ORDER=0 || exit 2
run NERF_X6CG_FLUSH=1 || exit 3
run NERF_X6CG_FLUSH=2 || exit 4
run NERF_AB=base2 || exit 5
