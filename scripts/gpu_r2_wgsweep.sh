# Weight-gradient launch-shape sweep on the VQ-VAE step (per-call breakdown per setting).
# Usage: bash scripts/gpu_r2_wgsweep.sh TAG
set -o pipefail
TAG=${1:-ws}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
run() { name=$1; shift; env "$@" timeout -k 10 200 python3 -u bench.py --arch vq --batch 128 --steps 30 --warmup 5 --no-cpu-baseline --no-dropin --kernel-breakdown > gpurun_out/${TAG}_$name.log 2>&1; }
run base VAE_X=0 || exit $?
run wpc1 VAE_WG_WGPERCU=1 || exit $?
run wpc4 VAE_WG_WGPERCU=4 || exit $?
run mink16 VAE_WG_MINK=16 || exit $?
run nowgemm VAE_NO_WGEMM=1 || exit $?
run slab VAE_WG_SLAB_MIN=8 || exit $?
