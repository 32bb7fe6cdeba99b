# Weight-gradient K-slice floor sweep on VQ-VAE and VanillaVAE.  Usage: bash scripts/gpu_r2_wgsweep2.sh TAG
set -o pipefail
TAG=${1:-ws}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
run() { name=$1; shift; env "$@" timeout -k 10 200 python3 -u bench.py --arch vq --batch 128 --steps 30 --warmup 5 --no-cpu-baseline --no-dropin --kernel-breakdown > gpurun_out/${TAG}_vq_$name.log 2>&1 &&
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-dropin --kernel-breakdown > gpurun_out/${TAG}_van_$name.log 2>&1; }
run base VAE_X=0 || exit $?
run mink16 VAE_WG_MINK=16 || exit $?
run mink32 VAE_WG_MINK=32 || exit $?
run mink64 VAE_WG_MINK=64 || exit $?
run mink16w1 VAE_WG_MINK=16 VAE_WG_WGPERCU=1 || exit $?
