# Weight-gradient K-slice quantisation A/B (VAE_WG_NOQUANT) on VQ-VAE and VanillaVAE, then GPU suite.
# Usage: bash scripts/gpu_r2_quant.sh TAG
set -o pipefail
TAG=${1:-q}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
run() { name=$1; shift; env "$@" timeout -k 10 200 python3 -u bench.py --arch vq --batch 128 --steps 30 --warmup 5 --no-cpu-baseline --no-dropin --kernel-breakdown > gpurun_out/${TAG}_vq_$name.log 2>&1 &&
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-dropin --kernel-breakdown > gpurun_out/${TAG}_van_$name.log 2>&1; }
run quant VAE_X=0 || exit $?
run noquant VAE_WG_NOQUANT=1 || exit $?
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
