# Full GPU suite + VanillaVAE and VQ-VAE bench lines with per-call breakdown.  Usage: bash scripts/gpu_r2_check.sh TAG
set -o pipefail
TAG=${1:-ck}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 240 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --kernel-breakdown > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --arch vq --batch 128 --steps 50 --warmup 5 --no-cpu-baseline --kernel-breakdown > gpurun_out/${TAG}_vq.log 2>&1
