# VQ kernels: parity tests, VQ-VAE and VanillaVAE bench lines with per-call breakdown.
# Usage: bash scripts/gpu_r2_vq2.sh TAG
set -o pipefail
TAG=${1:-vq}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_vq.py tests/test_gpu_parity_shapes.py -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --arch vq --batch 128 --steps 50 --warmup 5 --no-cpu-baseline --kernel-breakdown > gpurun_out/${TAG}_vq.log 2>&1 || exit $?
timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --kernel-breakdown > gpurun_out/${TAG}_van.log 2>&1
