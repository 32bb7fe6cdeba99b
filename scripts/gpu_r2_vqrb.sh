# vq_fwd rows-per-workgroup A/B (VAE_VQF_RB 1 = 64 rows, 2 = 128): VQ tests under both, VQ-VAE bench.
# Usage: bash scripts/gpu_r2_vqrb.sh TAG
set -o pipefail
TAG=${1:-rb}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_vq.py -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests2.log 2>&1 || exit $?
VAE_VQF_RB=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_vq.py tests/test_gpu_parity_shapes.py -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests1.log 2>&1 || exit $?
run() { name=$1; shift; env "$@" timeout -k 10 200 python3 -u bench.py --arch vq --batch 128 --steps 30 --warmup 5 --no-cpu-baseline --no-dropin --kernel-breakdown > gpurun_out/${TAG}_$name.log 2>&1; }
run rb2 VAE_VQF_RB=2 || exit $?
run rb1 VAE_VQF_RB=1
