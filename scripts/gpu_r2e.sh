# Quick: GEMM/VQ tests, VQ-VAE bench with breakdown, VanillaVAE bench.  Usage: bash scripts/gpu_r2e.sh TAG
set -o pipefail
TAG=${1:-e}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_cgemm.py tests/test_gpu_vq.py -q -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_cg.log 2>&1 || exit $?
timeout -k 10 200 python3 -u bench.py --arch vq --batch 128 --steps 30 --warmup 5 --no-cpu-baseline --no-dropin --kernel-breakdown > gpurun_out/${TAG}_vq.log 2>&1 || exit $?
timeout -k 10 120 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-dropin > gpurun_out/${TAG}_bench.log 2>&1
