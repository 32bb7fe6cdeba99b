# Parity tests, then the VanillaVAE bench (per-kernel breakdown) and the VQ-VAE bench.  Usage: bash scripts/gpu_both.sh TAG
set -o pipefail
TAG=${1:-it}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 240 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --kernel-breakdown > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --arch vq --batch 128 --steps 20 --warmup 3 --no-cpu-baseline --kernel-breakdown > gpurun_out/${TAG}_vq.log 2>&1
