# VQ tests + VQ bench.  Usage: bash scripts/gpu_vq.sh TAG
set -o pipefail
TAG=${1:-vq}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vq.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --arch vq --batch 128 --steps 20 --warmup 3 --cpu-seconds 10 --kernel-breakdown > gpurun_out/${TAG}_bench.log 2>&1
