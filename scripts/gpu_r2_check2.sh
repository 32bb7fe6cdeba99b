# Column-sum check (rocprofv3 stats on the VQ-VAE step), VanillaVAE per-call breakdown, 2-rank bench.
# Usage: bash scripts/gpu_r2_check2.sh TAG
set -o pipefail
TAG=${1:-c2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_vq.py tests/test_gpu_ops.py -q --timeout 120 --timeout-method thread > $O/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --kernel-breakdown > $O/${TAG}_van.log 2>&1 || exit $?
timeout -k 10 200 python3 -u bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline --no-dropin > $O/${TAG}_van_2rank.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_ktvq -o run -- python3 $R/bench.py --arch vq --batch 128 --steps 10 --warmup 3 --no-cpu-baseline --no-dropin > $O/${TAG}_ktvq.log 2>&1
