# VQ-VAE sweep: vq_bwd rows per thread, 128x128 weight-gradient ring depth.  Usage: bash scripts/gpu_r2_sweep3.sh TAG
set -o pipefail
TAG=${1:-s3}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_vq.py -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
run() { name=$1; shift; env "$@" timeout -k 10 200 python3 -u bench.py --arch vq --batch 128 --steps 30 --warmup 5 --no-cpu-baseline --no-dropin --kernel-breakdown > gpurun_out/${TAG}_$name.log 2>&1; }
run base VAE_X=0 || exit $?
run run32 VAE_VQB_RUN=32 || exit $?
run run128 VAE_VQB_RUN=128 || exit $?
run ns3 VAE_WG_NS=3 || exit $?
run ns4 VAE_WG_NS=4 || exit $?
VAE_WG_NS=3 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_vq.py -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests_ns3.log 2>&1
