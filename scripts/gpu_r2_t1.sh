# 1x1 weight-gradient tile sweep (VAE_WG_T1X1) x K-slice floor on the VQ-VAE step.  Usage: bash scripts/gpu_r2_t1.sh TAG
set -o pipefail
TAG=${1:-t1}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
run() { name=$1; shift; env "$@" timeout -k 10 200 python3 -u bench.py --arch vq --batch 128 --steps 30 --warmup 5 --no-cpu-baseline --no-dropin --kernel-breakdown > gpurun_out/${TAG}_$name.log 2>&1; }
run base VAE_X=0 || exit $?
run t64 VAE_WG_T1X1=64 || exit $?
run t64m8 VAE_WG_T1X1=64 VAE_WG_MINK=8 || exit $?
run t32 VAE_WG_T1X1=32 || exit $?
VAE_WG_T1X1=64 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_vq.py -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
