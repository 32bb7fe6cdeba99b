# Iteration: new-kernel parity, per-block probe, bench breakdown.  Usage: bash scripts/gpu_r2_iter2.sh TAG
set -o pipefail
TAG=${1:-it}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_cgemm.py tests/test_gpu_adam.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_cg.log 2>&1 || exit $?
VAE_HIP_LIB=probe timeout -k 10 200 python3 -u tools/kprobe.py --out gpurun_out/${TAG}_kp.json > gpurun_out/${TAG}_kp.log 2>&1 || exit $?
timeout -k 10 240 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --kernel-breakdown > gpurun_out/${TAG}_bench.log 2>&1
