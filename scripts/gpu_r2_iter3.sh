# Iteration: new-kernel parity, full GPU suite, bench breakdown.  Usage: bash scripts/gpu_r2_iter3.sh TAG
set -o pipefail
TAG=${1:-it}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_cgemm.py tests/test_gpu_adam.py -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_cg.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_cgemm.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 240 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --kernel-breakdown > gpurun_out/${TAG}_bench.log 2>&1
