# Full GPU suite (-m gpu, verbose with durations), then the bench with its breakdown.
# Usage: bash scripts/gpu_r2_full.sh TAG
set -o pipefail
TAG=${1:-full}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -s --durations=15 --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --kernel-breakdown > gpurun_out/${TAG}_bench.log 2>&1
