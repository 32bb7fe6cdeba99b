# Full -m gpu suite, then the round-2 measurements (bench lines, kernel traces, PMC passes).
# Usage: bash scripts/gpu_r2_all.sh TAG
set -o pipefail
TAG=${1:-all}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
bash scripts/gpu_r2_measure.sh ${TAG}
