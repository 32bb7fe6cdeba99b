# Round-2 closing run: full GPU suite, then every bench line + rocprofv3 stats + PMC passes.
# Usage: bash scripts/gpu_r2_final.sh TAG
set -o pipefail
TAG=${1:-fin}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
bash scripts/gpu_r2_measure.sh $TAG
