# What the driver runs at round end, on the committed tree: GPU suite, smoke(), default bench.
# Usage: bash scripts/gpu_r2_round_end.sh TAG
set -o pipefail
TAG=${1:-re}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > $O/${TAG}_bench.log 2>&1
