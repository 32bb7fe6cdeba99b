# GPU tests only (optionally a -k filter).  Usage: bash scripts/gpu_tests.sh TAG [-k expr]
set -o pipefail
TAG=${1:-t}; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread "$@" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log; exit $rc
