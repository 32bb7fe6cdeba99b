# Kernel trace (timestamps) of a short graph-replayed bench.  Usage: bash scripts/gpu_trace.sh TAG [bench args]
set -o pipefail
TAG=${1:-tr}
shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG} -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $R/gpurun_out/${TAG}.log 2>&1
