# L2 hit/miss and memory-side read requests per kernel (one PMC pass; no trace domains).
# Usage: bash scripts/gpu_pmc_l2.sh TAG
set -o pipefail
TAG=${1:-l2}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $R/gpurun_out/${TAG} -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-graph > $R/gpurun_out/${TAG}.log 2>&1
