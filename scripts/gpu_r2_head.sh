# Head backward slab change: full GPU suite, VanillaVAE + IWAE bench lines, rocprofv3 stats.
# Usage: bash scripts/gpu_r2_head.sh TAG
set -o pipefail
TAG=${1:-hd}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 20 --kernel-breakdown > $O/${TAG}_vanilla.log 2>&1 || exit $?
timeout -k 10 240 python3 -u bench.py --arch iwae --batch 64 --steps 100 --warmup 10 --no-cpu-baseline > $O/${TAG}_iwae.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_kt -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin > $O/${TAG}_kt.log 2>&1
