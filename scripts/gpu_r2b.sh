# Parity re-check, per-block probe and kernel-trace stats of the VanillaVAE bench.  Usage: bash scripts/gpu_r2b.sh TAG
set -o pipefail
TAG=${1:-b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd $R && mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity_shapes.py tests/test_gpu_dp.py -v -s --timeout 300 --timeout-method thread > $O/${TAG}_par.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
VAE_HIP_LIB=probe timeout -k 10 200 python3 -u tools/kprobe.py --out $O/${TAG}_kp.json > $O/${TAG}_kp.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_kt -o run -- python3 $R/bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dropin > $O/${TAG}_kt.log 2>&1
