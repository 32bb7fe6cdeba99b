# tests + bench + kernel-trace profile + per-block probe.  Usage: bash scripts/gpu_iter_prof.sh TAG
set -o pipefail
TAG=${1:-it}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 240 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit $?
cd $R && VAE_HIP_LIB=probe timeout -k 10 200 python3 -u tools/kprobe.py --out gpurun_out/${TAG}_kp.json > gpurun_out/${TAG}_kp.log 2>&1
