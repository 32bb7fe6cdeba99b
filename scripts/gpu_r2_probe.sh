# Probe + kernel trace of the current HEAD.  Usage: bash scripts/gpu_r2_probe.sh TAG
set -o pipefail
TAG=${1:-p}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_cgemm.py tests/test_gpu_adam.py -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_cg.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
VAE_HIP_LIB=probe timeout -k 10 200 python3 -u tools/kprobe.py --out gpurun_out/${TAG}_kp.json > gpurun_out/${TAG}_kp.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_kt -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-graph > $R/gpurun_out/${TAG}_kt.log 2>&1
