# bf16 gradient test with and without the padded RGB path, then both benches.
set -o pipefail
TAG=${1:-pc}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
VAE_NO_PAD_RGB=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_step.py -m gpu -q -k "bf16_gradients" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_nopad.log 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 240 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --kernel-breakdown > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --arch vq --batch 128 --steps 20 --warmup 3 --no-cpu-baseline --kernel-breakdown > gpurun_out/${TAG}_vq.log 2>&1
