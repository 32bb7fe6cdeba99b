set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_vq.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/ws_tests.log 2>&1 || exit $?
for cap in 32 64 128 256; do
  VAE_WGRAD_SPLITCAP=$cap timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --kernel-breakdown > gpurun_out/ws_v_$cap.log 2>&1 || exit $?
  VAE_WGRAD_SPLITCAP=$cap timeout -k 10 200 python -u bench.py --arch vq --batch 128 --steps 10 --warmup 3 --no-cpu-baseline --kernel-breakdown > gpurun_out/ws_q_$cap.log 2>&1 || exit $?
done
