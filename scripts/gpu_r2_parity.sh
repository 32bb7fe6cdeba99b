# Parity at bench shapes, DP vs oracle, bf16 vs autocast oracle.  Usage: bash scripts/gpu_r2_parity.sh TAG
set -o pipefail
TAG=${1:-par}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity_shapes.py tests/test_gpu_dp.py "tests/test_gpu_step.py::test_bf16_mode_tracks_bf16_autocast_oracle" -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_par.log 2>&1
