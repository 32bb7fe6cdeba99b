# Per-block phase probe only.  Usage: bash scripts/gpu_kp.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
VAE_HIP_LIB=probe timeout -k 10 200 python3 -u tools/kprobe.py --out gpurun_out/${1:-kp}_kp.json > gpurun_out/${1:-kp}_kp.log 2>&1
