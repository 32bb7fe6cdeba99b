set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
VAE_HIP_LIB=probe timeout -k 10 200 python3 -u tools/kprobe.py --out gpurun_out/${1:-kp}.json > gpurun_out/${1:-kp}.log 2>&1
