# Per-block probe with and without the A-operand transform (diagnostic).  Usage: bash scripts/gpu_kp2.sh TAG
set -o pipefail
TAG=${1:-kp2}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
VAE_HIP_LIB=probe timeout -k 10 200 python3 -u tools/kprobe.py --out gpurun_out/${TAG}_xf.json > gpurun_out/${TAG}_xf.log 2>&1 || exit $?
VAE_PROBE_NOXF=1 VAE_HIP_LIB=probe timeout -k 10 200 python3 -u tools/kprobe.py --out gpurun_out/${TAG}_noxf.json > gpurun_out/${TAG}_noxf.log 2>&1
