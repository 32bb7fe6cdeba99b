# Launch-mode matrix of the VanillaVAE bench.  Usage: bash scripts/gpu_launch_matrix.sh TAG
set -o pipefail
TAG=${1:-lm}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline"
timeout -k 10 200 $B > gpurun_out/${TAG}_graph.log 2>&1 || exit $?
timeout -k 10 200 $B --no-graph > gpurun_out/${TAG}_eager.log 2>&1 || exit $?
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 $B > gpurun_out/${TAG}_graph_devka.log 2>&1 || exit $?
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 $B --no-graph > gpurun_out/${TAG}_eager_devka.log 2>&1 || exit $?
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 200 $B > gpurun_out/${TAG}_graph_pkt.log 2>&1 || exit $?
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 $B > gpurun_out/${TAG}_graph_nopkt.log 2>&1
