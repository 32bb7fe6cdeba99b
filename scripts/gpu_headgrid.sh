# Sweep the persistent grid of the head backward (VAE_HEAD_GRID) on the VanillaVAE B=64 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for g in 192 256 320 384 512; do
  VAE_HEAD_GRID=$g timeout -k 10 120 python -u bench.py --steps 100 --kernel-breakdown --no-cpu-baseline > gpurun_out/hg_$g.log 2>&1 || exit $?
done
