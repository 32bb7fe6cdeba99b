set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O; cd $GRAFT_REPO_ROOT
for bn in ${C3BN:-64 128}; do
  echo "bn=$bn" >> $O/c3dbg.log
  VAE_C3_BN=$bn timeout -k 10 100 python3 -u tools/c3bench.py 2>&1 | grep -v amdgpu >> $O/c3dbg.log || exit 1
done
