# A/B bench variants.  Usage: bash scripts/gpu_cmp.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in "--serial" "" ; do
  timeout -k 10 120 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline $v > gpurun_out/${1}_$(echo x$v | tr -d ' -').log 2>&1 || exit $?
done
VAE_NO_CGEMM=1 timeout -k 10 120 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${1}_nocg.log 2>&1
