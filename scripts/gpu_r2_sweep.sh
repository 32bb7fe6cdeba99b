# Launch-shape sweep: bench step time + per-call breakdown under each tunable setting.
# Usage: bash scripts/gpu_r2_sweep.sh TAG
set -o pipefail
TAG=${1:-sw}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-dropin --kernel-breakdown \
    > gpurun_out/${TAG}_${name}.log 2>&1
}
run base && \
run minwg4 VAE_CG_MINWG=4 && \
run minwg8 VAE_CG_MINWG=8 && \
run split2 VAE_CG_SPLITWG=2 && \
run split4 VAE_CG_SPLITWG=4 && \
run wg4 VAE_WG_WGPERCU=4 && \
run wg1 VAE_WG_WGPERCU=1 && \
run conc VAE_CG_MINWG=2 && true
