# Full measurement pass: parity tests, bench (+cpu baseline), kernel-trace profiles of the
# VanillaVAE and VQ-VAE benches, PMC HBM traffic passes.  Usage: bash scripts/gpu_round.sh TAG
set -o pipefail
TAG=${1:-rd}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 240 python -u bench.py --kernel-breakdown > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_vqprof -o run -- python3 $R/bench.py --arch vq --batch 128 --steps 20 --warmup 3 --cpu-seconds 10 > $R/gpurun_out/${TAG}_vqprof.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_pmcf -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-graph > $R/gpurun_out/${TAG}_pmcf.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${TAG}_pmcw -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-graph > $R/gpurun_out/${TAG}_pmcw.log 2>&1
