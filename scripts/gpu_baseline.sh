set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g1_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/g1_tests.log
timeout -k 10 240 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --kernel-breakdown > gpurun_out/g1_bench.log 2>&1 && \
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/g1_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/g1_prof.log 2>&1
