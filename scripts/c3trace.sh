set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
REPS=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3trace -o run -- python3 $GRAFT_REPO_ROOT/tools/c3bench.py > $O/c3trace.log 2>&1
