# Round-2 measurements: bench lines for every 1-GPU config, kernel-trace stats and PMC passes.
# Usage: bash scripts/gpu_r2_measure.sh TAG
set -o pipefail
TAG=${1:-m}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py --steps 200 --warmup 20 --kernel-breakdown > $O/${TAG}_vanilla.log 2>&1 || exit $?
timeout -k 10 240 python3 -u bench.py --arch betaH --batch 32 --steps 200 --warmup 20 --no-cpu-baseline > $O/${TAG}_betaH.log 2>&1 || exit $?
timeout -k 10 240 python3 -u bench.py --arch iwae --batch 64 --steps 100 --warmup 10 --no-cpu-baseline > $O/${TAG}_iwae.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --arch vq --batch 128 --steps 50 --warmup 5 --no-cpu-baseline --kernel-breakdown > $O/${TAG}_vq.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_kt -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin > $O/${TAG}_kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_ktvq -o run -- python3 $R/bench.py --arch vq --batch 128 --steps 10 --warmup 3 --no-cpu-baseline --no-dropin > $O/${TAG}_ktvq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/${TAG}_pa -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-graph --no-dropin > $O/${TAG}_pa.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 FETCH_SIZE --output-format csv -d $O/${TAG}_pb -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-graph --no-dropin > $O/${TAG}_pb.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/${TAG}_pc -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-graph --no-dropin > $O/${TAG}_pc.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 FETCH_SIZE --output-format csv -d $O/${TAG}_pvq -o run -- python3 $R/bench.py --arch vq --batch 128 --steps 2 --warmup 1 --no-cpu-baseline --no-graph --no-dropin > $O/${TAG}_pvq.log 2>&1
