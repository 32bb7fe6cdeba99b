set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd $GRAFT_REPO_ROOT && timeout -k 10 120 python3 -u tools/c3bench.py > $O/c3b.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
REPS=5 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY --output-format csv -d $O/c3pmc_a -o run -- python3 $GRAFT_REPO_ROOT/tools/c3bench.py > $O/c3pmc_a.log 2>&1 || exit $?
REPS=5 timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 --output-format csv -d $O/c3pmc_b -o run -- python3 $GRAFT_REPO_ROOT/tools/c3bench.py > $O/c3pmc_b.log 2>&1 || exit $?
