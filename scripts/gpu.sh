# One parameterised driver for every GPU-box job of this repo (run through gpurun):
#
#   gpurun -- bash scripts/gpu.sh TAG STEP [STEP ...]
#
# Steps run in order, each under its own time limit; the first failing step ends the job (no
# GPU step runs after a fault, abort or timeout).  Output: gpurun_out/TAG_<step>.log (+ dirs).
#
#   tests            pytest -m gpu (all GPU tests)
#   tests:EXPR       pytest -m gpu -k EXPR
#   tenv:V=x,W=y:EXPR  pytest -m gpu -k EXPR with environment overrides
#   smoke            __graft_entry__.smoke()
#   bench            default bench line (driver's command: N=1, CPU baseline included)
#   quick            VanillaVAE bench, 200 steps, no CPU baseline, per-call breakdown
#   qenv:V=x,W=y     the quick bench with environment overrides (tunable sweeps)
#   aenv:V=x:A:B     the same as arch:A:B with environment overrides
#   arch:A:B         bench --arch A --batch B (betaH, iwae, vq, ae_big ...), no CPU baseline
#   archcpu:A:B      the same with the CPU baseline legs (the oracle on the host cores)
#   prof             rocprofv3 --kernel-trace --stats over a short VanillaVAE bench
#   prof:A:B         the same for --arch A --batch B
#   pmc              PMC passes (SQ / MFMA / FETCH / WRITE) of the graph-replayed VanillaVAE step, one
#                    run each; summary stamped with the build digest and GIT_HEAD (pass GIT_HEAD=...)
#   pmc:A:B          the same for --arch A --batch B
#   kprobe           per-block phase probe (needs `make probe`)
#   kbench[:ARGS]    per-launch microbench under a kernel trace (tools/kbench.py, ARGS comma-separated)
#   headbench        the decoder-head kernels back to back (tools/headbench.py): fwd, bwd, bwd halves
#   adambench        vae_adam_step_ex with each class of deferred reductions (tools/adambench.py)
#   c3bench[:ENV]    the VQ-VAE image-tile kernels back to back (tools/c3bench.py), ENV e.g.
#                    VAE_C3_DBG=5 (phase ablation: 1 no chunk loads, 2 no MFMAs, 4 no LDS stores)
#   c3trace          tools/c3bench.py under rocprofv3 --kernel-trace --stats
#   c3pmc            tools/c3bench.py under two PMC passes (MFMA busy, LDS bank conflicts, waits)
set -o pipefail
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
PT="python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"

run() {   # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name" >&2
  (cd $R && timeout -k 10 $secs "$@") > $O/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >&2
  return $rc
}

prof() {  # name bench-args...
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $O/${TAG}_${name} -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin "$@") \
     > $O/${TAG}_${name}.log 2>&1 || return $?
  cd $R && python3 tools/prof_summary.py --dir $O/${TAG}_${name} --out $O/${TAG}_${name}_kstats.json \
     --config "bench.py --steps 20 --warmup 5 $*" >> $O/${TAG}_${name}.log 2>&1
}

pmc() {   # name bench-args...   (one counter group per run: rocprofv3 does not split passes)
  # the graph-replayed step (the timed one); PMCNOGRAPH=1 profiles the eager launch sequence
  local name=$1; shift
  local B="python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-dropin ${PMCNOGRAPH:+--no-graph} $*"
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/${TAG}_${name}_pa -o run -- $B > $O/${TAG}_${name}_pa.log 2>&1 || return $?
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 FETCH_SIZE --output-format csv -d $O/${TAG}_${name}_pb -o run -- $B > $O/${TAG}_${name}_pb.log 2>&1 || return $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/${TAG}_${name}_pc -o run -- $B > $O/${TAG}_${name}_pc.log 2>&1 || return $?
  cd $R && python3 tools/pmc_summary.py --dirs $O/${TAG}_${name}_pa $O/${TAG}_${name}_pb $O/${TAG}_${name}_pc \
     --out $O/${TAG}_${name}_pmc.json --config "$*" > $O/${TAG}_${name}_pmcsum.log 2>&1
}

for step in "$@"; do
  IFS=: read -r kind a1 a2 a3 <<< "$step"
  case $kind in
    tests) if [ -n "$a1" ]; then run tests_${a1//[^A-Za-z0-9]/_} 900 $PT -k "$a1"; else run tests 900 $PT; fi ;;
    tenv) run tenv_${a1//[=,]/_} 900 env ${a1//,/ } $PT -k "$a2" ;;
    smoke) run smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python3 -u bench.py ;;
    quick) run quick 300 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --kernel-breakdown ;;
    qenv) run qenv_${a1//[=,]/_} 300 env ${a1//,/ } python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-dropin ;;
    aenv) run aenv_${a1//[=,]/_}_${a2}_${a3} 300 env ${a1//,/ } python3 -u bench.py --arch $a2 --batch $a3 --steps 100 --warmup 10 --no-cpu-baseline ;;
    arch) run arch_${a1}_${a2} 300 python3 -u bench.py --arch $a1 --batch $a2 --steps 100 --warmup 10 --no-cpu-baseline --kernel-breakdown ;;
    archcpu) run archcpu_${a1}_${a2} 400 python3 -u bench.py --arch $a1 --batch $a2 --steps 100 --warmup 10 --kernel-breakdown ;;
    prof) if [ -n "$a1" ]; then prof prof_$a1 --arch $a1 --batch $a2; else prof prof; fi ;;
    pmc) if [ -n "$a1" ]; then pmc pmc_$a1 --arch $a1 --batch $a2; else pmc pmc; fi ;;
    headbench) run headbench 200 python3 -u tools/headbench.py ;;
    adambench) run adambench 200 python3 -u tools/adambench.py ;;
    hbenv) run hbenv_${a1//[=,]/_} 200 env ${a1//,/ } python3 -u tools/headbench.py ;;
    kprobe) run kprobe 200 env VAE_HIP_LIB=probe python3 -u tools/kprobe.py --out $O/${TAG}_kp.json ;;
    kbench) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
               -d $O/${TAG}_kb -o kb -- python3 $R/tools/kbench.py --out $O/${TAG}_kb_groups.json ${a1//,/ }) \
               > $O/${TAG}_kbench.log 2>&1 ;;
    c3bench) run c3bench_${a1//[=,]/_} 200 env ${a1//,/ } python3 -u tools/c3bench.py ;;
    c3trace) (cd /tmp && export TMPDIR=/tmp && REPS=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
               -d $O/${TAG}_c3trace -o run -- python3 $R/tools/c3bench.py) > $O/${TAG}_c3trace.log 2>&1 ;;
    c3pmc) (cd /tmp && export TMPDIR=/tmp && \
            REPS=5 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY \
              --output-format csv -d $O/${TAG}_c3pmc_a -o run -- python3 $R/tools/c3bench.py > $O/${TAG}_c3pmc_a.log 2>&1 && \
            REPS=5 timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 \
              --output-format csv -d $O/${TAG}_c3pmc_b -o run -- python3 $R/tools/c3bench.py > $O/${TAG}_c3pmc_b.log 2>&1) ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
  rc=$?
  # a test step whose tests failed (pytest rc 1) ends nothing: the process exited normally; any
  # other failure (abort, fault, time limit) ends the job before the next GPU step
  if [ $rc -eq 1 ] && { [ "$kind" = tests ] || [ "$kind" = tenv ]; }; then echo "step $step: test failures (rc=1), continuing" >&2; FAILED=1; continue; fi
  [ $rc -eq 0 ] || { echo "step $step failed rc=$rc" >&2; exit $rc; }
done
exit ${FAILED:-0}
