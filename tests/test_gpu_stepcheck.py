"""Every kernel of the timed bf16 step, pinned at the benchmarked shapes: one step of
bench.py's exact path per BASELINE configuration of the VanillaVAE family, each op recomputed in fp64
from the GPU's own inputs (tests/stepcheck.py: teacher-forced, operand rounding mirrored), and every
kernel the step launched (vae_launch_log) mapped to at least one passing check of a call that
launches it.

  VanillaVAE B=64        configs[1] (the headline; models/vanilla_vae.py:25-146)
  BetaVAE-H B=32         configs[2] per GPU (global 256 over 8; beta_vae.py:129-152)
  IWAE K=5 B=64          configs[3] (decoder and head at B*S = 320; iwae.py:95-160)

The per-kernel map is written to gpurun_out/kernel_coverage_<arch>_<B>.json (tools/kernel_coverage.py
joins it with the profiles' kernel lists)."""
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [("vanilla", 64, 1, True), ("betaH", 32, 1, True), ("iwae", 64, 1, True),
         ("betaH", 32, 2, False), ("vanilla", 16, 1, True), ("vanilla", 16, 1, False)]


def _tag(a, b, s, d):
    return f"{a}_{b}" + (f"_seg{s}" if s > 1 else "") + ("" if d else "_nodefer")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("arch,batch,segments,defer", CASES, ids=[_tag(*c) for c in CASES])
def test_bench_step_every_op_teacher_forced(arch, batch, segments, defer):
    """(segments = 2, defer False: the weight gradients as two batches each reducing its own slices,
    as the N > 1 step's two gradient buckets run them at the per-GPU shape of configs[2]; B = 16:
    the shape of the one-rank RCCL tests, with and without the deferred reductions)"""
    from stepcheck import coverage, run_bench_step
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    checks, names_step, per_call = run_bench_step(arch, batch, segments=segments, defer=defer)
    for c in checks:
        print(("ok  " if c.ok else "BAD ") + f"{c.name} [{c.call[0]}#{c.call[1]}]: " +
              ", ".join(f"{k} {v:.3g}" if isinstance(v, float) else f"{k} {v}" for k, v in c.detail.items()))
    cov, step_kernels, missing = coverage(checks, names_step, per_call)
    out = os.path.join(REPO, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    tag = _tag(arch, batch, segments, defer)
    with open(os.path.join(out, f"kernel_coverage_{tag}.json"), "w") as f:
        json.dump({"arch": arch, "batch": batch, "test": f"tests/test_gpu_stepcheck.py::"
                   f"test_bench_step_every_op_teacher_forced[{tag}]",
                   "step_kernels": step_kernels, "coverage": cov,
                   "checks": [{"name": c.name, "call": list(c.call), "ok": c.ok, **c.detail} for c in checks]},
                  f, indent=1)
    bad = [c for c in checks if not c.ok]
    assert not bad, [(c.name, c.detail) for c in bad]
    assert len(step_kernels) >= 15, step_kernels
    assert not missing, f"kernels of the step no passing check covers: {missing}"
