#!/usr/bin/env python3
"""Diagnostic: per-launch time of the step's GEMM calls with their operand transforms as
planned vs. forced to NONE (same shapes, same data; results are not checked) — how much of a
GEMM launch is the on-load BatchNorm/LeakyReLU (or BN-backward) transform."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pytorch-vae_amd")]
import torch  # noqa: E402


def main():
    from vae_amd import _lib as L
    from vae_amd.engine import FusedAdam, TrainStep
    from vae_amd.net import StepPlan, VAENet
    net = VAENet(latent_dim=128, dtype=torch.bfloat16, device="cuda", generator=torch.Generator().manual_seed(0))
    plan = StepPlan(net, 64)
    opt = FusedAdam(net, lr=0.005)
    plan.x.copy_(torch.rand(plan.x.shape, device="cuda"))
    plan.eps.copy_(torch.randn(plan.eps.shape, device="cuda"))
    step = TrainStep(net, plan, opt, graph=False)
    step()
    torch.cuda.synchronize()
    sp = L.stream_ptr()
    calls = plan.fwd_calls + plan.bwd_calls

    def t(fn, ref, n=50):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(5):
            L.call(fn, ref, sp)
        e0.record()
        for _ in range(n):
            L.call(fn, ref, sp)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n * 1e3

    for i, (fn, ref) in enumerate(calls):
        if ref is None or not isinstance(ref._obj, (L.ConvArgs, L.LinearArgs)):
            continue
        a = ref._obj
        base = t(fn, ref)
        saved = {}
        for f in ("x_xf", "dy_xf", "dx_epi"):
            if hasattr(a, f):
                x = getattr(a, f)
                saved[f] = (x.kind, x.aux)
                if x.kind != 0:
                    x.kind = 0
        none = t(fn, ref)
        for f, (k, aux) in saved.items():
            getattr(a, f).kind = k
        print(f"[{i:2d}] {fn:24s} as planned {base:7.2f} us   transforms off {none:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
