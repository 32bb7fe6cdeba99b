#!/usr/bin/env python3
"""Times vae_step_begin_ex of the VanillaVAE B=64 step (diagnostic) with each of its block ranges
alone: zeroing (the region minus the kept gradients), the padded image, the swapped weight copies."""
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
    step = TrainStep(net, plan, opt, graph=True, device_eps=1265)
    step()
    torch.cuda.synchronize()
    full = step._begin[0]
    st = torch.cuda.current_stream()

    def timeit(a, reps=50):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        L.call("vae_step_begin_ex", ctypes.byref(a), st.cuda_stream)
        torch.cuda._sleep(200000)
        e0.record(st)
        for _ in range(reps):
            L.call("vae_step_begin_ex", ctypes.byref(a), st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    def variant(**kw):
        a = L.StepBeginArgs.from_buffer_copy(full)
        for k, v in kw.items():
            setattr(a, k, v)
        return a
    rows = [("full", variant()), ("no keep (zero all)", variant(nkeep=0)), ("zero only", variant(x=None, npad=0, nswap=0)),
            ("image only", variant(bytes=0, npad=0, nswap=0)), ("swaps only", variant(bytes=0, x=None, npad=0)),
            ("no swaps", variant(nswap=0))]
    for name, a in rows:
        print(f"{name:22s} {timeit(a):8.2f} us")


if __name__ == "__main__":
    main()
