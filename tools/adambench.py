#!/usr/bin/env python3
"""Times vae_adam_step_ex on the VanillaVAE B=64 step's deferred reductions (diagnostic): all of
them, each class alone (head / full-resolution ConvT / grouped weight gradients), none (= the plain
optimizer over the same buffers), and vae_adam_step itself — HIP events around back-to-back
launches on one stream."""
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
    step = TrainStep(net, plan, opt, graph=True, device_eps=1265)
    step()
    torch.cuda.synchronize()
    slabs, elbo = step._slabs, step._elbo
    for s in slabs:
        print(f"slab: count {s.count} rows {s.rows} ld {s.ld}")
    st = torch.cuda.current_stream()
    sp = st.cuda_stream

    def timeit(fn, reps=50):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda._sleep(200000)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    cls = {"head": [s for s in slabs if s.rows == 512 or s.count == 3],
           "hires": [s for s in slabs if s.rows == 256],
           "wgrad": [s for s in slabs if s.rows < 64]}
    rows = [("vae_adam_step", timeit(lambda: opt.apply(plan.grads, sp, refresh_swaps=False))),
            ("ex none", timeit(lambda: opt.apply_deferred(plan.grads, [], None, sp))),
            ("ex all + loss", timeit(lambda: opt.apply_deferred(plan.grads, slabs, elbo, sp))),
            ("ex all", timeit(lambda: opt.apply_deferred(plan.grads, slabs, None, sp)))]
    for k, v in cls.items():
        rows.append((f"ex {k} only ({len(v)})", timeit(lambda v=v: opt.apply_deferred(plan.grads, v, None, sp))))
    for name, us in rows:
        print(f"{name:28s} {us:8.2f} us")


if __name__ == "__main__":
    main()
