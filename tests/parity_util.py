"""Parity bars grounded in the oracle's own reproducibility.

The fp32 gradients of this network at initialisation amplify rounding ~1000x through the
backward, so two CPU runs of the oracle that differ only in thread count (summation order) already
disagree: 1.1e-4 relative norm at B=16, measured 1.4e-3 at B=64 and 2.4e-3 at B=32 (BetaVAE-H).
How large that spread comes out depends on the host's thread count (the GPU box runs 16 threads,
this container 8), so the spread per tensor is the larger of
  - the thread-count spread: the oracle at the default thread count vs on 1 thread, and
  - the fp32 rounding error of the oracle itself: the fp32 oracle vs the same oracle in fp64
    (the reference's own CPU path carries exactly that error),
and the bar per tensor is max(floor, 3 x that spread)."""
import torch

from oracle import vae_oracle as O


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def oracle_with_spread(arch, sd, x, eps=None, threads=1, **kw):
    """(oracle at the default thread count, its per-gradient relative-norm spread)."""
    o = O.train_step(arch, sd, x, eps, do_adam=False, **kw)
    n0 = torch.get_num_threads()
    try:
        torch.set_num_threads(threads)
        o1 = O.train_step(arch, sd, x, eps, do_adam=False, **kw)
    finally:
        torch.set_num_threads(n0)
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    o64 = O.train_step(arch, sd64, x.double(), None if eps is None else eps.double(), do_adam=False, **kw)
    spread = {k: max(_rel(o["grads"][k], o1["grads"][k]), _rel(o["grads"][k], o64["grads"][k]))
              for k in o["grads"]}
    return o, spread


def grad_bar(name, spread, floor_w=1e-3, floor_bn=3e-3):
    floor = floor_bn if name.endswith(".1.weight") or name.endswith(".1.bias") else floor_w
    return max(floor, 3.0 * spread.get(name, 0.0))
