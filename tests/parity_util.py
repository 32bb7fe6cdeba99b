"""Parity bars grounded in the oracle's own reproducibility.

The fp32 gradients of this network at initialisation amplify rounding ~1000x through the
backward, so two CPU runs of the oracle that differ only in thread count (summation order) already
disagree: 1.1e-4 relative norm at B=16, measured 1.4e-3 at B=64 and 2.4e-3 at B=32 (BetaVAE-H).  A
fixed 1e-3 bar is therefore below the reference's own spread at the benchmarked shapes; the bar
per tensor is max(floor, 3 x that tensor's measured thread-count spread)."""
import torch

from oracle import vae_oracle as O


def oracle_with_spread(arch, sd, x, eps=None, threads=1, **kw):
    """(oracle at the default thread count, its per-gradient relative-norm spread vs `threads`)."""
    o = O.train_step(arch, sd, x, eps, do_adam=False, **kw)
    n0 = torch.get_num_threads()
    try:
        torch.set_num_threads(threads)
        o1 = O.train_step(arch, sd, x, eps, do_adam=False, **kw)
    finally:
        torch.set_num_threads(n0)
    spread = {k: float((o["grads"][k].double() - o1["grads"][k].double()).norm()
                       / o1["grads"][k].double().norm().clamp_min(1e-30)) for k in o["grads"]}
    return o, spread


def grad_bar(name, spread, floor_w=1e-3, floor_bn=3e-3):
    floor = floor_bn if name.endswith(".1.weight") or name.endswith(".1.bias") else floor_w
    return max(floor, 3.0 * spread.get(name, 0.0))
