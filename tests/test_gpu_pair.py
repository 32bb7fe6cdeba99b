"""vae_conv_bwd_pair: a BatchNorm'd block's data and weight gradients as one grid (vaehip.h).

The pair call must give the results of the two calls made one after the other.  At step level:
the VanillaVAE-family bf16 step at the benchmarked shapes with the pairs (the default) against
the same step with VAE_PAIR=0 (the layers' weight gradients in the segment's grouped batch):
identical data-gradient chains (the same tile body, bit for bit: every dx, the loss terms) and
weight gradients equal up to fp32 accumulation order (K slices added by atomics).  The pair grids
must actually have run (launch log), so a silent fallback to two launches fails the test."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _names(lib):
    import ctypes
    need = lib.vae_launch_log_names(None, 0)
    buf = ctypes.create_string_buffer(int(need))
    lib.vae_launch_log_names(buf, need)
    return buf.value.decode(errors="replace")


def _backward(plan, calls, lib, st):
    from vae_amd.net import run_calls
    plan.reset_backward()
    lib.vae_launch_log(1)
    try:
        run_calls(plan, calls, st)
    finally:
        lib.vae_launch_log(0)
    torch.cuda.synchronize()
    grads = {k: v.cpu() for k, v in plan.net.layout.export_reference(plan.grads).items()}
    dx = [t.float().cpu() for t in plan.g_enc[:-1] + plan.g_dec]
    return grads, dx, _names(lib)


def _rel(a, b):
    d = b.double()
    n = float(d.norm())
    return float((a.double() - d).norm()) / n if n > 0 else float(a.double().norm())


@pytest.mark.parametrize("loss,batch,samples", [("vanilla", 64, 1), ("betaH", 32, 1), ("iwae", 64, 5)])
def test_pair_backward_equals_unpaired_backward(loss, batch, samples):
    """One forward, then the backward twice from it: with the pair calls (VAE_PAIR=1's list)
    and with VAE_PAIR=0's list (every weight gradient in the grouped batch).  Both differ only in
    fp32 accumulation order (atomics): each tensor must agree with the unpaired result as closely
    as the unpaired backward run twice agrees with itself (3x that noise floor + 1e-3)."""
    from oracle import vae_oracle as O
    from vae_amd import _lib as L
    from vae_amd.engine import FusedAdam
    from vae_amd.net import PAIR_FN, StepPlan, VAENet, batch_filter_calls, size_workspaces
    sd = O.make_params(O.vanilla_param_spec(), 1265)
    x, eps = O.make_inputs(batch, 128, 17, samples=samples if samples > 1 else None)
    net = VAENet(latent_dim=128, dtype=torch.bfloat16, device="cuda")
    net.load_reference_state_dict(sd)
    old = os.environ.get("VAE_PAIR")
    os.environ["VAE_PAIR"] = "1"
    try:
        plan = StepPlan(net, batch, loss=loss, kld_weight=2.5e-4, samples=samples)
    finally:
        if old is None:
            del os.environ["VAE_PAIR"]
        else:
            os.environ["VAE_PAIR"] = old
    paired = list(plan.bwd_calls)
    keep = (plan.workspace, plan.workspace_side)            # the paired calls' workspaces
    old = os.environ.get("VAE_PAIR")
    os.environ["VAE_PAIR"] = "0"
    try:
        unpaired, _ = batch_filter_calls(plan.bwd_calls_raw, [len(plan.bwd_calls_raw)])
    finally:
        if old is None:
            del os.environ["VAE_PAIR"]
        else:
            os.environ["VAE_PAIR"] = old
    size_workspaces(plan, [plan.fwd_calls, unpaired])
    assert sum(1 for fn, _ in paired if fn == PAIR_FN) >= 6
    assert not any(fn == PAIR_FN for fn, _ in unpaired)
    opt = FusedAdam(net, lr=0.005)
    plan.x.copy_(x)
    plan.eps.copy_(eps.reshape(plan.eps.shape))
    st = L.stream_ptr()
    L.call("vae_step_begin", plan.zero.data_ptr(), plan.zero.numel() * 4, opt.step.data_ptr(), st)
    plan.forward(st)
    lib = L.load()
    g1, dx1, names1 = _backward(plan, paired, lib, st)
    g0, dx0, names0 = _backward(plan, unpaired, lib, st)
    g2, dx2, _ = _backward(plan, unpaired, lib, st)           # the same list again: the noise floor
    del keep
    assert "pair_kernel" in names1 and "pair_kernel" not in names0

    def bar(floor):
        return 3 * floor + 1e-3
    # every dx of the data-gradient chain; the BatchNorm-backward sums (fp32 atomics) differ in
    # order from run to run and the chain amplifies that through nine BatchNorms — the unpaired
    # list run twice measures it
    for i, (a, b, c) in enumerate(zip(dx1, dx0, dx2)):
        assert _rel(a, b) <= bar(_rel(c, b)), (i, _rel(a, b), _rel(c, b))
    bad = []
    for k, ref in g0.items():
        if k.endswith(".0.bias") and float(ref.abs().max()) < 1e-5:
            continue                      # pre-BatchNorm conv biases: analytically zero (noise)
        e, f = _rel(g1[k], ref), _rel(g2[k], ref)
        if not e <= bar(f):
            bad.append((k, e, f))
    assert not bad, bad
