"""The swapped-axes bf16 weight copies (vaehip.h wt_t: [b][r*s][a] of a native [a][r][s][b] weight)
that the bf16 convT forward and conv data-gradient GEMMs read.  A graphed TrainStep refreshes them in
its step-head launch (vae_step_begin_ex swap range) instead of a launch behind the optimizer, so
between steps they trail the parameters by one optimizer update: checked here against torch's own
permute of the fp32 parameters before the last step, and, after any other plan's launch list has
run (net.run_calls refreshes stale copies), against the current parameters."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _expected(net, params):
    out = {}
    for name in net.wt_t:
        spec = net.layout.by_name[name]
        a, r, r2, b = spec.native_shape
        w = params[spec.offset:spec.offset + spec.numel].view(a, r * r2, b)
        out[name] = w.permute(2, 1, 0).contiguous().to(torch.bfloat16).flatten()
    return out


def _actual(net):
    out = {}
    base = net.lowp_t.data_ptr()
    flat = net.lowp_t
    for name, ptr in net.wt_t.items():
        spec = net.layout.by_name[name]
        o = (ptr - base) // 2
        out[name] = flat[o:o + spec.numel]
    return out


def test_graphed_step_refreshes_swapped_copies_in_its_head():
    from vae_amd.engine import FusedAdam, TrainStep
    from vae_amd.net import StepPlan, VAENet
    net = VAENet(latent_dim=128, dtype=torch.bfloat16, device="cuda", generator=torch.Generator().manual_seed(3))
    plan = StepPlan(net, 16)
    g = torch.Generator(device="cuda").manual_seed(5)
    plan.x.copy_(torch.rand(plan.x.shape, generator=g, device="cuda"))
    step = TrainStep(net, plan, FusedAdam(net, lr=0.005), graph=True, device_eps=9)
    assert step._begin_swaps and len(net.wt_t) >= 8
    for _ in range(3):
        before = net.params.clone()
        step()
    torch.cuda.synchronize()
    assert net.swaps_stale
    exp, act = _expected(net, before), _actual(net)
    for name in exp:                     # refreshed by the last step's head, from its start weights
        assert torch.equal(act[name], exp[name]), name
    assert not torch.equal(net.params, before)
    # any other launch list on this net (here: an eval-mode plan's forward) refreshes them first
    ev = StepPlan(net, 16, training=False)
    ev.x.copy_(plan.x)
    ev.forward()
    torch.cuda.synchronize()
    assert not net.swaps_stale
    exp, act = _expected(net, net.params), _actual(net)
    for name in exp:
        assert torch.equal(act[name], exp[name]), name
