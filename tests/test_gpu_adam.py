"""FusedAdam (vae_adam_step) against torch.optim.Adam over several steps (experiment.py:308-311).

At step 1 Adam's bias-corrected moments are m̂ = g and v̂ = g², so a single-step check cannot see
the β1/β2 recurrences or the bias corrections; here five steps run on fixed random gradients of
varying scale, with and without weight decay, and the parameters, both moment buffers and the
bf16 weight copy are compared after every step."""
import types

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wd", [0.0, 0.05])
@pytest.mark.parametrize("lr,betas", [(5e-3, (0.9, 0.999)), (7e-3, (0.8, 0.99))])
def test_fused_adam_matches_torch_adam(wd, lr, betas):
    from vae_amd import _lib as L
    from vae_amd.engine import FusedAdam
    n = 200_003
    g = torch.Generator().manual_seed(7)
    p0 = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g) * s for s in (1.0, 0.1, 3.0, 1e-3, 0.5)]
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=lr, betas=betas, eps=1e-8, weight_decay=wd)
    net = types.SimpleNamespace(params=p0.cuda(), lowp=torch.zeros(n, dtype=torch.bfloat16, device="cuda"),
                                device=torch.device("cuda"))
    fa = FusedAdam(net, lr=lr, betas=betas, eps=1e-8, weight_decay=wd)
    st = L.stream_ptr()
    for k, gk in enumerate(grads):
        ref.grad = gk.clone()
        opt.step()
        L.call("vae_step_begin", None, 0, fa.step.data_ptr(), st)      # ++step (as every training step)
        fa.apply(gk.cuda())
        torch.cuda.synchronize()
        state = opt.state[ref]
        got = net.params.cpu()
        want = ref.detach()
        assert int(fa.step.item()) == k + 1
        assert float((got - want).abs().max()) < 2e-6, k
        # moments: fp32 rounding (an fma vs mul+add) relative to the buffer's scale — elements
        # that cancel to ~0 have no meaningful relative error
        m_ref, v_ref = state["exp_avg"], state["exp_avg_sq"]
        assert float((fa.m.cpu() - m_ref).abs().max()) < 1e-6 * float(m_ref.abs().max()), k
        assert float((fa.v.cpu() - v_ref).abs().max()) < 1e-6 * float(v_ref.abs().max()), k
        assert torch.equal(net.lowp.cpu(), got.to(torch.bfloat16)), k
    # the trajectory moved well beyond rounding: a wrong recurrence would show here
    assert float((net.params.cpu() - p0).abs().max()) > 3 * lr          # (Adam moves <= ~lr per step)
