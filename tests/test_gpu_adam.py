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


def test_adam_ex_reduces_deferred_slabs_and_matches_torch_adam():
    """vae_adam_step_ex (the one-rank step's optimizer launch): each descriptor's gradient is the
    ascending-row sum of its partial rows — written into the gradient buffer — and then the same
    Adam update as torch.optim.Adam over five steps.  Descriptors like the step's: a tall slab of
    512 rows (the head's filter partials, ld 867, two descriptors sharing it: weight 864 columns,
    bias 3), one of 256 rows (the full-resolution ConvT's), short ones of 29 and 3 rows (grouped
    weight-gradient K slices); the rest of the buffer is a plain gradient.  Also the deferred loss:
    with has_elbo the launch writes vae_elbo_fwd's terms."""
    import ctypes
    from vae_amd import _lib as L
    from vae_amd.engine import FusedAdam
    n = 262_144
    gen = torch.Generator().manual_seed(11)
    p0 = torch.randn(n, generator=gen)
    net = types.SimpleNamespace(params=p0.cuda(), lowp=torch.zeros(n, dtype=torch.bfloat16, device="cuda"),
                                device=torch.device("cuda"))
    fa = FusedAdam(net, lr=5e-3)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=5e-3, betas=(0.9, 0.999), eps=1e-8)
    head = torch.zeros(512 * 867, device="cuda")
    hires = torch.zeros(256 * 9216, device="cuda")
    s29 = torch.zeros(29 * 18432, device="cuda")
    s3 = torch.zeros(3 * 73728, device="cuda")
    # (dst offset, count, slab tensor, column offset, rows, ld)
    spec = [(1024, 864, head, 0, 512, 867), (2048, 3, head, 864, 512, 867), (4096, 9216, hires, 0, 256, 9216),
            (16384, 18432, s29, 0, 29, 18432), (65536, 73728, s3, 0, 3, 73728)]
    gbuf = torch.zeros(n, device="cuda")
    st = L.stream_ptr()
    for k in range(5):
        scale = (1.0, 0.1, 3.0, 1e-3, 0.5)[k]
        gfull = torch.randn(n, generator=gen) * scale
        for t in (head, hires, s29, s3):
            t.copy_(torch.randn(t.numel(), generator=gen) * scale)
        slabs = []
        for off, count, t, c0, rows, ld in spec:
            rows_view = t.view(rows, ld)[:, c0:c0 + count].double().cpu()
            gfull[off:off + count] = rows_view.sum(0).float()
            slabs.append(L.GradSlab(dst=gbuf.data_ptr() + 4 * off, count=count, slab=t.data_ptr() + 4 * c0,
                                    rows=rows, ld=ld))
        gbuf.copy_(gfull.cuda())
        for off, count, *_ in spec:
            gbuf[off:off + count] = float("nan")          # must be overwritten by the reduction
        ref.grad = gfull.clone()
        opt.step()
        L.call("vae_step_begin", None, 0, fa.step.data_ptr(), st)
        fa.apply_deferred(gbuf, slabs, None, st)
        torch.cuda.synchronize()
        g_got = gbuf.cpu()
        assert torch.isfinite(g_got).all(), k
        err = (g_got - gfull).abs()
        if float(err.max()) > 1e-5 * float(gfull.abs().max()):
            bad = torch.nonzero(err > 1e-5 * float(gfull.abs().max())).flatten()
            raise AssertionError(f"step {k}: {bad.numel()} wrong gradient elements, first {bad[:16].tolist()}, "
                                 f"got {g_got[bad[:4]].tolist()} want {gfull[bad[:4]].tolist()}")
        got, want = net.params.cpu(), ref.detach()
        assert float((got - want).abs().max()) < 2e-6, k
        state = opt.state[ref]
        assert float((fa.m.cpu() - state["exp_avg"]).abs().max()) < 1e-5 * float(state["exp_avg"].abs().max()), k
        assert torch.equal(net.lowp.cpu(), got.to(torch.bfloat16)), k
    # the deferred loss: one extra workgroup of the same launch writes vae_elbo_fwd's terms
    B, D, E = 64, 128, 3 * 64 * 64
    mulv = (torch.randn(B, 2 * D, generator=gen) * 0.3).cuda()
    sse = (torch.rand(B, generator=gen) * 100).cuda()
    out = torch.zeros(4, device="cuda")
    per_img, hc, kc = (torch.zeros(B, device="cuda") for _ in range(3))
    e = L.ElboArgs(kind=L.LOSS_VANILLA, batch=B, samples=1, latent=D, img_elems=E, kld_weight=2.5e-4)
    e.mulv, e.sse, e.out, e.per_img, e.head_coef, e.kl_coef = (mulv.data_ptr(), sse.data_ptr(), out.data_ptr(),
                                                                per_img.data_ptr(), hc.data_ptr(), kc.data_ptr())
    L.call("vae_step_begin", None, 0, fa.step.data_ptr(), st)
    fa.apply_deferred(gbuf, [], e, st)
    out2 = torch.zeros(4, device="cuda")
    e.out = out2.data_ptr()
    L.call("vae_elbo_fwd", ctypes.byref(e), st)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), out2.cpu()), (out, out2)
