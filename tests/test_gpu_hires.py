"""The decoder's full-resolution last ConvTranspose2d (final_layer.0, models/vanilla_vae.py:64-70:
32 -> 32 channels, 32x32 -> 64x64, k3 s2 p1 op1) on its dedicated kernels (vae_hires.hip),
through the C ABI, against PyTorch fp32 on the CPU: the output, the next BatchNorm's producer
statistics (Σ(y - bias), Σ(y - bias)^2 over the replicas), the running-statistic update of the
input BatchNorm.  (The generic conv-GEMM path these shapes used to have a switch for is covered at
other shapes by test_gpu_cgemm.py.)  bf16 operands:
the tolerance is the bf16 one of the other op tests (2e-2 of the max) — the kernels accumulate in
fp32 and the statistics come from the fp32 accumulators."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from gpu_util import BNState, nhwc, rel, to_nchw

pytestmark = pytest.mark.gpu

N, C, H = 8, 32, 32
TOL = 2e-2


def _fwd_args(L, st, wd, wtd, bd, out, sums, reps):
    a = L.ConvArgs(dtype=L.BF16, n=N, h=H, w=H, c=C, k=C, p=2 * H, q=2 * H, r=3, stride=2, pad=1)
    a.x = st.y_dev.data_ptr()
    a.x_xf = st.xf()
    a.wt = wd.data_ptr()
    a.wt_t = wtd.data_ptr()
    a.bias = bd.data_ptr()
    a.y = out.data_ptr()
    a.y_sum, a.y_sumsq = sums[0].data_ptr(), sums[1].data_ptr()
    a.sum_reps, a.sum_rstride = reps, C
    return a


def _run_fwd():
    from vae_amd import _lib as L
    torch.manual_seed(4)
    y_prev = torch.randn(N, C, H, H) * 1.5 + 0.3
    st = BNState(y_prev, seed=1, dtype=torch.bfloat16)
    # the reference sees the bf16-rounded input the kernel reads
    st.y_nchw = to_nchw(st.y_dev)
    w = torch.randn(C, C, 3, 3) * 0.1                       # ConvTranspose2d [ci][co][r][s]
    b = torch.randn(C) * 0.1
    wd = w.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)        # native [ci][r][s][co]
    wtd = w.permute(1, 2, 3, 0).contiguous().to("cuda", torch.bfloat16)       # wt_t   [co][r][s][ci]
    bd = b.cuda()
    out = torch.empty(N, 2 * H, 2 * H, C, device="cuda", dtype=torch.bfloat16)
    reps = 8
    sums = torch.zeros(2, reps, C, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    a = _fwd_args(L, st, wd, wtd, bd, out, sums, reps)
    a.x_xf.running_mean, a.x_xf.running_var = rm.data_ptr(), rv.data_ptr()
    L.call("vae_convT2d_fwd", ctypes.byref(a), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    act = st.act_ref()
    wb = w.to(torch.bfloat16).float()
    ref = F.conv_transpose2d(act.to(torch.bfloat16).float(), wb, b, stride=2, padding=1, output_padding=1)
    return to_nchw(out), ref, sums.sum(1).cpu(), (ref - b.view(1, -1, 1, 1)), (rm.cpu(), rv.cpu()), st


def test_final_convT_fwd():
    out, ref, sums, pre, (rm, rv), st = _run_fwd()
    assert rel(out, ref) < TOL
    ps = pre.double()
    s1, s2 = ps.sum(dim=(0, 2, 3)), (ps * ps).sum(dim=(0, 2, 3))
    assert rel(sums[0], s1) < TOL and rel(sums[1], s2) < TOL
    # running statistics of the INPUT BatchNorm (momentum 0.1, unbiased variance) from the
    # producer statistics it was given, updated once
    cnt = st.count
    mean = st.sum.double() / cnt
    var = st.sumsq.double() / cnt - mean * mean
    torch.testing.assert_close(rm.double(), 0.1 * mean, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(rv.double(), 0.9 + 0.1 * var * cnt / (cnt - 1), rtol=1e-4, atol=1e-6)


def _bwd_case():
    """Both gradients of final_layer.0 through vae_convT2d_bwd against torch autograd on the CPU:
    act = lrelu(BN_x(x)), y = conv_transpose2d(act, W, b), z = BN_y(y); upstream g = dL/dz."""
    from vae_amd import _lib as L
    from gpu_util import give_workspace
    bf = lambda t: t.to(torch.bfloat16).float()
    torch.manual_seed(6)
    x = bf(torch.randn(N, C, H, H) * 1.3 + 0.2)
    sx = BNState(x, seed=2, dtype=torch.bfloat16)
    w = bf(torch.randn(C, C, 3, 3) * 0.1)
    b = torch.randn(C) * 0.1
    with torch.no_grad():
        y = bf(F.conv_transpose2d(bf(sx.act_ref()), w, b, stride=2, padding=1, output_padding=1))
    sy = BNState(y, shift=b, seed=3, dtype=torch.bfloat16)
    g = bf(torch.randn(N, C, 2 * H, 2 * H) * 0.05)
    # reference (fp32 autograd; act rounded to bf16 as the kernels stage it)
    xr = x.clone().requires_grad_(True)
    zx = F.batch_norm(xr, None, None, sx.gamma, sx.beta, True, 0.1, 1e-5)
    zx.retain_grad()
    act = F.leaky_relu(zx, 0.01)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = F.conv_transpose2d(act, wr, br, stride=2, padding=1, output_padding=1)
    yy = y.clone().requires_grad_(True)                    # BN_y on the stored (bf16) y
    gam = sy.gamma.clone().requires_grad_(True)
    bet = sy.beta.clone().requires_grad_(True)
    z = F.batch_norm(yy, None, None, gam, bet, True, 0.1, 1e-5)
    z.backward(g)
    dY = yy.grad                                           # dL/dy: what BN_DY computes on load
    yr.backward(dY)
    # device side
    xhat = (y - y.mean(dim=(0, 2, 3), keepdim=True)) / torch.sqrt(y.var(dim=(0, 2, 3), unbiased=False, keepdim=True) + 1e-5)
    dgam_in = (g * xhat).sum(dim=(0, 2, 3)).cuda()
    dbet_in = g.sum(dim=(0, 2, 3)).cuda()
    gd = nhwc(g, torch.bfloat16)
    wd = w.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)          # native [ci][r][s][co]
    dx = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
    dw = torch.zeros(C, 3, 3, C, device="cuda")
    db = torch.zeros(C, device="cuda")
    dgo, dbo = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    reps = 8
    esum = torch.zeros(2, reps, C, device="cuda")
    a = L.ConvArgs(dtype=L.BF16, n=N, h=H, w=H, c=C, k=C, p=2 * H, q=2 * H, r=3, stride=2, pad=1)
    a.x = sx.y_dev.data_ptr(); a.x_xf = sx.xf()
    a.dy = gd.data_ptr()
    a.dy_xf = sy.xf(L.X_BN_DY, aux=sy.y_dev, dgamma=dgam_in, dbeta=dbet_in)
    a.dy_xf.dgamma_out, a.dy_xf.dbeta_out = dgo.data_ptr(), dbo.data_ptr()
    a.wt = wd.data_ptr()
    a.dx = dx.data_ptr()
    a.dx_epi = sx.xf(aux=sx.y_dev)
    a.dx_dgamma, a.dx_dbeta = esum[0].data_ptr(), esum[1].data_ptr()
    a.sum_reps, a.sum_rstride = reps, C
    a.dw, a.db = dw.data_ptr(), db.data_ptr()
    ws = give_workspace(a, "vae_convT2d_bwd")
    L.call("vae_convT2d_bwd", ctypes.byref(a), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    del ws
    gx = zx.grad                                           # dL/dz_x: the data gradient's output
    xh_x = (x - x.mean(dim=(0, 2, 3), keepdim=True)) / torch.sqrt(x.var(dim=(0, 2, 3), unbiased=False, keepdim=True) + 1e-5)
    out = dict(dx=to_nchw(dx), dw=dw.cpu(), db=db.cpu(), dgo=dgo.cpu(), dbo=dbo.cpu(),
               es=esum.sum(1).cpu()[[1, 0]])                     # [Σg (dbeta), Σg·x̂ (dgamma)]
    ref = dict(dx=gx, dw=wr.grad.permute(0, 2, 3, 1).contiguous(), db=br.grad, dgo=gam.grad, dbo=bet.grad,
               es=torch.stack([gx.sum(dim=(0, 2, 3)), (gx * xh_x).sum(dim=(0, 2, 3))]))
    return out, ref


def test_final_convT_bwd_both_gradients():
    out, ref = _bwd_case()
    for k in ("dx", "dw", "es"):
        assert rel(out[k], ref[k]) < TOL, (k, rel(out[k], ref[k]))
    for k in ("dgo", "dbo"):                               # the BN affine gradients (fp32 sums)
        assert rel(out[k], ref[k]) < 1e-3, (k, rel(out[k], ref[k]))
    # the conv bias gradient under a train-mode BatchNorm is Σ dL/dy = 0 exactly (Σ x̂ = 0); the
    # closed form and autograd both return rounding noise around it
    torch.testing.assert_close(out["db"], ref["db"], rtol=0, atol=2e-4)
