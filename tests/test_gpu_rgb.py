"""The VQ-VAE's RGB ends on their dedicated kernels (vae_rgb.hip; models/vq_vae.py:98-105,
:156-164, :203), each against PyTorch fp32 autograd on the same bf16-rounded operands:

  * vae_convT2d_fwd_recon: ConvTranspose2d(128 -> 3, k4 s2 p1) on LeakyReLU(x) + Tanh + the
    reconstruction, per-image SSE and the MSE backward seed (the 8-channel packed RGB side);
  * vae_convT2d_bwd of that layer: data gradient with the LeakyReLU backward, weight gradient
    written straight into the parameter's [128][4][4][3] (dw_inner = 3) and the bias gradient;
  * vae_conv2d_bwd_filter of the input Conv2d(3 -> 128, k4 s2 p1) from the 8-channel image.

Bars: fp32 outputs (reconstruction, SSE, weight / bias gradients) within 1e-4 relative of the
fp32 reference on the same bf16 operands (fp32 accumulation, only the summation order differs);
bf16 outputs (the seed dy, the data gradient) within bf16 rounding (1e-2 relative)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SLOPE = 0.01


def _bf(t):
    return t.to(torch.bfloat16).float()


def _ws(a, fn, op):
    from vae_amd import _lib as L
    import ctypes
    q, _ = L.WS_QUERY[fn]
    out = ctypes.c_size_t(0)
    L.call(q, ctypes.byref(a), op, ctypes.byref(out))
    ws = torch.empty(max(1, (out.value + 3) // 4), dtype=torch.float32, device="cuda")
    a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel() * 4
    return ws, out.value


@pytest.mark.parametrize("n", [2, 128])
def test_rgb_out_fwd_recon_matches_torch(n):
    import ctypes
    from vae_amd import _lib as L
    g = torch.Generator().manual_seed(5 + n)
    x = _bf(torch.randn(n, 128, 32, 32, generator=g))
    w = _bf(torch.randn(128, 3, 4, 4, generator=g) * 0.05)           # ConvTranspose2d [Ci][Co][R][S]
    b = torch.randn(3, generator=g) * 0.1
    tgt = torch.rand(n, 3, 64, 64, generator=g)
    # the kernel's MFMA operand is the activation rounded to bf16 (the reference contract of a bf16
    # operand); unrounded, the negative side's 0.01 x carries ~2e-5 of rounding into y
    y = F.conv_transpose2d(_bf(F.leaky_relu(x, SLOPE)), w, b, stride=2, padding=1)
    yr = y.clone().requires_grad_(True)
    r = torch.tanh(yr)
    F.mse_loss(r, tgt).backward()
    # device operands: x NHWC bf16, W native [Ci][R][S][Co] padded to 8, bias padded to 8
    xd = x.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)
    w8 = torch.zeros(128, 4, 4, 8)
    w8[..., :3] = w.permute(0, 2, 3, 1)
    w8 = w8.to("cuda", torch.bfloat16)
    b8 = torch.zeros(8, device="cuda")
    b8[:3] = b.cuda()
    tgt_d = tgt.cuda()
    recon = torch.empty(n, 3, 64, 64, device="cuda")
    sse = torch.zeros(n, device="cuda")
    dy = torch.full((n, 64, 64, 8), 5.0, dtype=torch.bfloat16, device="cuda")
    a = L.ConvArgs(dtype=L.BF16, n=n, h=32, w=32, c=128, k=8, p=64, q=64, r=4, stride=2, pad=1)
    a.x, a.wt, a.bias = xd.data_ptr(), w8.data_ptr(), b8.data_ptr()
    a.x_xf = L.Xform(kind=L.X_ACT, channels=128, slope=SLOPE)
    rc = L.ReconArgs(dtype=L.BF16, n=n, h=64, w=64, c=3, ld=8, grad_scale=1.0 / tgt.numel())
    rc.target, rc.recon, rc.sse, rc.dy = tgt_d.data_ptr(), recon.data_ptr(), sse.data_ptr(), dy.data_ptr()
    lib = L.load()
    lib.vae_launch_log(1)
    L.call("vae_convT2d_fwd_recon", ctypes.byref(a), ctypes.byref(rc), L.stream_ptr())
    lib.vae_launch_log(0)
    torch.cuda.synchronize()
    need = lib.vae_launch_log_names(None, 0)
    buf = ctypes.create_string_buffer(int(need))
    lib.vae_launch_log_names(buf, need)
    assert b"rgb_out_fwd_kernel" in buf.value, buf.value          # the dedicated kernel ran
    np.testing.assert_allclose(recon.cpu().numpy(), r.detach().numpy(), rtol=0, atol=2e-5)
    np.testing.assert_allclose(sse.cpu().numpy(), ((r.detach() - tgt) ** 2).sum(dim=(1, 2, 3)).numpy(), rtol=1e-4)
    want = yr.grad.permute(0, 2, 3, 1)
    got = dy.float().cpu()
    assert float(got[..., 3:].abs().max()) == 0.0
    np.testing.assert_allclose(got[..., :3].numpy(), want.numpy(), rtol=1e-2, atol=1e-2 * float(want.abs().max()))


@pytest.mark.parametrize("n", [4, 128])
def test_rgb_out_bwd_matches_torch(n):
    from vae_amd import _lib as L
    g = torch.Generator().manual_seed(17 + n)
    x_pre = _bf(torch.randn(n, 128, 32, 32, generator=g))
    w = _bf(torch.randn(128, 3, 4, 4, generator=g) * 0.05)
    dy = _bf(torch.randn(n, 3, 64, 64, generator=g))
    xa = _bf(F.leaky_relu(x_pre, SLOPE)).requires_grad_(True)      # (the bf16 operand the kernel reads)
    wr = w.clone().requires_grad_(True)
    br = torch.zeros(3, requires_grad=True)
    (F.conv_transpose2d(xa, wr, br, stride=2, padding=1) * dy).sum().backward()
    want_dx = xa.grad * torch.where(x_pre > 0, 1.0, SLOPE)
    xd = x_pre.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)
    dy8 = torch.zeros(n, 64, 64, 8)
    dy8[..., :3] = dy.permute(0, 2, 3, 1)
    dy8 = dy8.to("cuda", torch.bfloat16)
    w8 = torch.zeros(128, 4, 4, 8)
    w8[..., :3] = w.permute(0, 2, 3, 1)
    w8 = w8.to("cuda", torch.bfloat16)
    dx = torch.empty_like(xd)
    dw = torch.full((128, 4, 4, 3), 0.5, device="cuda")              # accumulated into
    db = torch.full((3,), 0.25, device="cuda")
    a = L.ConvArgs(dtype=L.BF16, n=n, h=32, w=32, c=128, k=8, p=64, q=64, r=4, stride=2, pad=1)
    a.x, a.x_xf = xd.data_ptr(), L.Xform(kind=L.X_ACT, channels=128, slope=SLOPE)
    a.dy, a.wt, a.dx = dy8.data_ptr(), w8.data_ptr(), dx.data_ptr()
    a.dx_epi = L.Xform(kind=L.X_ACT, channels=128, slope=SLOPE)
    a.dx_epi.aux = xd.data_ptr()
    a.dw, a.db, a.dw_inner = dw.data_ptr(), db.data_ptr(), 3
    ws, need = _ws(a, "vae_convT2d_bwd", L.OP_BWD)
    assert need > 0
    L.call("vae_convT2d_bwd", a, L.stream_ptr())
    torch.cuda.synchronize()
    got_dx = dx.float().permute(0, 3, 1, 2).cpu()
    err = float((got_dx - want_dx).abs().max() / want_dx.abs().max())
    assert err < 1e-2, err
    want_dw = wr.grad.permute(0, 2, 3, 1) + 0.5
    np.testing.assert_allclose(dw.cpu().numpy(), want_dw.numpy(), rtol=1e-4, atol=1e-4 * float(wr.grad.abs().max()))
    np.testing.assert_allclose(db.cpu().numpy(), (br.grad + 0.25).numpy(), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("n", [4, 128])
def test_rgb_in_wgrad_matches_torch(n):
    from vae_amd import _lib as L
    g = torch.Generator().manual_seed(29 + n)
    img = _bf(torch.rand(n, 3, 64, 64, generator=g))
    dy = _bf(torch.randn(n, 128, 32, 32, generator=g))
    wr = torch.zeros(128, 3, 4, 4, requires_grad=True)
    br = torch.zeros(128, requires_grad=True)
    (F.conv2d(img, wr, br, stride=2, padding=1) * dy).sum().backward()
    x8 = torch.zeros(n, 64, 64, 8)
    x8[..., :3] = img.permute(0, 2, 3, 1)
    x8 = x8.to("cuda", torch.bfloat16)
    dyd = dy.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)
    dw = torch.zeros(128, 4, 4, 3, device="cuda")
    db = torch.zeros(128, device="cuda")
    a = L.ConvArgs(dtype=L.BF16, n=n, h=64, w=64, c=8, k=128, p=32, q=32, r=4, stride=2, pad=1)
    a.x, a.dy, a.dw, a.db, a.dw_inner = x8.data_ptr(), dyd.data_ptr(), dw.data_ptr(), db.data_ptr(), 3
    ws, need = _ws(a, "vae_conv2d_bwd_filter", L.OP_BWD_FILTER)
    L.call("vae_conv2d_bwd_filter", a, L.stream_ptr())
    torch.cuda.synchronize()
    want = wr.grad.permute(0, 2, 3, 1)
    np.testing.assert_allclose(dw.cpu().numpy(), want.numpy(), rtol=1e-4, atol=1e-4 * float(want.abs().max()))
    np.testing.assert_allclose(db.cpu().numpy(), br.grad.numpy(), rtol=1e-4, atol=1e-4 * float(br.grad.abs().max()))
