"""Single C-ABI entry points vs PyTorch-CPU fp32 (the same ops the reference's nn.Modules
call: F.conv2d, F.conv_transpose2d, F.linear, batch_norm, leaky_relu, tanh, mse).

Tolerances: fp32 mode 2e-5 max-relative (exact-fp32 MFMA, different summation order);
bf16 mode 2e-2 (bf16 operands, fp32 accumulation)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from gpu_util import BNState, give_workspace, nhwc, rel, to_nchw, tol

pytestmark = pytest.mark.gpu

DTYPES = [torch.float32, torch.bfloat16]


def _L():
    from vae_amd import _lib as L
    return L


def _stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("split", [0, 3])
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("cin,cout,hw", [(32, 64, 16), (64, 32, 8), (16, 48, 12)])
def test_conv2d_fwd_bnact_and_stats(dtype, cin, cout, hw, split):
    L = _L()
    torch.manual_seed(0)
    N = 4
    y_prev = torch.randn(N, cin, hw, hw) * 1.5 + 0.3
    bn = BNState(y_prev, shift=torch.randn(cin) * 0.1, dtype=dtype)
    w = torch.randn(cout, cin, 3, 3) * 0.1
    b = torch.randn(cout) * 0.1
    ref = F.conv2d(bn.act_ref(), w, b, stride=2, padding=1)
    out = torch.empty(N, hw // 2, hw // 2, cout, device="cuda", dtype=dtype)
    s = torch.zeros(2 * cout, device="cuda")
    wd = w.permute(0, 2, 3, 1).contiguous().to("cuda", dtype)
    bd = b.cuda()
    a = L.ConvArgs(dtype=L.dtype_code(dtype), n=N, h=hw, w=hw, c=cin, k=cout, p=hw // 2, q=hw // 2, r=3, stride=2, pad=1)
    a.x = bn.y_dev.data_ptr(); a.x_xf = bn.xf(); a.wt = wd.data_ptr(); a.bias = bd.data_ptr(); a.y = out.data_ptr()
    a.y_sum = s.data_ptr(); a.y_sumsq = s.data_ptr() + 4 * cout
    a.split_k = split
    ws = give_workspace(a, "vae_conv2d_fwd")
    L.call("vae_conv2d_fwd", ctypes.byref(a), _stream())
    torch.cuda.synchronize()
    assert rel(to_nchw(out), ref) < tol(dtype)
    acc = ref - b.view(1, -1, 1, 1)
    assert rel(s[:cout].cpu(), acc.sum((0, 2, 3))) < 10 * tol(dtype)
    assert rel(s[cout:].cpu(), (acc * acc).sum((0, 2, 3))) < 10 * tol(dtype)


@pytest.mark.parametrize("dtype", DTYPES)
def test_conv2d_fwd_first_layer_nchw(dtype):
    L = _L()
    torch.manual_seed(1)
    N, H = 4, 16
    x = torch.rand(N, 3, H, H)
    w = torch.randn(32, 3, 3, 3) * 0.2
    b = torch.randn(32) * 0.1
    ref = F.conv2d(x, w, b, stride=2, padding=1)
    xd = x.cuda()
    out = torch.empty(N, H // 2, H // 2, 32, device="cuda", dtype=dtype)
    wd = w.permute(0, 2, 3, 1).contiguous().to("cuda", dtype)
    bd = b.cuda()
    a = L.ConvArgs(dtype=L.dtype_code(dtype), n=N, h=H, w=H, c=3, k=32, p=H // 2, q=H // 2, r=3, stride=2, pad=1, x_nchw_f32=1)
    a.x = xd.data_ptr(); a.wt = wd.data_ptr(); a.bias = bd.data_ptr(); a.y = out.data_ptr()
    L.call("vae_conv2d_fwd", ctypes.byref(a), _stream())
    torch.cuda.synchronize()
    assert rel(to_nchw(out), ref) < tol(dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("cin,cout,hw", [(64, 32, 4), (32, 32, 8), (128, 64, 2)])
def test_convT2d_fwd(dtype, cin, cout, hw):
    L = _L()
    torch.manual_seed(2)
    N = 4
    x = torch.randn(N, cin, hw, hw)
    w = torch.randn(cin, cout, 3, 3) * 0.1
    b = torch.randn(cout) * 0.1
    ref = F.conv_transpose2d(x, w, b, stride=2, padding=1, output_padding=1)
    xd = nhwc(x, dtype)
    out = torch.empty(N, 2 * hw, 2 * hw, cout, device="cuda", dtype=dtype)
    wd = w.permute(0, 2, 3, 1).contiguous().to("cuda", dtype)
    bd = b.cuda()
    a = L.ConvArgs(dtype=L.dtype_code(dtype), n=N, h=hw, w=hw, c=cin, k=cout, p=2 * hw, q=2 * hw, r=3, stride=2, pad=1)
    a.x = xd.data_ptr(); a.wt = wd.data_ptr(); a.bias = bd.data_ptr(); a.y = out.data_ptr()
    L.call("vae_convT2d_fwd", ctypes.byref(a), _stream())
    torch.cuda.synchronize()
    assert rel(to_nchw(out), ref) < tol(dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("transposed", [False, True])
def test_conv_backward_plain(dtype, transposed):
    """bwd_data and bwd_filter with plain dy (no transforms) vs autograd."""
    L = _L()
    torch.manual_seed(3)
    N, cin, cout, hw = 4, 32, 64, 8
    x = torch.randn(N, cin, hw, hw, requires_grad=True)
    if transposed:
        w = (torch.randn(cin, cout, 3, 3) * 0.1).requires_grad_()
        b = (torch.randn(cout) * 0.1).requires_grad_()
        y = F.conv_transpose2d(x, w, b, stride=2, padding=1, output_padding=1)
        P = 2 * hw
    else:
        w = (torch.randn(cout, cin, 3, 3) * 0.1).requires_grad_()
        b = (torch.randn(cout) * 0.1).requires_grad_()
        y = F.conv2d(x, w, b, stride=2, padding=1)
        P = hw // 2
    gy = torch.randn_like(y)
    y.backward(gy)
    xd = nhwc(x.detach(), dtype)
    gyd = nhwc(gy, dtype)
    wd = w.detach().permute(0, 2, 3, 1).contiguous().to("cuda", dtype)
    dx = torch.empty(N, hw, hw, cin, device="cuda", dtype=dtype)
    dw = torch.zeros(wd.shape, device="cuda")
    db = torch.zeros(cout, device="cuda")
    a = L.ConvArgs(dtype=L.dtype_code(dtype), n=N, h=hw, w=hw, c=cin, k=cout, p=P, q=P, r=3, stride=2, pad=1)
    a.x = xd.data_ptr(); a.wt = wd.data_ptr(); a.dy = gyd.data_ptr(); a.dx = dx.data_ptr()
    a.dw = dw.data_ptr(); a.db = db.data_ptr()
    pre = "vae_convT2d" if transposed else "vae_conv2d"
    L.call(pre + "_bwd_data", ctypes.byref(a), _stream())
    L.call(pre + "_bwd_filter", ctypes.byref(a), _stream())
    torch.cuda.synchronize()
    assert rel(to_nchw(dx), x.grad) < tol(dtype)
    assert rel(dw.permute(0, 3, 1, 2).cpu(), w.grad) < tol(dtype)
    assert rel(db.cpu(), b.grad) < tol(dtype)


@pytest.mark.parametrize("split", [0, 2])
@pytest.mark.parametrize("dtype", DTYPES)
def test_conv2d_backward_bn(dtype, split):
    """dy through BN_DY (BN-backward on load) and dx through the BN_ACT epilogue, vs autograd
    of conv(lrelu(bn(y_prev))) -> bn -> (upstream grad)."""
    L = _L()
    torch.manual_seed(4)
    N, cin, cout, hw = 4, 32, 64, 8
    y_prev = (torch.randn(N, cin, hw, hw) * 1.2 + 0.2).requires_grad_()
    g_prev = 0.8 + 0.4 * torch.rand(cin); b_prev = torch.rand(cin) * 0.2 - 0.1
    gp = g_prev.clone().requires_grad_(); bp = b_prev.clone().requires_grad_()
    a_prev = F.leaky_relu(F.batch_norm(y_prev, None, None, gp, bp, True, 0.1, 1e-5), 0.01)
    w = (torch.randn(cout, cin, 3, 3) * 0.1).requires_grad_()
    bias = (torch.randn(cout) * 0.1).requires_grad_()
    y = F.conv2d(a_prev, w, bias, stride=2, padding=1)
    g_cur = 0.8 + 0.4 * torch.rand(cout); b_cur = torch.rand(cout) * 0.2 - 0.1
    gc = g_cur.clone().requires_grad_(); bc = b_cur.clone().requires_grad_()
    z = F.batch_norm(y, None, None, gc, bc, True, 0.1, 1e-5)
    gz = torch.randn_like(z)
    z.backward(gz)
    # device state: previous BN, current BN, and the upstream g = dL/dz (what the next
    # layer's epilogue would have produced) with Σg, Σg·x̂ (== dβ, dγ of the current BN)
    bnp = BNState(y_prev.detach(), dtype=dtype); bnp.gamma, bnp.beta = g_prev, b_prev
    bnp.dev["gamma"], bnp.dev["beta"] = g_prev.cuda(), b_prev.cuda()
    yv = y.detach()
    bnc = BNState(yv, shift=bias.detach(), dtype=dtype); bnc.gamma, bnc.beta = g_cur, b_cur
    bnc.dev["gamma"], bnc.dev["beta"] = g_cur.cuda(), b_cur.cuda()
    mean = yv.mean((0, 2, 3), keepdim=True); var = yv.var((0, 2, 3), unbiased=False, keepdim=True)
    xh = (yv - mean) / torch.sqrt(var + 1e-5)
    dgam = (gz * xh).sum((0, 2, 3)).cuda(); dbet = gz.sum((0, 2, 3)).cuda()
    gzd = nhwc(gz, dtype)
    wd = w.detach().permute(0, 2, 3, 1).contiguous().to("cuda", dtype)
    dx = torch.empty(N, hw, hw, cin, device="cuda", dtype=dtype)
    dgp = torch.zeros(cin, device="cuda"); dbp = torch.zeros(cin, device="cuda")
    dw = torch.zeros(wd.shape, device="cuda"); db = torch.zeros(cout, device="cuda")
    a = L.ConvArgs(dtype=L.dtype_code(dtype), n=N, h=hw, w=hw, c=cin, k=cout, p=hw // 2, q=hw // 2, r=3, stride=2, pad=1)
    a.dy = gzd.data_ptr()
    a.dy_xf = bnc.xf(L.X_BN_DY, aux=bnc.y_dev, dgamma=dgam, dbeta=dbet)
    a.wt = wd.data_ptr()
    a.dx = dx.data_ptr()
    a.dx_epi = bnp.xf(L.X_BN_ACT, aux=bnp.y_dev)
    a.dx_dgamma = dgp.data_ptr(); a.dx_dbeta = dbp.data_ptr()
    a.x = bnp.y_dev.data_ptr(); a.x_xf = bnp.xf(L.X_BN_ACT)
    a.dw = dw.data_ptr(); a.db = db.data_ptr()
    a.split_k = split
    ws = give_workspace(a, "vae_conv2d_bwd_data", "vae_conv2d_bwd_filter")
    L.call("vae_conv2d_bwd_data", ctypes.byref(a), _stream())
    L.call("vae_conv2d_bwd_filter", ctypes.byref(a), _stream())
    torch.cuda.synchronize()
    t = tol(dtype)
    # dx here is g_prev = dL/d(BN_prev output pre-LReLU); compare the BN-param grads it feeds
    assert rel(dgp.cpu(), gp.grad) < 20 * t
    assert rel(dbp.cpu(), bp.grad) < 20 * t
    assert rel(dw.permute(0, 3, 1, 2).cpu(), w.grad) < 5 * t
    assert (db.cpu() - bias.grad).abs().max() < 1e-3 * w.grad.abs().max()


@pytest.mark.parametrize("dtype", DTYPES)
def test_linear_all(dtype):
    L = _L()
    torch.manual_seed(5)
    M, K, N = 16, 256, 96
    x = torch.randn(M, K, requires_grad=True)
    w = (torch.randn(N, K) * 0.05).requires_grad_()
    b = (torch.randn(N) * 0.1).requires_grad_()
    y = F.linear(x, w, b)
    gy = torch.randn_like(y)
    y.backward(gy)
    xd = x.detach().to("cuda", dtype); wd = w.detach().to("cuda", dtype); bd = b.detach().cuda()
    yd = torch.empty(M, N, device="cuda")
    gyd = gy.to("cuda", dtype)
    dx = torch.empty(M, K, device="cuda", dtype=dtype)
    dw = torch.zeros(N, K, device="cuda"); db = torch.zeros(N, device="cuda")
    a = L.LinearArgs(dtype=L.dtype_code(dtype), m=M, n=N, k=K)
    a.x = xd.data_ptr(); a.wt = wd.data_ptr(); a.bias = bd.data_ptr(); a.y = yd.data_ptr(); a.y_f32 = 1
    a.dy = gyd.data_ptr(); a.dx = dx.data_ptr(); a.dw = dw.data_ptr(); a.db = db.data_ptr()
    L.call("vae_linear_fwd", ctypes.byref(a), _stream())
    L.call("vae_linear_bwd_data", ctypes.byref(a), _stream())
    L.call("vae_linear_bwd_filter", ctypes.byref(a), _stream())
    torch.cuda.synchronize()
    t = tol(dtype)
    assert rel(yd.cpu(), y.detach()) < t
    assert rel(dx.float().cpu(), x.grad) < t
    assert rel(dw.cpu(), w.grad) < t
    assert rel(db.cpu(), b.grad) < t


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("C,N", [(32, 2), (64, 2), (128, 2), (128, 9)])
def test_head_fwd_bwd(dtype, fused, C, N):
    """final Conv2d(C->3,k3,s1,p1)+Tanh and MSE vs autograd (vanilla_vae.py:73-75, :140;
    autoencoder.py:84-86 with C = 128, configs/big_ae.yaml); fused: vae_head_bwd (data + filter in
    one pass, per-block partials summed from a workspace).  C = 64 / 128 run the MFMA head kernels
    in bf16 only (N = 9 at C = 128: 288 tiles, more than the persistent backward's 256 workgroups)."""
    if C != 32 and dtype != torch.bfloat16:
        pytest.skip("64/128-channel heads: bf16 MFMA kernels (fp32 plans take the conv-GEMM route)")
    L = _L()
    torch.manual_seed(6)
    H = 64
    y_prev = torch.randn(N, C, H, H).requires_grad_()
    gam = 0.8 + 0.4 * torch.rand(C); bet = torch.rand(C) * 0.2 - 0.1
    gp = gam.clone().requires_grad_(); bp = bet.clone().requires_grad_()
    act = F.leaky_relu(F.batch_norm(y_prev, None, None, gp, bp, True, 0.1, 1e-5), 0.01)
    w = (torch.randn(3, C, 3, 3) * 0.1).requires_grad_()
    b = (torch.randn(3) * 0.1).requires_grad_()
    rec = torch.tanh(F.conv2d(act, w, b, padding=1))
    tgt = torch.rand(N, 3, H, H)
    loss = F.mse_loss(rec, tgt)
    loss.backward()
    bn = BNState(y_prev.detach(), dtype=dtype); bn.gamma, bn.beta = gam, bet
    bn.dev["gamma"], bn.dev["beta"] = gam.cuda(), bet.cuda()
    wd = w.detach().permute(0, 2, 3, 1).contiguous().cuda(); bd = b.detach().cuda()
    tg = tgt.cuda()
    recon = torch.empty(N, 3, H, H, device="cuda"); sse = torch.zeros(N, device="cuda")
    coef = torch.full((N,), 2.0 / rec.numel(), device="cuda")
    dx = torch.empty(N, H, H, C, device="cuda", dtype=dtype)
    dgp = torch.zeros(C, device="cuda"); dbp = torch.zeros(C, device="cuda")
    dw = torch.zeros(wd.shape, device="cuda"); db = torch.zeros(3, device="cuda")
    a = L.HeadArgs(dtype=L.dtype_code(dtype), n=N, h=H, w=H, c=C, samples=1)
    a.x = bn.y_dev.data_ptr(); a.x_xf = bn.xf(); a.wt = wd.data_ptr(); a.bias = bd.data_ptr(); a.target = tg.data_ptr()
    a.recon = recon.data_ptr(); a.sse = sse.data_ptr(); a.coef = coef.data_ptr()
    a.dx = dx.data_ptr(); a.dx_epi = bn.xf(aux=bn.y_dev); a.dx_dgamma = dgp.data_ptr(); a.dx_dbeta = dbp.data_ptr()
    a.dw = dw.data_ptr(); a.db = db.data_ptr()
    if fused:
        ws = give_workspace(a, "vae_head_bwd")
    lib = L.load()
    lib.vae_launch_log(1)
    L.call("vae_head_fwd", ctypes.byref(a), _stream())
    if fused:
        L.call("vae_head_bwd", ctypes.byref(a), _stream())
    else:
        L.call("vae_head_bwd_data", ctypes.byref(a), _stream())
        L.call("vae_head_bwd_filter", ctypes.byref(a), _stream())
    lib.vae_launch_log(0)
    torch.cuda.synchronize()
    if dtype == torch.bfloat16:
        need = lib.vae_launch_log_names(None, 0)
        buf = ctypes.create_string_buffer(int(need))
        lib.vae_launch_log_names(buf, need)
        fwd = f"head_fwd_stream<{C}," if C == 128 else f"head_fwd_mfma<{C},"
        bwd = "head_bwd_mfma<64, 2, 128>" if C == 128 else f"head_bwd_mfma<{C},"
        assert fwd.encode() in buf.value, buf.value
        assert bwd.encode() in buf.value, buf.value
    t = tol(dtype)
    if dtype == torch.bfloat16:
        # the kernel's operands are bf16 (stored y, the activation it stages, the weights), so its
        # pre-tanh error grows as sqrt(9 C) of bf16 rounding (C = 128: up to 0.03 of max); against
        # the same rounding emulated only the fp32 summation order differs
        mean = y_prev.detach().mean((0, 2, 3)); var = y_prev.detach().var((0, 2, 3), unbiased=False)
        ta = gam / torch.sqrt(var + 1e-5); tb = bet - mean * ta
        z_b = y_prev.detach().to(torch.bfloat16).float() * ta.view(1, -1, 1, 1) + tb.view(1, -1, 1, 1)
        act_b = F.leaky_relu(z_b, 0.01).to(torch.bfloat16).double()
        w_b = w.detach().to(torch.bfloat16).double()
        rec_b = torch.tanh(F.conv2d(act_b, w_b, b.detach().double(), padding=1)).float()
        assert rel(recon.cpu(), rec_b) < 1e-3
        assert abs(sse.sum().item() - ((rec_b - tgt) ** 2).sum().item()) < 1e-3 * ((rec_b - tgt) ** 2).sum().item()
    assert rel(recon.cpu(), rec.detach()) < t * (C / 32) ** 0.5
    assert abs(sse.sum().item() / rec.numel() - loss.item()) < t * loss.item()
    assert rel(dw.permute(0, 3, 1, 2).cpu(), w.grad) < 5 * t
    assert rel(db.cpu(), b.grad) < 5 * t
    assert rel(dgp.cpu(), gp.grad) < 20 * t
    assert rel(dbp.cpu(), bp.grad) < 20 * t
    # dx = dL/dz of the BatchNorm output z feeding the head (LeakyReLU backward applied)
    z = F.batch_norm(y_prev.detach(), None, None, gam, bet, True, 0.1, 1e-5).requires_grad_()
    rec2 = torch.tanh(F.conv2d(F.leaky_relu(z, 0.01), w.detach(), b.detach(), padding=1))
    F.mse_loss(rec2, tgt).backward()
    # norm-relative: with y stored in bf16 a handful of pixels with z = BN(y) ~ 0 take the other
    # LeakyReLU branch (a factor 1/slope on an element that is ~0 anyway)
    d = dx.float().permute(0, 3, 1, 2).cpu()
    assert float((d - z.grad).norm() / z.grad.norm()) < t


def test_step_record_tracks_terms_per_image_and_extremes():
    """vae_step_record (the device bookkeeping of experiment.py:45-86 training_step) against the
    reference's loop: per-image mean over samples, strict '>' / '<' running extremes with the
    first index winning ties, the image and the first sample's reconstruction copied."""
    L = _L()
    dev = "cuda"
    B, S, ie = 6, 2, 3 * 4 * 4
    best = torch.tensor([float("-inf"), float("inf")], device=dev)
    at = torch.full((4,), -1, dtype=torch.int32, device=dev)
    hi_img, lo_img = torch.zeros(ie, device=dev), torch.zeros(ie, device=dev)
    hi_rec, lo_rec = torch.zeros(ie, device=dev), torch.zeros(ie, device=dev)
    ref_best, ref_at = [float("-inf"), float("inf")], [(-1, -1), (-1, -1)]
    g = torch.Generator().manual_seed(3)
    for step in range(3):
        src = torch.randn(3, generator=g).to(dev)
        per_img = torch.rand(B * S, generator=g)
        if step == 1:
            per_img[2 * S:3 * S] = per_img.view(B, S).mean(1).max() + 1.0   # a tie for the max:
            per_img[4 * S:5 * S] = per_img[2 * S:3 * S]                       # index 2 must win
        img = torch.randn(B, ie, generator=g)
        rec = torch.randn(B * S, ie, generator=g)
        terms, per = torch.zeros(3, device=dev), torch.zeros(B, device=dev)
        a = L.RecordArgs(batch=B, samples=S, img_elems=ie, nterms=3, step=step)
        keep = [src, per_img.to(dev), img.to(dev), rec.to(dev)]
        a.src_terms, a.terms = keep[0].data_ptr(), terms.data_ptr()
        a.per_img, a.per = keep[1].data_ptr(), per.data_ptr()
        a.img, a.recon = keep[2].data_ptr(), keep[3].data_ptr()
        a.best, a.at = best.data_ptr(), at.data_ptr()
        a.hi_img, a.hi_recon, a.lo_img, a.lo_recon = hi_img.data_ptr(), hi_rec.data_ptr(), lo_img.data_ptr(), lo_rec.data_ptr()
        L.call("vae_step_record", ctypes.byref(a), _stream())
        torch.cuda.synchronize()
        pm = per_img.view(B, S).mean(1)
        torch.testing.assert_close(terms.cpu(), src.cpu())
        torch.testing.assert_close(per.cpu(), pm)
        for k, better in ((0, lambda v, b: v > b), (1, lambda v, b: v < b)):
            for i in range(B):                          # experiment.py:65-84, in order
                if better(float(pm[i]), ref_best[k]):
                    ref_best[k], ref_at[k] = float(pm[i]), (step, i)
                    want_img, want_rec = img[i], rec[i * S]
                    if k == 0:
                        hi_want = (want_img, want_rec)
                    else:
                        lo_want = (want_img, want_rec)
        assert abs(float(best[0]) - ref_best[0]) < 1e-6 and abs(float(best[1]) - ref_best[1]) < 1e-6
        assert tuple(at.tolist()) == (*ref_at[0], *ref_at[1])
        torch.testing.assert_close(hi_img.cpu(), hi_want[0]); torch.testing.assert_close(hi_rec.cpu(), hi_want[1])
        torch.testing.assert_close(lo_img.cpu(), lo_want[0]); torch.testing.assert_close(lo_rec.cpu(), lo_want[1])
