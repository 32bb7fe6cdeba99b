"""The image-tile 3x3 convolution (csrc/vae_c3.hip: stride 1, pad 1, 16 x 16 grid — the VQ-VAE's
residual stacks, vq_vae.py:57-70 and the Conv3x3 layers at :94-166) through the C ABI
(vae_conv2d_fwd / vae_conv2d_bwd_data pick it for these shapes in bf16) vs PyTorch-CPU fp32 on the
same bf16-rounded operands.  Tolerance 1e-2 max-relative: fp32 accumulation, bf16 output."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from gpu_util import give_workspace, nhwc, rel, to_nchw

pytestmark = pytest.mark.gpu
TOL = 1e-2


def _bf(t):
    return t.bfloat16().float()


@pytest.mark.parametrize("n,cin,cout,act,bias", [(4, 256, 256, True, False), (3, 64, 256, False, True),
                                                 (9, 32, 128, True, True), (2, 128, 384, False, False)])
def test_c3_forward(n, cin, cout, act, bias):
    from vae_amd import _lib as L
    torch.manual_seed(11)
    x = _bf(torch.randn(n, cin, 16, 16))
    w = _bf(torch.randn(cout, cin, 3, 3) * (1.0 / (3 * cin ** 0.5)))
    b = torch.randn(cout) * 0.1 if bias else None
    ref = F.conv2d(F.leaky_relu(x, 0.01) if act else x, w, b, padding=1)
    xd = nhwc(x, torch.bfloat16)
    wd = w.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)
    bd = b.cuda() if bias else None
    out = torch.empty(n, 16, 16, cout, device="cuda", dtype=torch.bfloat16)
    a = L.ConvArgs(dtype=L.BF16, n=n, h=16, w=16, c=cin, k=cout, p=16, q=16, r=3, stride=1, pad=1)
    a.x, a.wt, a.y = xd.data_ptr(), wd.data_ptr(), out.data_ptr()
    if act:
        a.x_xf = L.Xform(kind=L.X_ACT, channels=cin, slope=0.01)
    if bias:
        a.bias = bd.data_ptr()
    lib = L.load()
    lib.vae_launch_log(1)
    try:
        L.call("vae_conv2d_fwd", ctypes.byref(a), torch.cuda.current_stream().cuda_stream)
    finally:
        lib.vae_launch_log(0)
    torch.cuda.synchronize()
    need = lib.vae_launch_log_names(None, 0)
    buf = ctypes.create_string_buffer(int(need))
    lib.vae_launch_log_names(buf, need)
    # the LDS-DMA image-tile kernel for an untransformed input; an activated input stays on the
    # register-staged kernel, which applies the LeakyReLU once per element (vae_c3.hip c3_launch)
    want = b"c3_kernel<128>" if act else b"c3d_kernel"
    assert want in buf.value, buf.value
    assert rel(to_nchw(out), ref) < TOL


@pytest.mark.parametrize("n,cin,cout,res,act", [(4, 256, 256, True, True), (3, 256, 64, True, False),
                                                (5, 128, 128, False, True)])
def test_c3_backward_data(n, cin, cout, res, act):
    """dx = conv2d's input gradient (+ skip gradient) * lrelu'(x0) — the ResidualLayer backward."""
    from vae_amd import _lib as L
    torch.manual_seed(12)
    x = torch.randn(n, cin, 16, 16, requires_grad=True)
    w = _bf(torch.randn(cout, cin, 3, 3) * (1.0 / (3 * cin ** 0.5)))
    y = F.conv2d(x, w, padding=1)
    gy = _bf(torch.randn_like(y))
    y.backward(gy)
    ref = x.grad.clone()
    r = _bf(torch.randn(n, cin, 16, 16)) if res else None
    aux = _bf(torch.randn(n, cin, 16, 16)) if act else None
    if res:
        ref = ref + r
    if act:
        ref = torch.where(aux > 0, ref, ref * 0.01)
    gyd = nhwc(gy, torch.bfloat16)
    wt = w.permute(1, 2, 3, 0).contiguous().to("cuda", torch.bfloat16)          # WT[c][r][s][k]
    wd = w.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)
    dx = torch.empty(n, 16, 16, cin, device="cuda", dtype=torch.bfloat16)
    a = L.ConvArgs(dtype=L.BF16, n=n, h=16, w=16, c=cin, k=cout, p=16, q=16, r=3, stride=1, pad=1)
    a.dy, a.wt, a.wt_t, a.dx = gyd.data_ptr(), wd.data_ptr(), wt.data_ptr(), dx.data_ptr()
    keep = []
    if res:
        rd = nhwc(r, torch.bfloat16)
        keep.append(rd)
        a.residual = rd.data_ptr()
    if act:
        ad = nhwc(aux, torch.bfloat16)
        keep.append(ad)
        a.dx_epi = L.Xform(kind=L.X_ACT, channels=cin, slope=0.01, aux=ad.data_ptr())
    L.call("vae_conv2d_bwd_data", ctypes.byref(a), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert rel(to_nchw(dx), ref) < TOL


@pytest.mark.parametrize("n,cin,cout,act,bias", [(8, 256, 256, True, False), (5, 64, 256, False, True),
                                                 (3, 32, 128, True, True)])
def test_c3_backward_filter(n, cin, cout, act, bias):
    """dW (accumulated onto a nonzero start) and db of a 3x3 stride-1 conv on a 16 x 16 grid."""
    from vae_amd import _lib as L
    torch.manual_seed(13)
    x = _bf(torch.randn(n, cin, 16, 16))
    w = torch.zeros(cout, cin, 3, 3, requires_grad=True)
    b = torch.zeros(cout, requires_grad=True)
    y = F.conv2d(F.leaky_relu(x, 0.01) if act else x, w, b, padding=1)
    gy = _bf(torch.randn_like(y))
    y.backward(gy)
    dw0 = torch.randn(cout, 3, 3, cin) * 0.1
    xd = nhwc(x, torch.bfloat16)
    gyd = nhwc(gy, torch.bfloat16)
    dw = dw0.clone().cuda()
    db = torch.zeros(cout, device="cuda")
    a = L.ConvArgs(dtype=L.BF16, n=n, h=16, w=16, c=cin, k=cout, p=16, q=16, r=3, stride=1, pad=1)
    a.x, a.dy, a.dw = xd.data_ptr(), gyd.data_ptr(), dw.data_ptr()
    if act:
        a.x_xf = L.Xform(kind=L.X_ACT, channels=cin, slope=0.01)
    if bias:
        a.db = db.data_ptr()
    ws = give_workspace(a, "vae_conv2d_bwd_filter")
    from gpu_util import launched
    log = launched(lambda: L.call("vae_conv2d_bwd_filter", ctypes.byref(a), torch.cuda.current_stream().cuda_stream))
    # the LDS-DMA weight-gradient kernel, or for an activated input the register-staged one
    assert ("c3w_kernel" if act else "c3wd_kernel") in log, log
    torch.cuda.synchronize()
    del ws
    got = (dw.cpu() - dw0).permute(0, 3, 1, 2)
    assert rel(got, w.grad) < 2e-3
    if bias:
        assert rel(db.cpu(), b.grad) < 2e-3


@pytest.mark.parametrize("n,cin,cout,act", [(8, 256, 256, True), (3, 128, 256, False)])
def test_c1_backward_filter(n, cin, cout, act):
    """Pointwise (1x1) weight gradient on a 16 x 16 grid (vae_c3.hip c1w), accumulated."""
    from vae_amd import _lib as L
    torch.manual_seed(14)
    x = _bf(torch.randn(n, cin, 16, 16))
    w = torch.zeros(cout, cin, 1, 1, requires_grad=True)
    y = F.conv2d(F.relu(x) if act else x, w)
    gy = _bf(torch.randn_like(y))
    y.backward(gy)
    dw0 = torch.randn(cout, 1, 1, cin) * 0.1
    xd = nhwc(x, torch.bfloat16)
    gyd = nhwc(gy, torch.bfloat16)
    dw = dw0.clone().cuda()
    a = L.ConvArgs(dtype=L.BF16, n=n, h=16, w=16, c=cin, k=cout, p=16, q=16, r=1, stride=1, pad=0)
    a.x, a.dy, a.dw = xd.data_ptr(), gyd.data_ptr(), dw.data_ptr()
    if act:
        a.x_xf = L.Xform(kind=L.X_ACT, channels=cin, slope=0.0)
    ws = give_workspace(a, "vae_conv2d_bwd_filter")
    L.call("vae_conv2d_bwd_filter", ctypes.byref(a), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    del ws
    assert rel((dw.cpu() - dw0).permute(0, 3, 1, 2), w.grad) < 2e-3


@pytest.mark.parametrize("n,cin,cout,act,res,res_act,bias", [(4, 256, 256, True, True, True, False),
                                                             (3, 128, 256, False, True, False, True),
                                                             (2, 256, 128, True, False, False, False)])
def test_p1_forward(n, cin, cout, act, res, res_act, bias):
    """1x1 conv forward on the pixel-tile kernel (vae_p1.hip): relu/lrelu(x) @ W^T + b + xf(skip)."""
    from vae_amd import _lib as L
    torch.manual_seed(15)
    x = _bf(torch.randn(n, cin, 16, 16))
    w = _bf(torch.randn(cout, cin, 1, 1) * (1.0 / cin ** 0.5))
    b = torch.randn(cout) * 0.1 if bias else None
    r = _bf(torch.randn(n, cout, 16, 16)) if res else None
    ref = F.conv2d(F.relu(x) if act else x, w, b)
    if res:
        ref = ref + (F.leaky_relu(r, 0.01) if res_act else r)
    xd, out = nhwc(x, torch.bfloat16), torch.empty(n, 16, 16, cout, device="cuda", dtype=torch.bfloat16)
    wd = w.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)
    a = L.ConvArgs(dtype=L.BF16, n=n, h=16, w=16, c=cin, k=cout, p=16, q=16, r=1, stride=1, pad=0)
    a.x, a.wt, a.y = xd.data_ptr(), wd.data_ptr(), out.data_ptr()
    keep = []
    if act:
        a.x_xf = L.Xform(kind=L.X_ACT, channels=cin, slope=0.0)
    if bias:
        bd = b.cuda()
        keep.append(bd)
        a.bias = bd.data_ptr()
    if res:
        rd = nhwc(r, torch.bfloat16)
        keep.append(rd)
        a.residual = rd.data_ptr()
        if res_act:
            a.residual_xf = L.Xform(kind=L.X_ACT, channels=cout, slope=0.01)
    from gpu_util import launched
    log = launched(lambda: L.call("vae_conv2d_fwd", ctypes.byref(a), torch.cuda.current_stream().cuda_stream))
    assert "p1d_kernel" in log, log                          # the LDS-DMA pointwise kernel ran
    torch.cuda.synchronize()
    assert rel(to_nchw(out), ref) < TOL


def test_p1_backward_data():
    """1x1 conv data gradient on the pixel-tile kernel: (dy @ W) * relu'(t)."""
    from vae_amd import _lib as L
    torch.manual_seed(16)
    n, cin, cout = 4, 256, 256
    w = _bf(torch.randn(cout, cin, 1, 1) * (1.0 / cin ** 0.5))
    gy = _bf(torch.randn(n, cout, 16, 16))
    t = _bf(torch.randn(n, cin, 16, 16))
    ref = F.conv_transpose2d(gy, w)
    ref = torch.where(t > 0, ref, ref * 0.0)
    gyd, td = nhwc(gy, torch.bfloat16), nhwc(t, torch.bfloat16)
    wt = w.permute(1, 2, 3, 0).contiguous().to("cuda", torch.bfloat16)
    wd = w.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)
    dx = torch.empty(n, 16, 16, cin, device="cuda", dtype=torch.bfloat16)
    a = L.ConvArgs(dtype=L.BF16, n=n, h=16, w=16, c=cin, k=cout, p=16, q=16, r=1, stride=1, pad=0)
    a.dy, a.wt, a.wt_t, a.dx = gyd.data_ptr(), wd.data_ptr(), wt.data_ptr(), dx.data_ptr()
    a.dx_epi = L.Xform(kind=L.X_ACT, channels=cin, slope=0.0, aux=td.data_ptr())
    L.call("vae_conv2d_bwd_data", ctypes.byref(a), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert rel(to_nchw(dx), ref) < TOL
