"""The bf16 conv-GEMM path (csrc/vae_cgemm.hpp) through the C ABI, against an exact emulation.

bf16 mode rounds each operand to bf16 once (stored activations, the transformed operand on its
way into LDS, the weight copy) and accumulates in fp32.  The reference here applies the same
roundings in torch (transform in fp32 -> bf16, weights -> bf16) and then computes the conv in
fp64, so the only differences left are the fp32 summation order and the final bf16 rounding of
the output: max-abs error <= 6e-3 of the output's max (bf16 has 8 significant bits, 2^-8 =
3.9e-3), per-channel sums <= 1e-3.  That is ~3x tighter than the generic bf16 bar of
tests/test_gpu_ops.py and pins the new kernel's indexing (taps, phases, tiles, split-K).

Shapes cover every tile the planner picks (32x32 .. 128x128), split-K, the sub-pixel phases of
k3 s2 p1 op1 and k4 s2 p1 transposed convs, stride-1 data gradients, 8-channel (padded RGB)
operands, and both sources of the swapped-axes weights (caller's wt_t / built in the
workspace)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from gpu_util import give_workspace

pytestmark = pytest.mark.gpu

SLOPE = 0.01
OUT_TOL = 6e-3


def _L():
    from vae_amd import _lib as L
    return L


def bf(t):
    return t.to(torch.bfloat16).float()


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)


def nchw(t):
    return t.float().permute(0, 3, 1, 2).contiguous().cpu()


def relmax(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


class Xf:
    """A transform descriptor with a caller-made coefficient table (what vae_bn_finalize
    writes) plus the dummy statistics pointers the ABI validates."""

    def __init__(self, L, kind, C, table=None, aux=None):
        self.keep = [torch.zeros(4 * C, device="cuda")]
        d = self.keep[0]
        self.x = L.Xform(kind=kind, channels=C, slope=SLOPE, count=1.0, eps=1e-5, momentum=0.1)
        if kind in (L.X_BN_ACT, L.X_BN_DY):
            self.x.sum = self.x.sumsq = self.x.gamma = self.x.beta = d.data_ptr()
            self.x.dgamma = self.x.dbeta = d.data_ptr()
            t = table.contiguous().float().cuda()
            self.keep.append(t)
            self.x.table = t.data_ptr()
        if aux is not None:
            self.x.aux = aux.data_ptr()


def bn_act_table(C, g):
    a = 0.5 + torch.rand(C, generator=g)
    b = torch.rand(C, generator=g) - 0.5
    return a, b


def emulate_act(kind, L, y, a=None, b=None):
    """The kernel's A operand in NCHW fp32: transform in fp32 then round to bf16."""
    if kind == L.X_NONE:
        return y
    if kind == L.X_ACT:
        return bf(F.leaky_relu(y, SLOPE))
    return bf(F.leaky_relu(y * a.view(1, -1, 1, 1) + b.view(1, -1, 1, 1), SLOPE))


def run_fwd(transposed, N, cin, cout, hw, stride, R, pad, kind, split=0, give_wt_t=False, seed=0):
    L = _L()
    g = torch.Generator().manual_seed(seed)
    y = bf(torch.randn(N, cin, hw, hw, generator=g))
    a_t, b_t = bn_act_table(cin, g)
    if transposed:
        w = bf(torch.randn(cin, cout, R, R, generator=g) * 0.1)
        P = (hw - 1) * stride - 2 * pad + R + (stride - 1 if R == 3 else 0)
    else:
        w = bf(torch.randn(cout, cin, R, R, generator=g) * 0.1)
        P = (hw + 2 * pad - R) // stride + 1
    bias = torch.randn(cout, generator=g) * 0.1
    act = emulate_act(kind, L, y, a_t, b_t).double()
    if transposed:
        acc = F.conv_transpose2d(act, w.double(), None, stride=stride, padding=pad,
                                 output_padding=(stride - 1 if R == 3 else 0))
    else:
        acc = F.conv2d(act, w.double(), None, stride=stride, padding=pad)
    ref = acc + bias.double().view(1, -1, 1, 1)
    yd = nhwc(y)
    wd = w.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)
    out = torch.empty(N, P, P, cout, device="cuda", dtype=torch.bfloat16)
    sums = torch.zeros(2 * cout, device="cuda")
    bd = bias.cuda()
    xf = Xf(L, kind, cin, table=torch.cat([a_t, b_t, torch.zeros(2 * cin)]) if kind == L.X_BN_ACT else None)
    a = L.ConvArgs(dtype=L.BF16, n=N, h=hw, w=hw, c=cin, k=cout, p=P, q=P, r=R, stride=stride, pad=pad)
    a.x = yd.data_ptr(); a.x_xf = xf.x; a.wt = wd.data_ptr(); a.bias = bd.data_ptr(); a.y = out.data_ptr()
    a.y_sum = sums.data_ptr(); a.y_sumsq = sums.data_ptr() + 4 * cout
    a.split_k = split
    if give_wt_t:
        wt = w.permute(1, 2, 3, 0).contiguous().to("cuda", torch.bfloat16)     # [cout][r][s][cin]
        a.wt_t = wt.data_ptr()
    ws = give_workspace(a, "vae_convT2d_fwd" if transposed else "vae_conv2d_fwd")
    L.call("vae_convT2d_fwd" if transposed else "vae_conv2d_fwd", ctypes.byref(a), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert relmax(nchw(out), ref) < OUT_TOL
    assert relmax(sums[:cout].cpu(), acc.sum((0, 2, 3))) < 1e-3
    assert relmax(sums[cout:].cpu(), (acc * acc).sum((0, 2, 3))) < 1e-3


FWD = [  # N, cin, cout, hw, stride, R, pad
    (8, 32, 64, 32, 2, 3, 1),
    (4, 64, 128, 16, 2, 3, 1),
    (4, 128, 256, 8, 2, 3, 1),
    (2, 256, 512, 4, 2, 3, 1),          # deep K, few rows: split-K
    (16, 256, 256, 16, 1, 3, 1),        # VQ-VAE residual 3x3 (large tiles)
    (8, 8, 32, 64, 2, 3, 1),            # padded-RGB first layer
    (8, 128, 256, 32, 2, 4, 1),         # VQ-VAE encoder k4 s2
]


@pytest.mark.parametrize("shape", FWD)
@pytest.mark.parametrize("kind", ["none", "act", "bn_act"])
def test_cgemm_conv2d_fwd(shape, kind):
    L = _L()
    k = {"none": L.X_NONE, "act": L.X_ACT, "bn_act": L.X_BN_ACT}[kind]
    run_fwd(False, *shape, k)


def test_cgemm_conv2d_fwd_split():
    L = _L()
    run_fwd(False, 4, 64, 128, 16, 2, 3, 1, L.X_BN_ACT, split=3)


CONVT = [  # N, cin, cout, hw, stride, R, pad
    (8, 512, 256, 2, 2, 3, 1),
    (8, 256, 128, 4, 2, 3, 1),
    (8, 64, 32, 16, 2, 3, 1),
    (8, 32, 32, 32, 2, 3, 1),
    (8, 256, 128, 16, 2, 4, 1),         # VQ-VAE decoder k4 s2
]


@pytest.mark.parametrize("shape", CONVT)
@pytest.mark.parametrize("give_wt_t", [False, True])
def test_cgemm_convT2d_fwd(shape, give_wt_t):
    L = _L()
    run_fwd(True, *shape, L.X_BN_ACT if shape[5] == 3 else L.X_ACT, give_wt_t=give_wt_t)


def run_dgrad(transposed, N, cin, cout, hw, stride, R, pad, dy_kind, epi_kind, give_wt_t=False, seed=1):
    """dx of conv2d / conv_transpose2d: dy (optionally through BN-backward on load), then the
    epilogue's activation backward (+ Σg, Σg·x̂ for a BatchNorm-followed input)."""
    L = _L()
    g = torch.Generator().manual_seed(seed)
    if transposed:
        w = bf(torch.randn(cin, cout, R, R, generator=g) * 0.1)
        P = (hw - 1) * stride - 2 * pad + R + (stride - 1 if R == 3 else 0)
    else:
        w = bf(torch.randn(cout, cin, R, R, generator=g) * 0.1)
        P = (hw + 2 * pad - R) // stride + 1
    gy = bf(torch.randn(N, cout, P, P, generator=g))             # stored gradient
    yst = bf(torch.randn(N, cout, P, P, generator=g))            # stored pre-activation of the output
    A, Bc, Cc = (0.5 + torch.rand(cout, generator=g), torch.rand(cout, generator=g) - 0.5,
                 (torch.rand(cout, generator=g) - 0.5) * 0.1)
    if dy_kind == L.X_BN_DY:
        dyp = bf(A.view(1, -1, 1, 1) * gy + Bc.view(1, -1, 1, 1) * yst + Cc.view(1, -1, 1, 1))
    else:
        dyp = gy
    x0 = torch.zeros(N, cin, hw, hw, dtype=torch.float64, requires_grad=True)
    if transposed:
        out = F.conv_transpose2d(x0, w.double(), None, stride=stride, padding=pad,
                                 output_padding=(stride - 1 if R == 3 else 0))
    else:
        out = F.conv2d(x0, w.double(), None, stride=stride, padding=pad)
    out.backward(dyp.double())
    v = x0.grad
    xst = bf(torch.randn(N, cin, hw, hw, generator=g))           # stored pre-activation of x
    ea, eb = bn_act_table(cin, g)
    ep, eq = 0.5 + torch.rand(cin, generator=g), torch.rand(cin, generator=g) - 0.5
    if epi_kind == L.X_BN_ACT:
        z = xst * ea.view(1, -1, 1, 1) + eb.view(1, -1, 1, 1)
        gout = torch.where(z > 0, v, v * SLOPE)
        s1 = gout.sum((0, 2, 3))
        s2 = (gout * (xst * ep.view(1, -1, 1, 1) + eq.view(1, -1, 1, 1))).sum((0, 2, 3))
    elif epi_kind == L.X_ACT:
        gout = torch.where(xst > 0, v, v * SLOPE)
    else:
        gout = v
    gyd, ystd, xstd = nhwc(gy), nhwc(yst), nhwc(xst)
    wd = w.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)
    dx = torch.empty(N, hw, hw, cin, device="cuda", dtype=torch.bfloat16)
    dgam = torch.zeros(cin, device="cuda"); dbet = torch.zeros(cin, device="cuda")
    dyx = Xf(L, dy_kind, cout, table=torch.cat([A, Bc, Cc]) if dy_kind == L.X_BN_DY else None,
             aux=ystd if dy_kind == L.X_BN_DY else None)
    epx = Xf(L, epi_kind, cin, table=torch.cat([ea, eb, ep, eq]) if epi_kind == L.X_BN_ACT else None,
             aux=xstd if epi_kind != L.X_NONE else None)
    a = L.ConvArgs(dtype=L.BF16, n=N, h=hw, w=hw, c=cin, k=cout, p=P, q=P, r=R, stride=stride, pad=pad)
    a.dy = gyd.data_ptr(); a.dy_xf = dyx.x; a.wt = wd.data_ptr(); a.dx = dx.data_ptr(); a.dx_epi = epx.x
    a.dx_dgamma = dgam.data_ptr(); a.dx_dbeta = dbet.data_ptr()
    if give_wt_t:
        wt = w.permute(1, 2, 3, 0).contiguous().to("cuda", torch.bfloat16)
        a.wt_t = wt.data_ptr()
    ws = give_workspace(a, "vae_convT2d_bwd_data" if transposed else "vae_conv2d_bwd_data")
    L.call("vae_convT2d_bwd_data" if transposed else "vae_conv2d_bwd_data", ctypes.byref(a),
           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert relmax(nchw(dx), gout) < OUT_TOL
    if epi_kind == L.X_BN_ACT:
        assert relmax(dbet.cpu(), s1) < 1e-3
        assert relmax(dgam.cpu(), s2) < 1e-3


DGRAD = [  # N, cin, cout, hw (input of the conv), stride, R, pad
    (8, 32, 64, 16, 2, 3, 1),
    (8, 128, 256, 8, 2, 3, 1),
    (8, 256, 512, 4, 2, 3, 1),
    (8, 256, 256, 16, 1, 3, 1),          # VQ-VAE residual 3x3 data gradient
    (8, 128, 256, 32, 2, 4, 1),          # VQ-VAE encoder k4 s2
]


@pytest.mark.parametrize("shape", DGRAD)
@pytest.mark.parametrize("give_wt_t", [False, True])
def test_cgemm_conv2d_bwd_data(shape, give_wt_t):
    L = _L()
    run_dgrad(False, *shape, L.X_BN_DY, L.X_BN_ACT, give_wt_t=give_wt_t)


@pytest.mark.parametrize("epi", ["none", "act"])
def test_cgemm_conv2d_bwd_data_plain(epi):
    L = _L()
    run_dgrad(False, 8, 256, 256, 16, 1, 3, 1, L.X_NONE, L.X_NONE if epi == "none" else L.X_ACT)


DGRAD_T = [  # N, cin, cout, hw (input of the transposed conv), stride, R, pad
    (8, 512, 256, 2, 2, 3, 1),
    (8, 64, 32, 16, 2, 3, 1),
    (8, 32, 32, 32, 2, 3, 1),
    (8, 256, 128, 16, 2, 4, 1),
]


@pytest.mark.parametrize("shape", DGRAD_T)
def test_cgemm_convT2d_bwd_data(shape):
    L = _L()
    run_dgrad(True, *shape, L.X_BN_DY if shape[5] == 3 else L.X_NONE, L.X_BN_ACT if shape[5] == 3 else L.X_ACT)


# ---------------------------------------------------------------------------------------------
# Weight gradients (csrc/vae_wgemm.hpp) with the BatchNorm coefficients built in-kernel from
# the statistics (no precomputed table: vae_common.hpp tab_build), plus the closed-form conv
# bias gradient and dL/dgamma, dL/dbeta published by the first workgroup.

class BN:
    """A stored pre-BN tensor with consistent statistics (reps=1 sums over N*H*W, shift = the
    producing conv's bias) as the producing kernels leave them."""

    def __init__(self, y, g, shift=None):
        C = y.shape[1]
        self.y = y
        self.gamma = 0.7 + 0.6 * torch.rand(C, generator=g)
        self.beta = (torch.rand(C, generator=g) - 0.5) * 0.2
        self.shift = shift if shift is not None else torch.zeros(C)
        d = (y - self.shift.view(1, -1, 1, 1)).double()
        self.sum = d.sum((0, 2, 3)).float()
        self.sumsq = (d * d).sum((0, 2, 3)).float()
        self.count = y.numel() // C
        self.keep = []

    def xf(self, L, kind, aux_dev=None, dgamma=None, dbeta=None, dgamma_out=None, dbeta_out=None):
        C = self.gamma.numel()
        x = L.Xform(kind=kind, channels=C, slope=SLOPE, count=float(self.count), eps=1e-5, momentum=0.1)
        for name in ("sum", "sumsq", "shift", "gamma", "beta"):
            t = getattr(self, name).float().cuda()
            self.keep.append(t)
            setattr(x, name, t.data_ptr())
        x.reps, x.rstride = 1, C
        if dgamma is not None:
            for name, t in (("dgamma", dgamma), ("dbeta", dbeta)):
                t = t.float().cuda()
                self.keep.append(t)
                setattr(x, name, t.data_ptr())
        if dgamma_out is not None:
            x.dgamma_out, x.dbeta_out = dgamma_out.data_ptr(), dbeta_out.data_ptr()
        if aux_dev is not None:
            x.aux = aux_dev.data_ptr()
        return x

    def act(self):
        z = F.batch_norm(self.y.double(), None, None, self.gamma.double(), self.beta.double(), True, 0.1, 1e-5)
        return bf(F.leaky_relu(z, SLOPE).float())


def prep_wgrad(transposed, N, cin, cout, hw, stride, R, pad, x_kind, dy_kind, seed=3):
    """One bf16 weight-gradient call's arguments (kernel-side operands) and its fp64 reference."""
    L = _L()
    g = torch.Generator().manual_seed(seed)
    if transposed:
        P = (hw - 1) * stride - 2 * pad + R + (stride - 1 if R == 3 else 0)
        wshape = (cin, cout, R, R)
    else:
        P = (hw + 2 * pad - R) // stride + 1
        wshape = (cout, cin, R, R)
    xst = bf(torch.randn(N, cin, hw, hw, generator=g) * 1.3 + 0.2)
    yst = bf(torch.randn(N, cout, P, P, generator=g) * 1.1 - 0.1)      # pre-BN output (BN_DY aux)
    gst = bf(torch.randn(N, cout, P, P, generator=g))                   # dL/dz of its BatchNorm
    bnx = BN(xst, g)
    bny = BN(yst, g, shift=torch.randn(cout, generator=g) * 0.1)
    # operands as the kernel forms them
    if x_kind == L.X_BN_ACT:
        act = bnx.act()
    elif x_kind == L.X_ACT:
        act = bf(F.leaky_relu(xst, SLOPE))
    else:
        act = xst
    if dy_kind == L.X_BN_DY:
        yv = yst.double().requires_grad_(True)
        z = F.batch_norm(yv, None, None, bny.gamma.double(), bny.beta.double(), True, 0.1, 1e-5)
        z.backward(gst.double())
        dyp = bf(yv.grad.float())
        db_exact = yv.grad.sum((0, 2, 3))          # ~0: a train-mode BatchNorm's input gradient sums to 0
        xh = ((yst.double() - yst.double().mean((0, 2, 3), keepdim=True)) /
              torch.sqrt(yst.double().var((0, 2, 3), unbiased=False, keepdim=True) + 1e-5))
        dgam, dbet = (gst.double() * xh).sum((0, 2, 3)), gst.double().sum((0, 2, 3))
    else:
        dyp, dgam, dbet, db_exact = gst, None, None, None
    w0 = torch.zeros(wshape, dtype=torch.float64, requires_grad=True)
    if transposed:
        out = F.conv_transpose2d(act.double(), w0, None, stride=stride, padding=pad,
                                 output_padding=(stride - 1 if R == 3 else 0))
    else:
        out = F.conv2d(act.double(), w0, None, stride=stride, padding=pad)
    out.backward(dyp.double())
    want = w0.grad.permute(0, 2, 3, 1)                                 # native [a][r][s][b]
    xd, yd, gd = nhwc(xst), nhwc(yst), nhwc(gst)
    dw = torch.zeros(want.shape, device="cuda")
    db = torch.zeros(cout, device="cuda")
    dgo = torch.zeros(cout, device="cuda"); dbo = torch.zeros(cout, device="cuda")
    a = L.ConvArgs(dtype=L.BF16, n=N, h=hw, w=hw, c=cin, k=cout, p=P, q=P, r=R, stride=stride, pad=pad)
    a.x = xd.data_ptr(); a.x_xf = bnx.xf(L, x_kind) if x_kind == L.X_BN_ACT else L.Xform(kind=x_kind, channels=cin, slope=SLOPE)
    a.dy = gd.data_ptr()
    if dy_kind == L.X_BN_DY:
        a.dy_xf = bny.xf(L, L.X_BN_DY, aux_dev=yd, dgamma=dgam, dbeta=dbet, dgamma_out=dgo, dbeta_out=dbo)
        a.db = db.data_ptr()
    a.dw = dw.data_ptr()
    fn = "vae_convT2d_bwd_filter" if transposed else "vae_conv2d_bwd_filter"
    return dict(a=a, fn=fn, want=want, dw=dw, db=db, dgo=dgo, dbo=dbo, db_exact=db_exact, dyp=dyp, dgam=dgam,
                dbet=dbet, keep=(xd, yd, gd, bnx, bny), R=R, untransformed=(x_kind == L.X_NONE and dy_kind == L.X_NONE))


def check_wgrad(w):
    """The call's dW (and closed-form bias / BN affine gradients) against the fp64 reference."""
    torch.cuda.synchronize()
    dw, want, R = w["dw"], w["want"], w["R"]
    assert relmax(dw.cpu(), want) < 2e-3
    if w["untransformed"]:
        # untransformed operands are exact bf16 in the fp64 reference: only fp32 accumulation order
        # separates the two, so the whole tensor must agree to ~1e-6 (a dropped or doubled K slice,
        # tap or row block shows here long before it moves the max-abs bar)
        d = dw.cpu().double() - want
        err = float(d.norm() / want.norm())
        if not err < 1e-4:
            per_tap = [float(d[:, r, s_].norm() / want[:, r, s_].norm()) for r in range(R) for s_ in range(R)]
            raise AssertionError(f"weight gradient rel-norm error {err:.3e}; per tap {per_tap}")
    if w["db_exact"] is not None:
        # closed form A*Σg + B*Σy + C*M (vaehip.h bn_args): exact up to fp32 cancellation
        assert float((w["db"].cpu().double() - w["db_exact"]).abs().max()) < \
            1e-6 * float(w["dyp"].double().abs().sum((0, 2, 3)).max())
        assert relmax(w["dgo"].cpu(), w["dgam"]) < 1e-5 and relmax(w["dbo"].cpu(), w["dbet"]) < 1e-5


def run_wgrad(transposed, N, cin, cout, hw, stride, R, pad, x_kind, dy_kind, seed=3):
    """One standalone bf16 weight-gradient call (its queried workspace given) against fp64."""
    L = _L()
    w = prep_wgrad(transposed, N, cin, cout, hw, stride, R, pad, x_kind, dy_kind, seed)
    a, fn = w["a"], w["fn"]
    ws = give_workspace(a, fn)           # 4 bytes when the plan takes none
    L.call(fn, ctypes.byref(a), torch.cuda.current_stream().cuda_stream)
    check_wgrad(w)


WGRAD = [  # N, cin, cout, hw (conv input), stride, R, pad
    (8, 32, 64, 32, 2, 3, 1),
    (8, 64, 128, 16, 2, 3, 1),
    (8, 256, 512, 4, 2, 3, 1),
    (8, 8, 32, 64, 2, 3, 1),             # padded-RGB first layer (x untransformed)
]


@pytest.mark.parametrize("shape", WGRAD)
def test_wgemm_conv2d_bn(shape):
    L = _L()
    run_wgrad(False, *shape, L.X_NONE if shape[1] == 8 else L.X_BN_ACT, L.X_BN_DY)


def test_wgemm_conv2d_vq_shapes():
    L = _L()
    run_wgrad(False, 4, 256, 256, 16, 1, 3, 1, L.X_ACT, L.X_NONE)
    run_wgrad(False, 4, 128, 256, 32, 2, 4, 1, L.X_ACT, L.X_NONE)


WGRAD_T = [  # N, cin, cout, hw (convT input), stride, R, pad
    (8, 512, 256, 2, 2, 3, 1),
    (8, 128, 64, 8, 2, 3, 1),
    (8, 32, 32, 32, 2, 3, 1),
]


@pytest.mark.parametrize("shape", WGRAD_T)
def test_wgemm_convT2d_bn(shape):
    L = _L()
    run_wgrad(True, *shape, L.X_BN_ACT, L.X_BN_DY)


def test_wgemm_convT2d_vq_shape():
    L = _L()
    run_wgrad(True, 4, 256, 128, 16, 2, 4, 1, L.X_ACT, L.X_NONE)


def test_cgemm_fwd_table_built_in_kernel():
    """Forward conv with BN_ACT from the raw statistics (no table): tab_build + running stats."""
    L = _L()
    g = torch.Generator().manual_seed(9)
    N, cin, cout, hw = 8, 64, 128, 16
    y = bf(torch.randn(N, cin, hw, hw, generator=g) * 0.9 + 0.4)
    bn = BN(y, g, shift=torch.randn(cin, generator=g) * 0.05)
    w = bf(torch.randn(cout, cin, 3, 3, generator=g) * 0.1)
    ref = F.conv2d(bn.act().double(), w.double(), None, stride=2, padding=1)
    out = torch.empty(N, hw // 2, hw // 2, cout, device="cuda", dtype=torch.bfloat16)
    rm = torch.zeros(cin, device="cuda"); rv = torch.ones(cin, device="cuda")
    xf = bn.xf(L, L.X_BN_ACT)
    xf.running_mean, xf.running_var = rm.data_ptr(), rv.data_ptr()
    yd = nhwc(y)
    wd = w.permute(0, 2, 3, 1).contiguous().to("cuda", torch.bfloat16)
    a = L.ConvArgs(dtype=L.BF16, n=N, h=hw, w=hw, c=cin, k=cout, p=hw // 2, q=hw // 2, r=3, stride=2, pad=1)
    a.x = yd.data_ptr(); a.x_xf = xf; a.wt = wd.data_ptr(); a.y = out.data_ptr()
    L.call("vae_conv2d_fwd", ctypes.byref(a), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert relmax(nchw(out), ref) < OUT_TOL
    mean = y.double().mean((0, 2, 3))
    var_u = y.double().var((0, 2, 3), unbiased=True)
    assert relmax(rm.cpu(), 0.1 * mean) < 1e-4
    assert relmax(rv.cpu() - 0.9, 0.1 * var_u) < 1e-4


# the VanillaVAE backward's nine weight gradients (B = 16): convT decoder, conv encoder, padded RGB
BATCH = [(True, 16, 64, 32, 16, 2, 3, 1), (True, 16, 128, 64, 8, 2, 3, 1), (True, 16, 256, 128, 4, 2, 3, 1),
         (True, 16, 512, 256, 2, 2, 3, 1), (False, 16, 256, 512, 4, 2, 3, 1), (False, 16, 128, 256, 8, 2, 3, 1),
         (False, 16, 64, 128, 16, 2, 3, 1), (False, 16, 32, 64, 32, 2, 3, 1), (False, 16, 8, 32, 64, 2, 3, 1)]


def test_wgrad_batch_matches_reference_and_is_deterministic():
    """vae_conv_bwd_filter_batch (one XCD-partitioned grid, K-slice partials in slabs reduced in slice
    order): every layer's dW / bias / BN affine gradients against fp64, and two runs bit-identical."""
    L = _L()
    ws = []
    for seed, (tr, N, cin, cout, hw, s_, R, pad) in enumerate(BATCH):
        xk = L.X_BN_ACT if (tr and cin != 512) or (not tr and cin != 8) else L.X_NONE
        ws.append(prep_wgrad(tr, N, cin, cout, hw, s_, R, pad, xk, L.X_BN_DY, seed=10 + seed))
    n = len(ws)
    kinds = (ctypes.c_int32 * n)(*[L.LAYER_CONVT2D if w["fn"].startswith("vae_convT") else L.LAYER_CONV2D for w in ws])
    items = (ctypes.c_void_p * n)(*[ctypes.addressof(w["a"]) for w in ws])
    need = ctypes.c_size_t(0)
    L.call("vae_conv_bwd_filter_batch_workspace_size", n, kinds, items, ctypes.byref(need))
    wsb = torch.empty(max(16, need.value), dtype=torch.uint8, device="cuda")
    results = []
    for rep in range(2):
        for w in ws:
            for t in ("dw", "db", "dgo", "dbo"):
                w[t].zero_()
        L.call("vae_conv_bwd_filter_batch", n, kinds, items, wsb.data_ptr(), wsb.numel(),
               torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        results.append([w["dw"].clone() for w in ws] + [w["db"].clone() for w in ws])
        if rep == 0:
            for w in ws:
                check_wgrad(w)
    for a, b in zip(*results):
        assert torch.equal(a, b)
