"""The LDS-DMA conv GEMM (csrc/vae_bgemm.hip) through the C ABI, against the exact emulation of
tests/test_gpu_cgemm.py (same roundings in torch, fp64 conv; bars: output max-abs <= 6e-3 of its
max, per-channel sums <= 1e-3).

It takes the transform-free large layers — the Autoencoder's wide convs / transposed convs at
B = 64 (models/autoencoder.py:16-86 with configs/big_ae.yaml widths), the VQ-VAE's strided 4x4
layers at B = 128 — forward (bias + BatchNorm statistics epilogue) and data gradient (activation
backward + BatchNorm-backward sums), with and without split-K; each case also checks, through the
library's launch log, that bgemm_kernel is the kernel that ran."""
import ctypes

import pytest
import torch

from test_gpu_cgemm import run_dgrad, run_fwd

pytestmark = pytest.mark.gpu


def _launched(fn):
    from vae_amd import _lib as L
    lib = L.load()
    lib.vae_launch_log(1)
    try:
        fn()
    finally:
        lib.vae_launch_log(0)
    need = lib.vae_launch_log_names(None, 0)
    buf = ctypes.create_string_buffer(int(need))
    lib.vae_launch_log_names(buf, need)
    return buf.value.decode()


FWD = [  # N, cin, cout, hw, stride, R, pad
    (64, 128, 256, 32, 2, 3, 1),        # big_ae encoder.1 (256 tiles, split 2)
    (64, 256, 512, 16, 2, 3, 1),        # big_ae encoder.2 (split-K)
    (64, 1024, 2048, 4, 2, 3, 1),       # big_ae encoder.4 (16 tiles: deep split)
    (128, 128, 256, 32, 2, 4, 1),       # VQ-VAE encoder.1 (k4 s2)
]


@pytest.mark.parametrize("shape", FWD)
def test_bgemm_conv2d_fwd(shape):
    from vae_amd import _lib as L
    log = _launched(lambda: run_fwd(False, *shape, L.X_NONE))
    assert "bgemm_kernel" in log, log


CONVT = [
    (64, 2048, 1024, 2, 2, 3, 1),       # big_ae decoder.0
    (64, 256, 128, 16, 2, 3, 1),        # big_ae decoder.3
    (128, 256, 128, 16, 2, 4, 1),       # VQ-VAE decoder ConvT(256 -> 128)
]


@pytest.mark.parametrize("shape", CONVT)
@pytest.mark.parametrize("give_wt_t", [False, True])
def test_bgemm_convT2d_fwd(shape, give_wt_t):
    from vae_amd import _lib as L
    log = _launched(lambda: run_fwd(True, *shape, L.X_NONE, give_wt_t=give_wt_t))
    assert "bgemm_kernel" in log, log


DGRAD = [  # N, cin, cout, hw (conv input), stride, R, pad
    (64, 256, 512, 16, 2, 3, 1),        # big_ae encoder.2 data gradient
    (128, 128, 256, 32, 2, 4, 1),       # VQ-VAE encoder.1
]


@pytest.mark.parametrize("shape", DGRAD)
@pytest.mark.parametrize("epi", ["bn_act", "act"])
def test_bgemm_conv2d_bwd_data(shape, epi):
    from vae_amd import _lib as L
    e = L.X_BN_ACT if epi == "bn_act" else L.X_ACT
    log = _launched(lambda: run_dgrad(False, *shape, L.X_NONE, e))
    assert "bgemm_kernel" in log, log


DGRAD_T = [  # N, cin, cout, hw (transposed conv input), stride, R, pad
    (64, 512, 256, 8, 2, 3, 1),         # big_ae decoder.2 data gradient
    (64, 128, 128, 32, 2, 3, 1),        # big_ae final ConvT (19.3 GFLOP)
    (128, 256, 128, 16, 2, 4, 1),       # VQ-VAE decoder ConvT
]


@pytest.mark.parametrize("shape", DGRAD_T)
def test_bgemm_convT2d_bwd_data(shape):
    from vae_amd import _lib as L
    log = _launched(lambda: run_dgrad(True, *shape, L.X_NONE, L.X_BN_ACT if shape[5] == 3 else L.X_ACT))
    assert "bgemm_kernel" in log, log


def test_bn_apply_matches_torch():
    """vae_bn_apply: lrelu(BN(y)) from a coefficient table, lrelu(y), and A g + B y + C."""
    from gpu_util import nhwc
    from test_gpu_cgemm import Xf, bf
    from vae_amd import _lib as L
    g = torch.Generator().manual_seed(3)
    n, C, hw = 4, 256, 8
    y = bf(torch.randn(n, C, hw, hw, generator=g))
    gr = bf(torch.randn(n, C, hw, hw, generator=g))
    a_, b_ = 0.5 + torch.rand(C, generator=g), torch.rand(C, generator=g) - 0.5
    c_ = (torch.rand(C, generator=g) - 0.5) * 0.1
    yd, gd = nhwc(y, torch.bfloat16), nhwc(gr, torch.bfloat16)
    cases = [
        (L.X_BN_ACT, yd, torch.cat([a_, b_, torch.zeros(2 * C)]), None,
         torch.nn.functional.leaky_relu(y * a_.view(1, -1, 1, 1) + b_.view(1, -1, 1, 1), 0.01)),
        (L.X_ACT, yd, None, None, torch.nn.functional.leaky_relu(y, 0.01)),
        (L.X_BN_DY, gd, torch.cat([a_, b_, c_]), yd,
         a_.view(1, -1, 1, 1) * gr + b_.view(1, -1, 1, 1) * y + c_.view(1, -1, 1, 1)),
    ]
    for kind, src, table, aux, want in cases:
        xf = Xf(L, kind, C, table=table, aux=aux)
        out = torch.empty_like(src)
        a = L.BnApplyArgs(dtype=L.BF16, rows=n * hw * hw, channels=C)
        a.x, a.xf, a.out = src.data_ptr(), xf.x, out.data_ptr()
        L.call("vae_bn_apply", ctypes.byref(a), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = out.float().permute(0, 3, 1, 2).cpu()
        err = float((got - want).abs().max() / want.abs().max())
        assert err < 8e-3, (kind, err)


WGRAD_B = [  # transposed, N, cin, cout, hw (input grid), stride, R, pad
    (False, 64, 256, 512, 16, 2, 3, 1),     # big_ae encoder.2 (K split over workgroups: atomics)
    (False, 64, 1024, 2048, 4, 2, 3, 1),    # big_ae encoder.4 (one K slice: plain accumulate)
    (True, 64, 512, 256, 8, 2, 3, 1),       # big_ae decoder ConvT
    (False, 64, 128, 256, 32, 2, 4, 1),     # VQ-VAE encoder.1 (k4 s2)
    (True, 64, 256, 128, 16, 2, 4, 1),      # VQ-VAE decoder ConvT(256 -> 128)
    (True, 64, 256, 128, 16, 2, 3, 1),      # big_ae decoder.3 (16384 pixels, 26 K slices)
    (True, 64, 128, 128, 32, 2, 3, 1),      # big_ae final ConvT (65536 pixels, 54 K slices)
    (True, 16, 128, 128, 32, 2, 3, 1),      # the same at B=16 (tests/test_gpu_ae_wide.py)
]


@pytest.mark.parametrize("shape", WGRAD_B)
def test_bwg_weight_gradient(shape):
    """Weight gradients of transform-free operands (the materialised activation / gradient) on the
    LDS-DMA kernel (bwg_kernel), against the fp64 autograd weight gradient (bar 2e-3 of max)."""
    from test_gpu_cgemm import run_wgrad
    from vae_amd import _lib as L
    tr, *rest = shape
    log = _launched(lambda: run_wgrad(tr, *rest, L.X_NONE, L.X_NONE))
    assert "bwg_kernel" in log, log
