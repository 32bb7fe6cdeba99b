#!/usr/bin/env python3
"""Microbenchmark of the image-tile 3x3 kernels (csrc/vae_c3.hip) at the VQ-VAE's residual-conv
shape (B=128, 16 x 16, 256 -> 256 channels): forward, data gradient and weight gradient through the
C ABI, REPS launches each, for rocprofv3 kernel traces / PMC passes (diagnostic)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pytorch-vae_amd")]

import torch  # noqa: E402


def main():
    from vae_amd import _lib as L
    reps = int(os.environ.get("REPS", "20"))
    n, C, K = 128, 256, 256
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(n, 16, 16, C, device=dev, generator=g).bfloat16()
    dy = torch.randn(n, 16, 16, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(K, 3, 3, C, device=dev, generator=g) * 0.02).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous()
    y = torch.empty(n, 16, 16, K, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(n, 16, 16, C, device=dev, dtype=torch.bfloat16)
    dw = torch.zeros(K, 3, 3, C, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    a = L.ConvArgs(dtype=L.BF16, n=n, h=16, w=16, c=C, k=K, p=16, q=16, r=3, stride=1, pad=1)
    a.x, a.wt, a.wt_t, a.y, a.dy, a.dx, a.dw = (x.data_ptr(), w.data_ptr(), wt.data_ptr(), y.data_ptr(),
                                                 dy.data_ptr(), dx.data_ptr(), dw.data_ptr())
    a.x_xf = L.Xform(kind=L.X_ACT, channels=C, slope=0.01)
    need = L.workspace_size("vae_conv2d_bwd_filter", a)
    ws = torch.empty(max(1, need // 4 + 1), device=dev)
    a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel() * 4
    for fn in ("vae_conv2d_fwd", "vae_conv2d_bwd_data", "vae_conv2d_bwd_filter"):
        for _ in range(reps):
            L.call(fn, ctypes.byref(a), st)
        torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for fn in ("vae_conv2d_fwd", "vae_conv2d_bwd_data", "vae_conv2d_bwd_filter"):
        ev[0].record()
        for _ in range(reps):
            L.call(fn, ctypes.byref(a), st)
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) * 1000 / reps
        print(f"{fn:24s} {us:8.2f} us/call  {2 * n * 256 * K * 9 * C / us / 1e6:7.1f} TF/s", flush=True)
    # the ResidualLayer's 1x1 weight gradient
    b = L.ConvArgs(dtype=L.BF16, n=n, h=16, w=16, c=C, k=K, p=16, q=16, r=1, stride=1, pad=0)
    b.x, b.dy, b.dw = x.data_ptr(), dy.data_ptr(), dw.data_ptr()
    b.x_xf = L.Xform(kind=L.X_ACT, channels=C, slope=0.0)
    b.workspace, b.workspace_bytes = ws.data_ptr(), ws.numel() * 4
    for _ in range(reps):
        L.call("vae_conv2d_bwd_filter", ctypes.byref(b), st)
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        L.call("vae_conv2d_bwd_filter", ctypes.byref(b), st)
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1000 / reps
    print(f"{'1x1 bwd_filter':24s} {us:8.2f} us/call  {2 * n * 256 * K * C / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
