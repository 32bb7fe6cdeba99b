#!/usr/bin/env python3
"""Microbenchmark of the decoder-head kernels (csrc/vae_head.hip) at the benchmarked shapes:
C = 32 (VanillaVAE, B = 64) and C = 128 (big_ae, B = 64), 64 x 64 images.  Times vae_head_fwd,
vae_head_bwd (data + filter), vae_head_bwd_data and vae_head_bwd_filter through the C ABI, REPS
back-to-back launches each with HIP events on the launch stream (diagnostic: which half of the
backward costs what)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pytorch-vae_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402


def bench(C, N, reps):
    from vae_amd import _lib as L
    from gpu_util import BNState, give_workspace
    H = 64
    g = torch.Generator().manual_seed(1)
    y_prev = torch.randn(N, C, H, H, generator=g)
    bn = BNState(y_prev, dtype=torch.bfloat16)
    w = torch.randn(3, C, 3, 3, generator=g) * 0.05
    wd = w.permute(0, 2, 3, 1).contiguous().cuda()
    bd = (torch.randn(3, generator=g) * 0.1).cuda()
    tg = torch.rand(N, 3, H, H, generator=g).cuda()
    recon = torch.empty(N, 3, H, H, device="cuda")
    sse = torch.zeros(N, device="cuda")
    coef = torch.full((N,), 2.0 / (N * 3 * H * H), device="cuda")
    dx = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
    dgp = torch.zeros(C, device="cuda")
    dbp = torch.zeros(C, device="cuda")
    dw = torch.zeros(wd.shape, device="cuda")
    db = torch.zeros(3, device="cuda")
    a = L.HeadArgs(dtype=L.BF16, n=N, h=H, w=H, c=C, samples=1)
    a.x = bn.y_dev.data_ptr(); a.x_xf = bn.xf(); a.wt = wd.data_ptr(); a.bias = bd.data_ptr()
    a.target = tg.data_ptr(); a.recon = recon.data_ptr(); a.sse = sse.data_ptr(); a.coef = coef.data_ptr()
    a.dx = dx.data_ptr(); a.dx_epi = bn.xf(aux=bn.y_dev); a.dx_dgamma = dgp.data_ptr(); a.dx_dbeta = dbp.data_ptr()
    a.dw = dw.data_ptr(); a.db = db.data_ptr()
    ws = give_workspace(a, "vae_head_bwd")  # noqa: F841 (kept alive)
    st = torch.cuda.current_stream().cuda_stream
    out = {}
    for fn in ("vae_head_fwd", "vae_head_bwd", "vae_head_bwd_data", "vae_head_bwd_filter"):
        for _ in range(3):
            L.call(fn, ctypes.byref(a), st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            L.call(fn, ctypes.byref(a), st)
        e1.record()
        torch.cuda.synchronize()
        out[fn] = e0.elapsed_time(e1) * 1e3 / reps
    return out


def main():
    reps = int(os.environ.get("REPS", "50"))
    for C in (32, 128):
        r = bench(C, 64, reps)
        print(f"C={C:4d} B=64  " + "  ".join(f"{k[9:]}: {v:7.2f} us" for k, v in r.items()), flush=True)


if __name__ == "__main__":
    main()
