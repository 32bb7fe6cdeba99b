#!/usr/bin/env python3
"""Calibration (diagnostic, not the product): the VanillaVAE training step written with plain
torch.nn on the GPU (MIOpen convolutions, channels-last bf16 autocast or fp32), timed per step
and per layer, to know what the vendor stack reaches on MI355X for these exact shapes.

    python3 tools/calib_torch_gpu.py [--batch 64] [--dtype bf16]
"""
import argparse
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


def vanilla(latent=128, hd=(32, 64, 128, 256, 512)):
    enc, c = [], 3
    for h in hd:
        enc += [nn.Conv2d(c, h, 3, 2, 1), nn.BatchNorm2d(h), nn.LeakyReLU()]
        c = h
    rev = list(hd[::-1])
    dec = []
    for i in range(len(rev) - 1):
        dec += [nn.ConvTranspose2d(rev[i], rev[i + 1], 3, 2, 1, 1), nn.BatchNorm2d(rev[i + 1]), nn.LeakyReLU()]
    fin = [nn.ConvTranspose2d(rev[-1], rev[-1], 3, 2, 1, 1), nn.BatchNorm2d(rev[-1]), nn.LeakyReLU(),
           nn.Conv2d(rev[-1], 3, 3, 1, 1), nn.Tanh()]
    return nn.ModuleDict(dict(enc=nn.Sequential(*enc), fc=nn.Linear(hd[-1] * 4, 2 * latent),
                              din=nn.Linear(latent, hd[-1] * 4), dec=nn.Sequential(*dec), fin=nn.Sequential(*fin)))


def step(m, x, eps, hd_last=512):
    h = m["enc"](x).flatten(1)
    mu, lv = m["fc"](h).chunk(2, dim=1)
    z = eps * torch.exp(0.5 * lv) + mu
    r = m["din"](z).view(-1, hd_last, 2, 2)
    rec = m["fin"](m["dec"](r))
    recon = F.mse_loss(rec.float(), x.float())
    kld = torch.mean(-0.5 * torch.sum(1 + lv - mu ** 2 - lv.exp(), dim=1), dim=0)
    return recon + 1e-8 * kld


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    dev = "cuda"
    torch.backends.cudnn.benchmark = True
    m = vanilla().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.Adam(m.parameters(), lr=5e-3)
    x = torch.rand(a.batch, 3, 64, 64, device=dev).to(memory_format=torch.channels_last)
    eps = torch.randn(a.batch, 128, device=dev)
    ac = torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.dtype == "bf16")

    def one():
        with ac:
            loss = step(m, x, eps)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    for _ in range(10):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(f"torch eager {a.dtype} step: {dt * 1e3:.3f} ms  ({a.batch / dt:.0f} img/s)")
    # per-layer conv forward / backward
    shapes = [("conv", 3, 32, 64), ("conv", 32, 64, 32), ("conv", 64, 128, 16), ("conv", 128, 256, 8), ("conv", 256, 512, 4),
              ("convT", 512, 256, 2), ("convT", 256, 128, 4), ("convT", 128, 64, 8), ("convT", 64, 32, 16), ("convT", 32, 32, 32),
              ("head", 32, 3, 64)]
    dt_ = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    for kind, ci, co, hw in shapes:
        xi = torch.randn(a.batch, ci, hw, hw, device=dev, dtype=dt_).to(memory_format=torch.channels_last).requires_grad_(True)
        if kind == "conv":
            L = nn.Conv2d(ci, co, 3, 2, 1).to(dev, dt_).to(memory_format=torch.channels_last)
        elif kind == "convT":
            L = nn.ConvTranspose2d(ci, co, 3, 2, 1, 1).to(dev, dt_).to(memory_format=torch.channels_last)
        else:
            L = nn.Conv2d(ci, co, 3, 1, 1).to(dev, dt_).to(memory_format=torch.channels_last)
        y = L(xi)
        g = torch.randn_like(y)
        for _ in range(5):
            L(xi).backward(g)
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        n = 20
        e[0].record()
        for _ in range(n):
            y = L(xi)
        e[1].record()
        for _ in range(n):
            torch.autograd.grad(y, [xi, L.weight], g, retain_graph=True)
        e[2].record()
        torch.cuda.synchronize()
        print(f"{kind:5s} {ci:4d}->{co:4d} @{hw:3d}: fwd {e[0].elapsed_time(e[1]) / n * 1e3:7.1f} us  "
              f"bwd(data+filter) {e[1].elapsed_time(e[2]) / n * 1e3:7.1f} us")


if __name__ == "__main__":
    main()
