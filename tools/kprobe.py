#!/usr/bin/env python3
"""Per-block phase timing of every GEMM launch of the step (diagnostic).

    make -C pytorch-vae_amd/csrc probe && VAE_HIP_LIB=probe python3 tools/kprobe.py

Uses libvaehip_probe.so, whose GEMM kernels append one record per block:
{block id, wall start, wall end, clk at start / tables ready / K-loop done / end, HW_ID}.
Prints, per launch: blocks, launch span (first start -> last end), and the median / max
per-block durations of the prologue (tables + first tile), K loop and epilogue.
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pytorch-vae_amd")]
os.environ.setdefault("VAE_HIP_LIB", "probe")

import numpy as np  # noqa: E402
import torch  # noqa: E402

WALL_HZ = 100e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--out", default="gpurun_out/kprobe.json")
    args = ap.parse_args()
    from vae_amd import _lib as L
    from vae_amd.engine import FusedAdam, TrainStep
    from vae_amd.net import StepPlan, VAENet, call_one
    lib = L.load()
    assert "probe" in lib._name, "load the probe build (VAE_HIP_LIB=probe)"
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    net = VAENet(latent_dim=128, dtype=dtype, device="cuda", generator=torch.Generator().manual_seed(0))
    plan = StepPlan(net, args.batch)
    opt = FusedAdam(net, lr=0.005)
    g = torch.Generator(device="cuda").manual_seed(1)
    plan.x.copy_(torch.rand(plan.x.shape, generator=g, device="cuda"))
    plan.eps.copy_(torch.randn(plan.eps.shape, generator=g, device="cuda"))
    cap = 1 << 16
    buf = torch.zeros(8 + 8 * cap, dtype=torch.int64, device="cuda")
    buf[1] = cap
    lib.vae_probe_set.argtypes = [ctypes.c_void_p]
    lib.vae_probe_set.restype = None
    lib.vae_probe_set(ctypes.c_void_p(buf.data_ptr()))
    step = TrainStep(net, plan, opt, graph=False)
    step()
    step()
    torch.cuda.synchronize()
    sp = L.stream_ptr()
    calls = plan.fwd_calls + plan.bwd_calls
    rows = []
    for i, (fn, ref) in enumerate(calls):
        for rep in range(3):
            buf[8:].zero_()
            torch.cuda.synchronize()
            call_one(fn, ref, sp)
            torch.cuda.synchronize()
        r = buf[8:].view(cap, 8).cpu().numpy().astype(np.int64)
        r = r[r[:, 1] != 0]                      # slots written by a block (wall start != 0)
        n = len(r)
        if n == 0:
            rows.append({"launch": i, "fn": fn, "blocks": 0})
            continue
        w0, w3 = r[:, 1], r[:, 2]
        c = r[:, 3:7].astype(np.float64)
        span_us = (w3.max() - w0.min()) / WALL_HZ * 1e6
        dur_cyc = c[:, 3] - c[:, 0]
        dur_us = (w3 - w0) / WALL_HZ * 1e6
        hz = float(np.median(dur_cyc / np.maximum(dur_us, 1e-3))) * 1e6   # clk ticks per second
        ph = (c[:, 1:] - c[:, :-1]) / hz * 1e6
        start_skew = (w0.max() - w0.min()) / WALL_HZ * 1e6
        row = {"launch": i, "fn": fn, "blocks": n, "span_us": round(span_us, 2), "start_skew_us": round(start_skew, 2),
               "block_us_med": round(float(np.median(dur_us)), 2), "block_us_max": round(float(dur_us.max()), 2),
               "prologue_med": round(float(np.median(ph[:, 0])), 2), "loop_med": round(float(np.median(ph[:, 1])), 2),
               "epilogue_med": round(float(np.median(ph[:, 2])), 2), "epilogue_max": round(float(ph[:, 2].max()), 2),
               "clk_mhz": round(hz / 1e6, 1)}
        rows.append(row)
        print(json.dumps(row))
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(rows, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
