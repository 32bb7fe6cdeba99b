#!/usr/bin/env python3
"""Per-workgroup timing of the batched weight-gradient call of the VanillaVAE step (diagnostic).

    make -C pytorch-vae_amd/csrc probe && VAE_HIP_LIB=probe python3 tools/wgprobe.py

The probe build's grouped weight-gradient kernels write one record per workgroup (layer within the
launch, local block, wall start / end, launch tag, HW_ID).  Prints per launch and layer: workgroups,
median / max duration and the last end relative to the launch's first start.
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
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--out", default="gpurun_out/wgprobe.json")
    args = ap.parse_args()
    from vae_amd import _lib as L
    from vae_amd.engine import FusedAdam, TrainStep
    from vae_amd.net import StepPlan, VAENet, call_one
    lib = L.load()
    assert "probe" in lib._name, "load the probe build (VAE_HIP_LIB=probe)"
    net = VAENet(latent_dim=128, dtype=torch.bfloat16, device="cuda", generator=torch.Generator().manual_seed(0))
    plan = StepPlan(net, args.batch)
    opt = FusedAdam(net, lr=0.005)
    g = torch.Generator(device="cuda").manual_seed(1)
    plan.x.copy_(torch.rand(plan.x.shape, generator=g, device="cuda"))
    plan.eps.copy_(torch.randn(plan.eps.shape, generator=g, device="cuda"))
    cap = 4 * 8192
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
    idx = [i for i, (fn, _) in enumerate(plan.bwd_calls) if fn == "vae_conv_bwd_filter_batch"]
    items = [(fn, ref._obj) for fn, ref in plan.bwd_calls_raw if fn in ("vae_conv2d_bwd_filter", "vae_convT2d_bwd_filter")]
    for k, (fn, a) in enumerate(items):
        print(f"item {k}: {fn} n={a.n} {a.h}x{a.w}x{a.c} -> {a.p}x{a.q}x{a.k}")
    out = []
    for i in idx:
        fn, ref = plan.bwd_calls[i]
        for rep in range(4):
            buf[8:].zero_()
            torch.cuda.synchronize()
            call_one(fn, ref, sp)
            torch.cuda.synchronize()
        r = buf[8:].view(cap, 8).cpu().numpy().astype(np.int64)
        r = r[r[:, 1] != 0]
        t0 = r[:, 1].min()
        print(f"call {i}: {len(r)} workgroups, span {(r[:, 2].max() - t0) / WALL_HZ * 1e6:.2f} us")
        for x in sorted(set(r[:, 3].tolist())):
            rx = r[r[:, 3] == x]
            print(f"  xcd {x}: {len(rx)} wgs, last end {(rx[:, 2].max() - t0) / WALL_HZ * 1e6:.2f} us, "
                  f"layers {sorted(set((rx[:, 0] >> 32).tolist()))}")
        for layer in sorted(set((r[:, 0] >> 32).tolist())):
            rl = r[(r[:, 0] >> 32) == layer]
            dur = (rl[:, 2] - rl[:, 1]) / WALL_HZ * 1e6
            st = (rl[:, 1] - t0) / WALL_HZ * 1e6
            en = (rl[:, 2] - t0) / WALL_HZ * 1e6
            cyc = rl[:, 6].astype(np.float64)
            hz = float(np.median(cyc / np.maximum(dur, 1e-3)))          # cycles per us
            pro = rl[:, 4] / hz
            loop = (rl[:, 5] - rl[:, 4]) / hz
            epi = (rl[:, 6] - rl[:, 5]) / hz
            row = {"layer": int(layer), "wgs": len(rl), "dur_med": round(float(np.median(dur)), 2),
                   "pro_med": round(float(np.median(pro)), 2), "loop_med": round(float(np.median(loop)), 2),
                   "epi_med": round(float(np.median(epi)), 2), "dur_max": round(float(dur.max()), 2),
                   "start_max": round(float(st.max()), 2), "end_med": round(float(np.median(en)), 2),
                   "end_max": round(float(en.max()), 2)}
            print(json.dumps(row))
            out.append(row)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
