#!/usr/bin/env python3
"""Per-launch kernel microbenchmark of the fused step (diagnostic, run under rocprofv3).

    rocprofv3 --kernel-trace --output-format csv -d OUT -o kb -- python3 tools/kbench.py [--dtype bf16]

Builds the bench plan (VanillaVAE, B=64), runs one real step so every buffer holds live data,
then replays each launch of the step REPS times (optionally with forced split-K values),
separated by marker kernels so the trace can be cut into (launch, variant) groups.  Prints the
index of every group; tools/kbench_report.py joins it with the kernel trace.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pytorch-vae_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--splits", default="0", help="comma list of split_k values to try (0 = auto)")
    ap.add_argument("--only", default="", help="comma list of launch indices")
    ap.add_argument("--out", default="gpurun_out/kbench_groups.json")
    args = ap.parse_args()
    from vae_amd import _lib as L
    from vae_amd.engine import FusedAdam, TrainStep
    from vae_amd.net import StepPlan, VAENet, call_one
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    net = VAENet(latent_dim=128, dtype=dtype, device="cuda", generator=torch.Generator().manual_seed(0))
    plan = StepPlan(net, args.batch)
    opt = FusedAdam(net, lr=0.005)
    g = torch.Generator(device="cuda").manual_seed(1)
    plan.x.copy_(torch.rand(plan.x.shape, generator=g, device="cuda"))
    plan.eps.copy_(torch.randn(plan.eps.shape, generator=g, device="cuda"))
    step = TrainStep(net, plan, opt, graph=False)
    step()
    torch.cuda.synchronize()
    sp = L.stream_ptr()
    calls = plan.fwd_calls + plan.bwd_calls
    only = [int(i) for i in args.only.split(",") if i] or list(range(len(calls)))
    splits = [int(s) for s in args.splits.split(",")]
    groups = []
    for i in only:
        fn, ref = calls[i]
        for s in splits:
            obj = getattr(ref, "_obj", None)
            if obj is not None and hasattr(obj, "split_k"):
                obj.split_k = s
            elif s != 0:
                continue
            torch.cuda._sleep(1000)                      # marker kernel (spin_kernel)
            for _ in range(args.reps):
                call_one(fn, ref, sp)
            groups.append({"launch": i, "fn": fn, "split": s})
            if obj is not None and hasattr(obj, "split_k"):
                obj.split_k = 0
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump({"reps": args.reps, "groups": groups}, open(args.out, "w"))
    print(f"{len(groups)} groups")


if __name__ == "__main__":
    main()
