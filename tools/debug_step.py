"""Diagnostic: run one fused step call-by-call with a sync after each launch."""
import os
import sys
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pytorch-vae_amd"), os.path.join(REPO, "tests")]
from golden_util import case_inputs, load_case  # noqa: E402
from vae_amd import _lib as L  # noqa: E402
from vae_amd.net import StepPlan, VAENet, call_one  # noqa: E402

meta, ref = load_case(sys.argv[1] if len(sys.argv) > 1 else "vanilla_b16")
sd, x, eps = case_inputs(meta)
net = VAENet(latent_dim=128, dtype=torch.float32, device="cuda")
net.load_reference_state_dict(sd)
plan = StepPlan(net, meta["batch"], kld_weight=meta["M_N"])
plan.x.copy_(x); plan.eps.copy_(eps)
torch.cuda.synchronize()
st = L.stream_ptr()
step = torch.zeros(1, dtype=torch.int32, device="cuda")
L.call("vae_step_begin", plan.zero.data_ptr(), plan.zero.numel() * 4, step.data_ptr(), st)
torch.cuda.synchronize(); print("step_begin ok", flush=True)
for i, (fn, arg) in enumerate(plan.fwd_calls + plan.bwd_calls):
    print(f"[{i}] {fn} ...", flush=True)
    call_one(fn, arg, st)
    torch.cuda.synchronize()
print("all ok", plan.out.tolist())
