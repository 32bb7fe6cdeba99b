"""Multi-step VQ-VAE trajectory of the CPU oracle (test infrastructure, run as a script).

Question it answers (round-1 VERDICT item 6): is the bench's VQ_Loss ~1e11 after 23 steps a
property of the workload — Adam at lr 0.005 (configs/vae/vq_vae.yaml) on ONE fixed synthetic
U[0,1) batch of 128 images, repeated every step as bench.py does — or a defect of the HIP
multi-step path?  The oracle (fp32 CPU, the reference's formulas, models/vq_vae.py:24-211,
Adam experiment.py:308-311) runs the same loop and prints the loss terms per step as JSON lines.

    python tests/vq_trajectory.py [--batch 128] [--steps 23] [--lr 0.005] [--seed 1265]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import vae_oracle as O  # noqa: E402


def trajectory(batch, steps, lr, seed, beta=0.25):
    sd = O.make_params(O.vq_param_spec(), seed)
    P = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    opt = torch.optim.Adam(list(P.values()), lr=lr)
    x = torch.rand(batch, 3, 64, 64, generator=torch.Generator().manual_seed(seed + 1))
    out = []
    for k in range(steps):
        enc = O.vq_encode(P, x, O.VQ_HIDDEN)
        q, vq_loss, _, _ = O.vq_quantize(enc, P["vq_layer.embedding.weight"], beta)
        rec = O.vq_decode(P, q, O.VQ_HIDDEN)
        recons = F.mse_loss(rec, x)
        loss = recons + vq_loss
        opt.zero_grad()
        loss.backward()
        opt.step()
        row = {"step": k + 1, "loss": float(loss), "Reconstruction_Loss": float(recons), "VQ_Loss": float(vq_loss),
               "latent_absmax": float(enc.detach().abs().max())}
        out.append(row)
        print(json.dumps(row), flush=True)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=23)
    ap.add_argument("--lr", type=float, default=0.005)
    ap.add_argument("--seed", type=int, default=1265)
    a = ap.parse_args()
    trajectory(a.batch, a.steps, a.lr, a.seed)
