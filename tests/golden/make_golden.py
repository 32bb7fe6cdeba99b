"""Generate golden vectors by running the REFERENCE's own modules (survey container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [/root/reference]

Recipe (no reference code is copied; it is imported read-only):
  * torchvision is absent here; two in-memory stub modules expose a ``vgg19_bn`` that is
    never called (it is only imported by models/autoencoder.py:5 and models/dfcvae.py:4).
  * parameters come from ``oracle.vae_oracle.make_params`` (seeded, reproducible without
    the reference) and are loaded with ``load_state_dict`` into the reference model;
  * inputs come from ``oracle.vae_oracle.make_inputs``; eps is injected by swapping
    ``torch.randn_like`` for the duration of ``forward`` (models/vanilla_vae.py:116);
  * IWAE: models/iwae.py:103 raises on torch>=1.5 (``view`` of a permuted z), so the
    harness wraps ``decode`` with ``z.contiguous()`` — the reference file is untouched;
  * one step = forward, loss_function(M_N=...), backward, torch.optim.Adam(lr).step().

Outputs: tests/golden/<case>.npz — data only (inputs' SHA-256, outputs, loss terms,
grad/param summaries, BN running stats).  The reference never travels to the GPU box;
these fixtures do.
"""
from __future__ import annotations

import copy
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import vae_oracle as O  # noqa: E402

CASES = {
    # name: (arch, batch, ctor kwargs, M_N, lr, extra)
    "vanilla_b16": ("VanillaVAE", 16, dict(in_channels=3, latent_dim=128), 1e-8, 0.005, {}),
    "vanilla_b8_kl": ("VanillaVAE", 8, dict(in_channels=3, latent_dim=128), 0.5, 0.005, {}),
    "betaH_b16": ("BetaVAE", 16, dict(in_channels=3, latent_dim=128, loss_type="H", beta=4), 2.5e-4, 0.005, {}),
    "betaB_b8": ("BetaVAE", 8, dict(in_channels=3, latent_dim=128, loss_type="B", gamma=1000.0,
                                     max_capacity=25, Capacity_max_iter=1e5), 2.5e-4, 0.005, {}),
    "iwae_b4": ("IWAE", 4, dict(in_channels=3, latent_dim=128, num_samples=5), 2.5e-4, 0.007, {"S": 5}),
    "ae_b16": ("Autoencoder", 16, dict(in_channels=3, latent_dim=128), 0.0, 0.005, {}),
    "ae_center_b8": ("Autoencoder", 8, dict(in_channels=3, latent_dim=128, center_focus_sigma=11), 0.0, 0.0005, {}),
    "ae_mssim_b8": ("Autoencoder", 8, dict(in_channels=3, latent_dim=128, use_mssim_loss=True), 0.0, 0.005, {}),
    "ae_big_b4": ("Autoencoder", 4, dict(in_channels=3, latent_dim=128, hidden_dims=[128, 256, 512, 1024, 2048]),
                  0.0, 0.005, {}),
    "vq_b4": ("VQVAE", 4, dict(in_channels=3, embedding_dim=64, num_embeddings=512, img_size=64, beta=0.25),
              0.0, 0.005, {}),
}
SEED = 1265
HEAD = 64


def import_reference(ref_root):
    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")

    def vgg19_bn(*a, **k):
        raise RuntimeError("vgg19_bn is not available offline (not on the hot path)")

    tvm.vgg19_bn = vgg19_bn
    tv.models = tvm
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.models", tvm)
    sys.path.insert(0, ref_root)
    import models  # noqa: F401  (the reference package)
    return models


def summary(t):
    t = t.detach().double().flatten()
    return np.array([t.sum().item(), t.norm().item(), t.abs().max().item() if t.numel() else 0.0])


def run_case(models, name):
    arch, B, kw, M_N, lr, extra = CASES[name]
    torch.manual_seed(0)
    model = models.vae_models[arch](**copy.deepcopy(kw))     # (the reference reverses hidden_dims in place)
    spec = (O.vq_param_spec(embedding_dim=kw["embedding_dim"], num_embeddings=kw["num_embeddings"])
            if arch == "VQVAE" else O.ae_param_spec(latent_dim=kw["latent_dim"], hidden_dims=kw.get("hidden_dims"))
            if arch == "Autoencoder"
            else O.vanilla_param_spec(latent_dim=kw["latent_dim"]))
    sd = O.make_params(spec, SEED)
    model.load_state_dict(sd, strict=True)
    model.train()
    x, eps = O.make_inputs(B, kw.get("latent_dim", 64), SEED, samples=extra.get("S"))

    if arch == "IWAE":
        orig_decode = model.decode
        model.decode = lambda z: orig_decode(z.contiguous())
    real_randn_like = torch.randn_like

    def fake_randn_like(t, *a, **k):
        assert tuple(t.shape) == tuple(eps.shape), (t.shape, eps.shape)
        return eps.clone()

    captured = {}
    hook = (model.fc.register_forward_hook(lambda m, i, o: captured.__setitem__("z", o.detach().clone()))
            if arch == "Autoencoder" else None)
    torch.randn_like = fake_randn_like
    try:
        results = model(x, labels=torch.zeros(B))
    finally:
        torch.randn_like = real_randn_like
        if hook is not None:
            hook.remove()
    ld = model.loss_function(*results, M_N=M_N, optimizer_idx=0, batch_idx=0)
    ld["loss"].reshape(()).backward()

    arrays = {}
    meta = {"case": name, "arch": arch, "batch": B, "ctor": kw, "M_N": M_N, "lr": lr, "seed": SEED,
            "samples": extra.get("S"), "x_sha": O.sha256_of([x]), "eps_sha": O.sha256_of([eps]),
            "params_sha": O.sha256_of([sd[k] for k in sd]),
            "loss": {k: float(v.detach().reshape(-1)[0]) for k, v in ld.items()},
            "torch": torch.__version__}
    recon = results[0].detach()
    arrays["recon_head"] = recon[: (1 if arch == "IWAE" else min(B, 4))].numpy()
    flat = recon.reshape(recon.shape[0], -1) if arch != "IWAE" else recon.reshape(B * extra["S"], -1)
    arrays["recon_sum"] = flat.double().sum(1).numpy()
    arrays["recon_sq"] = (flat.double() ** 2).sum(1).numpy()
    if arch == "IWAE":
        xr = x.unsqueeze(1)
        arrays["per_img_mse"] = ((recon - xr) ** 2).flatten(2).mean(-1).numpy()
        mu, lv = results[2][:, 0], results[3][:, 0]
        arrays["mu"], arrays["log_var"] = mu.detach().numpy(), lv.detach().numpy()
        lp = ((recon - xr) ** 2).flatten(2).mean(-1)
        kld = -0.5 * torch.sum(1 + results[3] - results[2] ** 2 - results[3].exp(), dim=2)
        lw = (lp + M_N * kld).detach()
        arrays["log_weight"] = lw.numpy()
        arrays["weight"] = torch.softmax(lw, -1).numpy()
    else:
        arrays["per_img_mse"] = torch.nn.functional.mse_loss(recon, x, reduction="none").mean(dim=[1, 2, 3]).numpy()
    if arch in ("VanillaVAE", "BetaVAE"):
        arrays["mu"], arrays["log_var"] = results[2].detach().numpy(), results[3].detach().numpy()
    if arch == "Autoencoder":
        arrays["z"] = captured["z"].numpy()
    if arch == "VQVAE":
        with torch.no_grad():
            enc = model.encode(x)[0]
            lat = enc.permute(0, 2, 3, 1).contiguous().view(-1, model.embedding_dim)
            E = model.vq_layer.embedding.weight
            dist = torch.sum(lat ** 2, 1, keepdim=True) + torch.sum(E ** 2, 1) - 2 * lat @ E.t()
            arrays["indices"] = torch.argmin(dist, 1).numpy().astype(np.int64)
            top2 = torch.topk(dist, 2, dim=1, largest=False).values
            arrays["gap"] = (top2[:, 1] - top2[:, 0]).numpy()
            arrays["latents_sum"] = summary(enc)

    names = []
    for k, p in model.named_parameters():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        arrays[f"grad_stats/{k}"] = summary(g)
        arrays[f"grad_head/{k}"] = g.detach().flatten()[:HEAD].numpy()
        names.append(k)
    meta["param_names"] = names
    for k, t in model.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            arrays[f"running/{k}"] = t.numpy()
    opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=0.0)
    opt.step()
    for k, p in model.named_parameters():
        arrays[f"new_stats/{k}"] = summary(p)
        arrays[f"new_head/{k}"] = p.detach().flatten()[:HEAD].numpy()
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    out = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(out, **arrays)
    print(f"wrote {out} ({os.path.getsize(out) / 1024:.0f} KiB) loss={meta['loss']}")


def main():
    ref_root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    torch.set_num_threads(8)
    models = import_reference(ref_root)
    only = sys.argv[2:] or list(CASES)
    for name in only:
        run_case(models, name)


if __name__ == "__main__":
    main()
