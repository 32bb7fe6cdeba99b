"""Load the golden vectors in tests/golden/*.npz (written by tests/golden/make_golden.py)."""
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["vanilla_b16", "vanilla_b8_kl", "betaH_b16", "betaB_b8", "iwae_b4", "vq_b4", "ae_b16", "ae_center_b8",
         "ae_mssim_b8", "ae_big_b4"]


def load_case(name):
    z = np.load(os.path.join(GOLDEN_DIR, f"{name}.npz"), allow_pickle=False)
    arrays = {k: z[k] for k in z.files if k != "meta"}
    meta = json.loads(bytes(z["meta"]).decode())
    return meta, arrays


def summary(t):
    t = t.detach().double().flatten().cpu()
    return np.array([t.sum().item(), t.norm().item(), t.abs().max().item() if t.numel() else 0.0])


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def case_inputs(meta):
    """Rebuild params and inputs from the recipe and check them against the fixture's SHA."""
    from oracle import vae_oracle as O
    kw = meta["ctor"]
    if meta["arch"] == "VQVAE":
        spec = O.vq_param_spec(embedding_dim=kw["embedding_dim"], num_embeddings=kw["num_embeddings"])
    elif meta["arch"] == "Autoencoder":
        spec = O.ae_param_spec(latent_dim=kw["latent_dim"], hidden_dims=kw.get("hidden_dims"))
    else:
        spec = O.vanilla_param_spec(latent_dim=kw["latent_dim"])
    sd = O.make_params(spec, meta["seed"])
    x, eps = O.make_inputs(meta["batch"], kw.get("latent_dim", 64), meta["seed"], samples=meta["samples"])
    assert O.sha256_of([x]) == meta["x_sha"], "input recipe drifted"
    assert O.sha256_of([eps]) == meta["eps_sha"], "eps recipe drifted"
    assert O.sha256_of([sd[k] for k in sd]) == meta["params_sha"], "param recipe drifted"
    return sd, x, eps


def oracle_kwargs(meta):
    kw = meta["ctor"]
    d = dict(M_N=meta["M_N"], lr=meta["lr"])
    if meta["arch"] == "BetaVAE":
        d.update(beta=kw.get("beta", 4), gamma=kw.get("gamma", 1000.0), loss_type=kw.get("loss_type", "B"),
                 max_capacity=kw.get("max_capacity", 25), Capacity_max_iter=kw.get("Capacity_max_iter", 1e5),
                 num_iter=1)
    if meta["arch"] == "VQVAE":
        d.update(vq_beta=kw.get("beta", 0.25))
    if meta["arch"] == "Autoencoder":
        d.update(center_focus_sigma=kw.get("center_focus_sigma"), use_mssim_loss=kw.get("use_mssim_loss", False),
                 hidden_dims=kw.get("hidden_dims"))
    return d
