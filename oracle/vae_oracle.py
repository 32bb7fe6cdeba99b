"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

This module is the checker for the MI355X VAE training step.  It is imported only by
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``;
the product package (``pytorch-vae_amd/vae_amd``) never imports, links or executes it.

What it is: a functional, fp32, NCHW restatement on PyTorch-CPU (ATen) of the reference
hot path of bplaut/PyTorch-VAE — the same ATen ops the reference's ``nn.Module``s call,
written as plain functions over a reference-layout state dict so that

  * eps (``torch.randn_like`` in the reference) is injectable,
  * BatchNorm running statistics are returned instead of mutated in a module,
  * one teacher-forced training step (forward, loss dict, backward, Adam) is one call.

Pinning: ``tests/test_oracle_golden.py`` checks every function here against golden
vectors produced by running the reference's own modules (``tests/golden/make_golden.py``,
run in the survey container where ``/root/reference`` is importable).

Reference citations (paths relative to the reference root):
  VanillaVAE  models/vanilla_vae.py:11-146      BetaVAE  models/beta_vae.py:12-152
  IWAE        models/iwae.py:10-160             VQVAE    models/vq_vae.py:7-211
  step caller experiment.py:45-86               Adam     experiment.py:308-311
"""
from __future__ import annotations

import hashlib
import math
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

DEFAULT_HIDDEN = [32, 64, 128, 256, 512]          # models/vanilla_vae.py:22
VQ_HIDDEN = [128, 256]                           # models/vq_vae.py:92
BN_EPS = 1e-5                                    # nn.BatchNorm2d default
BN_MOMENTUM = 0.1                                # nn.BatchNorm2d default
LRELU_SLOPE = 0.01                               # nn.LeakyReLU default

# --------------------------------------------------------------------------------------
# Parameter specs (reference state_dict names / shapes) and the seeded recipe
# --------------------------------------------------------------------------------------


def vanilla_param_spec(in_channels: int = 3, latent_dim: int = 128,
                       hidden_dims: Optional[List[int]] = None) -> List[Tuple[str, tuple, str]]:
    """(name, shape, kind) in reference state_dict order — models/vanilla_vae.py:20-75.

    kind ∈ {conv_w, convT_w, lin_w, bias, bn_w, bn_b, bn_rm, bn_rv, bn_nbt}; a bias carries
    the fan-in of its layer via the preceding weight."""
    h = list(hidden_dims or DEFAULT_HIDDEN)
    spec = []
    cin = in_channels
    for i, hd in enumerate(h):                                   # :25-35
        spec += [(f"encoder.{i}.0.weight", (hd, cin, 3, 3), "conv_w"),
                 (f"encoder.{i}.0.bias", (hd,), "bias")]
        spec += _bn_spec(f"encoder.{i}.1", hd)
        cin = hd
    spec += [("fc_mu.weight", (latent_dim, h[-1] * 4), "lin_w"), ("fc_mu.bias", (latent_dim,), "bias"),
             ("fc_var.weight", (latent_dim, h[-1] * 4), "lin_w"), ("fc_var.bias", (latent_dim,), "bias"),
             ("decoder_input.weight", (h[-1] * 4, latent_dim), "lin_w"),
             ("decoder_input.bias", (h[-1] * 4,), "bias")]           # :36-43
    r = h[::-1]
    for i in range(len(r) - 1):                                  # :47-58
        spec += [(f"decoder.{i}.0.weight", (r[i], r[i + 1], 3, 3), "convT_w"),
                 (f"decoder.{i}.0.bias", (r[i + 1],), "bias")]
        spec += _bn_spec(f"decoder.{i}.1", r[i + 1])
    spec += [("final_layer.0.weight", (r[-1], r[-1], 3, 3), "convT_w"),
             ("final_layer.0.bias", (r[-1],), "bias")]           # :64-75
    spec += _bn_spec("final_layer.1", r[-1])
    spec += [("final_layer.3.weight", (3, r[-1], 3, 3), "conv_w"), ("final_layer.3.bias", (3,), "bias")]
    return spec


def ae_param_spec(in_channels: int = 3, latent_dim: int = 128,
                  hidden_dims: Optional[List[int]] = None) -> List[Tuple[str, tuple, str]]:
    """models/autoencoder.py:16-93 in state_dict order: the VanillaVAE stack with one `fc`
    (Linear 4C -> D, :50) in place of fc_mu / fc_var (five stride-2 layers, the configs' case)."""
    spec = []
    for name, shape, kind in vanilla_param_spec(in_channels, latent_dim, hidden_dims):
        if name == "fc_mu.weight":
            spec.append(("fc.weight", shape, kind))
        elif name == "fc_mu.bias":
            spec.append(("fc.bias", shape, kind))
        elif not name.startswith("fc_var."):
            spec.append((name, shape, kind))
    return spec


def _bn_spec(pre: str, c: int):
    return [(f"{pre}.weight", (c,), "bn_w"), (f"{pre}.bias", (c,), "bn_b"),
            (f"{pre}.running_mean", (c,), "bn_rm"), (f"{pre}.running_var", (c,), "bn_rv"),
            (f"{pre}.num_batches_tracked", (), "bn_nbt")]


def vq_param_spec(in_channels: int = 3, embedding_dim: int = 64, num_embeddings: int = 512,
                  hidden_dims: Optional[List[int]] = None) -> List[Tuple[str, tuple, str]]:
    """models/vq_vae.py:90-166 in state_dict order."""
    h = list(hidden_dims or VQ_HIDDEN)
    spec = []
    cin = in_channels
    idx = 0
    for hd in h:                                                   # :95-102
        spec += [(f"encoder.{idx}.0.weight", (hd, cin, 4, 4), "conv_w"), (f"encoder.{idx}.0.bias", (hd,), "bias")]
        cin = hd
        idx += 1
    spec += [(f"encoder.{idx}.0.weight", (cin, cin, 3, 3), "conv_w"), (f"encoder.{idx}.0.bias", (cin,), "bias")]
    idx += 1
    for _ in range(6):                                              # :111-112
        spec += [(f"encoder.{idx}.resblock.0.weight", (cin, cin, 3, 3), "conv_w"),
                 (f"encoder.{idx}.resblock.2.weight", (cin, cin, 1, 1), "conv_w")]
        idx += 1
    idx += 1                                                        # :113 LeakyReLU (no params)
    spec += [(f"encoder.{idx}.0.weight", (embedding_dim, cin, 1, 1), "conv_w"),
             (f"encoder.{idx}.0.bias", (embedding_dim,), "bias")]
    spec += [("vq_layer.embedding.weight", (num_embeddings, embedding_dim), "codebook")]
    spec += [("decoder.0.0.weight", (h[-1], embedding_dim, 3, 3), "conv_w"), ("decoder.0.0.bias", (h[-1],), "bias")]
    idx = 1
    for _ in range(6):
        spec += [(f"decoder.{idx}.resblock.0.weight", (h[-1], h[-1], 3, 3), "conv_w"),
                 (f"decoder.{idx}.resblock.2.weight", (h[-1], h[-1], 1, 1), "conv_w")]
        idx += 1
    idx += 1                                                        # LeakyReLU
    r = h[::-1]
    for i in range(len(r) - 1):
        spec += [(f"decoder.{idx}.0.weight", (r[i], r[i + 1], 4, 4), "convT_w"),
                 (f"decoder.{idx}.0.bias", (r[i + 1],), "bias")]
        idx += 1
    spec += [(f"decoder.{idx}.0.weight", (r[-1], 3, 4, 4), "convT_w"), (f"decoder.{idx}.0.bias", (3,), "bias")]
    return spec


def make_params(spec, seed: int = 1265) -> "OrderedDict[str, torch.Tensor]":
    """Seeded parameter recipe, reproducible on any box with torch (no reference needed).

    Weights/biases ~ U(±1/sqrt(fan_in)) (the scale of PyTorch's default init, fan_in taken
    from dim 1 like torch does — for ConvTranspose2d that is C_out·k·k); BN affine params are
    perturbed away from (1, 0) and running stats away from (0, 1) so every term of the BN
    forward/backward and running-stat update is exercised."""
    g = torch.Generator().manual_seed(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    fan_in = 1
    for name, shape, kind in spec:
        if kind in ("conv_w", "convT_w", "lin_w"):
            fan_in = shape[1] * (shape[2] * shape[3] if len(shape) == 4 else 1)
            b = 1.0 / math.sqrt(fan_in)
            t = (torch.rand(shape, generator=g) * 2 - 1) * b
        elif kind == "bias":
            b = 1.0 / math.sqrt(fan_in)
            t = (torch.rand(shape, generator=g) * 2 - 1) * b
        elif kind == "bn_w":
            t = 0.8 + 0.4 * torch.rand(shape, generator=g)
        elif kind == "bn_b":
            t = (torch.rand(shape, generator=g) * 2 - 1) * 0.1
        elif kind == "bn_rm":
            t = (torch.rand(shape, generator=g) * 2 - 1) * 0.1
        elif kind == "bn_rv":
            t = 0.9 + 0.2 * torch.rand(shape, generator=g)
        elif kind == "bn_nbt":
            t = torch.tensor(0, dtype=torch.long)
        elif kind == "codebook":
            k = shape[0]
            t = (torch.rand(shape, generator=g) * 2 - 1) / k          # models/vq_vae.py:22
        else:
            raise ValueError(kind)
        sd[name] = t.contiguous()
    return sd


def make_inputs(batch: int, latent_dim: int = 128, seed: int = 1265, samples: Optional[int] = None,
                img: int = 64, channels: int = 3) -> Tuple[torch.Tensor, torch.Tensor]:
    """x ~ U[0,1) (ToTensor range, dataset.py:78-79) and eps ~ N(0,1), one generator."""
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(batch, channels, img, img, generator=g)
    eps_shape = (batch, latent_dim) if samples is None else (batch, samples, latent_dim)
    eps = torch.randn(eps_shape, generator=g)
    return x, eps


def sha256_of(tensors) -> str:
    h = hashlib.sha256()
    for t in tensors:
        h.update(t.detach().contiguous().cpu().numpy().tobytes())
    return h.hexdigest()


# --------------------------------------------------------------------------------------
# Functional forward pieces
# --------------------------------------------------------------------------------------


def _bn_act(x, P, pre, training, stats_out, act=True):
    """BatchNorm2d(train) + LeakyReLU — vanilla_vae.py:30-31 (and :56-57, :71-72)."""
    rm = P[pre + ".running_mean"].detach().clone()
    rv = P[pre + ".running_var"].detach().clone()
    y = F.batch_norm(x, rm, rv, P[pre + ".weight"], P[pre + ".bias"], training, BN_MOMENTUM, BN_EPS)
    stats_out[pre + ".running_mean"] = rm
    stats_out[pre + ".running_var"] = rv
    return F.leaky_relu(y, LRELU_SLOPE) if act else y


def vanilla_encode(P, x, hidden_dims, training, stats):
    """models/vanilla_vae.py:77-92."""
    h = x
    for i in range(len(hidden_dims)):
        h = F.conv2d(h, P[f"encoder.{i}.0.weight"], P[f"encoder.{i}.0.bias"], stride=2, padding=1)
        h = _bn_act(h, P, f"encoder.{i}.1", training, stats)
    h = torch.flatten(h, start_dim=1)
    mu = F.linear(h, P["fc_mu.weight"], P["fc_mu.bias"])
    log_var = F.linear(h, P["fc_var.weight"], P["fc_var.bias"])
    return mu, log_var


def vanilla_decode(P, z, hidden_dims, training, stats):
    """models/vanilla_vae.py:94-105 (view uses hidden_dims[-1]; the reference hard-codes 512)."""
    r = hidden_dims[::-1]
    h = F.linear(z, P["decoder_input.weight"], P["decoder_input.bias"]).view(-1, r[0], 2, 2)
    for i in range(len(r) - 1):
        h = F.conv_transpose2d(h, P[f"decoder.{i}.0.weight"], P[f"decoder.{i}.0.bias"],
                               stride=2, padding=1, output_padding=1)
        h = _bn_act(h, P, f"decoder.{i}.1", training, stats)
    h = F.conv_transpose2d(h, P["final_layer.0.weight"], P["final_layer.0.bias"],
                           stride=2, padding=1, output_padding=1)
    h = _bn_act(h, P, "final_layer.1", training, stats)
    h = F.conv2d(h, P["final_layer.3.weight"], P["final_layer.3.bias"], padding=1)
    return torch.tanh(h)


def ae_encode(P, x, hidden_dims, training, stats):
    """models/autoencoder.py:147-163: encoder, flatten, fc -> z."""
    h = x
    for i in range(len(hidden_dims)):
        h = F.conv2d(h, P[f"encoder.{i}.0.weight"], P[f"encoder.{i}.0.bias"], stride=2, padding=1)
        h = _bn_act(h, P, f"encoder.{i}.1", training, stats)
    return F.linear(torch.flatten(h, start_dim=1), P["fc.weight"], P["fc.bias"])


def center_weight_mask(h, w, sigma):
    """models/autoencoder.py:95-125: Gaussian weights around the image centre, mean 1."""
    yy, xx = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing="ij")
    d2 = (yy - (h - 1) / 2) ** 2 + (xx - (w - 1) / 2) ** 2
    wgt = torch.exp(-d2 / (2 * sigma ** 2))
    return (wgt * (h * w / wgt.sum())).unsqueeze(0).unsqueeze(0)


def mssim_window(window_size: int, channels: int, sigma: float = 1.5):
    """models/mssim_vae.py:205-215: the separable window as the reference builds it — note the
    reference's exponent is +(x - w//2)^2 / (2 sigma^2) (an inverted bell), kept as is."""
    k = torch.tensor([math.exp((i - window_size // 2) ** 2 / (2 * sigma ** 2)) for i in range(window_size)])
    k = (k / k.sum()).unsqueeze(1)
    w2 = k.mm(k.t()).float().unsqueeze(0).unsqueeze(0)
    return w2.expand(channels, 1, window_size, window_size).contiguous()


def mssim_loss(img1, img2, window_size: int = 11, normalize: bool = True):
    """models/mssim_vae.py:217-282: 1 - MS-SSIM over 5 levels (avg-pool 2x2 between levels),
    size_average=True, dynamic range 1, normalised (s+1)/2."""
    C = img1.shape[1]
    win = mssim_window(window_size, C).to(img1)
    pad = window_size // 2
    weights = torch.tensor([0.0448, 0.2856, 0.3001, 0.2363, 0.1333], device=img1.device)
    ms, mc = [], []
    for _ in range(weights.numel()):
        mu1 = F.conv2d(img1, win, padding=pad, groups=C)
        mu2 = F.conv2d(img2, win, padding=pad, groups=C)
        mu1_sq, mu2_sq, mu12 = mu1.pow(2), mu2.pow(2), mu1 * mu2
        s1 = F.conv2d(img1 * img1, win, padding=pad, groups=C) - mu1_sq
        s2 = F.conv2d(img2 * img2, win, padding=pad, groups=C) - mu2_sq
        s12 = F.conv2d(img1 * img2, win, padding=pad, groups=C) - mu12
        c1, c2 = 0.01 ** 2, 0.03 ** 2
        v1 = 2.0 * s12 + c2
        v2 = s1 + s2 + c2
        mc.append(torch.mean(v1 / v2))
        ms.append((((2 * mu12 + c1) * v1) / ((mu1_sq + mu2_sq + c1) * v2)).mean())
        img1, img2 = F.avg_pool2d(img1, (2, 2)), F.avg_pool2d(img2, (2, 2))
    ms, mc = torch.stack(ms), torch.stack(mc)
    if normalize:
        ms, mc = (ms + 1) / 2, (mc + 1) / 2
    return 1 - torch.prod((mc ** weights)[:-1] * (ms ** weights)[-1])


def ae_loss(recons, x, center_focus_sigma=None, use_mssim=False):
    """models/autoencoder.py:230-262 (no VGG): MSE, the centre-weighted MSE or the MSSIM loss."""
    if center_focus_sigma is not None:
        m = center_weight_mask(x.shape[2], x.shape[3], center_focus_sigma)
        rl = ((recons - x) ** 2 * m.expand(x.shape[0], x.shape[1], -1, -1)).mean()
    elif use_mssim:
        rl = mssim_loss(recons, x)
    else:
        rl = F.mse_loss(recons, x)
    zero = torch.tensor(0.0)
    return {"loss": rl, "Reconstruction_Loss": rl, "KLD": zero, "feature_loss": zero}


def reparameterize(mu, log_var, eps):
    """models/vanilla_vae.py:107-117 with eps injected."""
    std = torch.exp(0.5 * log_var)
    return eps * std + mu


def vanilla_loss(recons, x, mu, log_var, M_N):
    """models/vanilla_vae.py:124-146 — note 'KLD' is returned negated."""
    recons_loss = F.mse_loss(recons, x)
    kld_loss = torch.mean(-0.5 * torch.sum(1 + log_var - mu ** 2 - log_var.exp(), dim=1), dim=0)
    loss = recons_loss + M_N * kld_loss
    return {"loss": loss, "Reconstruction_Loss": recons_loss.detach(), "KLD": -kld_loss.detach()}


def beta_loss(recons, x, mu, log_var, M_N, beta=4.0, gamma=1000.0, loss_type="B",
              C_max=25.0, C_stop_iter=1e5, num_iter=1):
    """models/beta_vae.py:129-152; num_iter is the value *after* the reference's += 1."""
    recons_loss = F.mse_loss(recons, x)
    kld_loss = torch.mean(-0.5 * torch.sum(1 + log_var - mu ** 2 - log_var.exp(), dim=1), dim=0)
    if loss_type == "H":
        loss = recons_loss + beta * M_N * kld_loss
    elif loss_type == "B":
        c_max = torch.tensor([float(C_max)], dtype=torch.float32)     # beta_vae.py:28, fp32
        C = torch.clamp(c_max / C_stop_iter * num_iter, 0, float(c_max[0]))
        loss = (recons_loss + gamma * M_N * (kld_loss - C).abs()).reshape(())
    else:
        raise ValueError("Undefined loss type.")
    return {"loss": loss, "Reconstruction_Loss": recons_loss, "KLD": kld_loss}


def iwae_forward(P, x, eps, hidden_dims, training, stats):
    """models/iwae.py:121-127 with the intended row-major [B·S, D] decode (iwae.py:103
    raises on torch>=1.5 because z inherits permuted strides)."""
    mu, log_var = vanilla_encode(P, x, hidden_dims, training, stats)
    B, S, D = eps.shape
    mu_s = mu.unsqueeze(1).expand(B, S, D)
    lv_s = log_var.unsqueeze(1).expand(B, S, D)
    z = reparameterize(mu_s, lv_s, eps)
    recon = vanilla_decode(P, z.reshape(B * S, D), hidden_dims, training, stats)
    recon = recon.view(B, S, recon.size(1), recon.size(2), recon.size(3))
    return recon, mu_s, lv_s, z


def iwae_loss(recons, x, mu, log_var, M_N):
    """models/iwae.py:129-160."""
    S = recons.shape[1]
    xr = x.unsqueeze(1).expand(-1, S, -1, -1, -1)
    log_p_x_z = ((recons - xr) ** 2).flatten(2).mean(-1)
    kld_loss = -0.5 * torch.sum(1 + log_var - mu ** 2 - log_var.exp(), dim=2)
    log_weight = log_p_x_z + M_N * kld_loss
    weight = F.softmax(log_weight, dim=-1)
    loss = torch.mean(torch.sum(weight * log_weight, dim=-1), dim=0)
    return {"loss": loss, "Reconstruction_Loss": log_p_x_z.mean(), "KLD": -kld_loss.mean()}, log_weight, weight


def _res(P, pre, h):
    """ResidualLayer — models/vq_vae.py:57-70."""
    t = F.conv2d(h, P[pre + ".resblock.0.weight"], None, padding=1)
    t = F.relu(t)
    t = F.conv2d(t, P[pre + ".resblock.2.weight"], None)
    return h + t


def vq_encode(P, x, hidden_dims):
    """models/vq_vae.py:94-122."""
    h = x
    idx = 0
    for _ in hidden_dims:
        h = F.leaky_relu(F.conv2d(h, P[f"encoder.{idx}.0.weight"], P[f"encoder.{idx}.0.bias"],
                                  stride=2, padding=1), LRELU_SLOPE)
        idx += 1
    h = F.leaky_relu(F.conv2d(h, P[f"encoder.{idx}.0.weight"], P[f"encoder.{idx}.0.bias"], padding=1), LRELU_SLOPE)
    idx += 1
    for _ in range(6):
        h = _res(P, f"encoder.{idx}", h)
        idx += 1
    h = F.leaky_relu(h, LRELU_SLOPE)
    idx += 1
    h = F.leaky_relu(F.conv2d(h, P[f"encoder.{idx}.0.weight"], P[f"encoder.{idx}.0.bias"]), LRELU_SLOPE)
    return h


def vq_quantize(latents, E, beta, force_indices=None):
    """VectorQuantizer.forward — models/vq_vae.py:24-55.  Returns also the int64 indices
    and the per-row distance gap d2-d1 (used to judge index exactness near ties).
    force_indices: teacher forcing — use these codes instead of the argmin (for checking the
    rest of the step when a near-tie row resolved differently under another summation order)."""
    lat = latents.permute(0, 2, 3, 1).contiguous()
    flat = lat.view(-1, E.shape[1])
    dist = torch.sum(flat ** 2, dim=1, keepdim=True) + torch.sum(E ** 2, dim=1) - 2 * torch.matmul(flat, E.t())
    inds = torch.argmin(dist, dim=1) if force_indices is None else force_indices.to(torch.int64).view(-1)
    top2 = torch.topk(dist.detach(), 2, dim=1, largest=False).values
    gap = top2[:, 1] - top2[:, 0]
    q = E[inds].view(lat.shape)              # == one-hot @ E (exact)
    commitment = F.mse_loss(q.detach(), lat)
    embedding = F.mse_loss(q, lat.detach())
    vq_loss = commitment * beta + embedding
    q = lat + (q - lat).detach()
    return q.permute(0, 3, 1, 2).contiguous(), vq_loss, inds, gap


def vq_decode(P, z, hidden_dims):
    """models/vq_vae.py:128-166."""
    h = F.leaky_relu(F.conv2d(z, P["decoder.0.0.weight"], P["decoder.0.0.bias"], padding=1), LRELU_SLOPE)
    idx = 1
    for _ in range(6):
        h = _res(P, f"decoder.{idx}", h)
        idx += 1
    h = F.leaky_relu(h, LRELU_SLOPE)
    idx += 1
    r = hidden_dims[::-1]
    for _ in range(len(r) - 1):
        h = F.leaky_relu(F.conv_transpose2d(h, P[f"decoder.{idx}.0.weight"], P[f"decoder.{idx}.0.bias"],
                                            stride=2, padding=1), LRELU_SLOPE)
        idx += 1
    h = torch.tanh(F.conv_transpose2d(h, P[f"decoder.{idx}.0.weight"], P[f"decoder.{idx}.0.bias"],
                                      stride=2, padding=1))
    return h


# --------------------------------------------------------------------------------------
# Adam (torch.optim.Adam single-tensor semantics, experiment.py:308-311)
# --------------------------------------------------------------------------------------


def adam_step(p, g, m, v, step, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
    """In-place Adam update of p, m, v; `step` is the step count after increment."""
    b1, b2 = betas
    if weight_decay != 0:
        g = g + weight_decay * p
    m.lerp_(g, 1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)


# --------------------------------------------------------------------------------------
# One teacher-forced training step
# --------------------------------------------------------------------------------------

TRAINABLE_KINDS = ("conv_w", "convT_w", "lin_w", "bias", "bn_w", "bn_b", "codebook")


def train_step(arch: str, sd, x, eps=None, *, M_N: float, lr: float = 0.005, hidden_dims=None,
               beta=4.0, gamma=1000.0, loss_type="H", max_capacity=25.0, Capacity_max_iter=1e5,
               num_iter=1, vq_beta=0.25, do_adam=True, training=True, vq_indices=None,
               center_focus_sigma=None, use_mssim_loss=False):
    """forward -> loss_function -> backward -> Adam on a copy of ``sd``.

    Returns a dict: outputs (recon, mu, log_var / vq_loss, indices), loss terms, per-image
    MSE (experiment.py:60-62), grads (reference layout), updated running stats, new params."""
    spec_kinds = _kinds_of(arch, sd, hidden_dims)
    P = OrderedDict()
    for k, t in sd.items():
        t = t.detach().clone()
        if spec_kinds[k] in TRAINABLE_KINDS:
            t.requires_grad_(True)
        P[k] = t
    stats: Dict[str, torch.Tensor] = {}
    out: Dict[str, object] = {}
    if arch in ("VanillaVAE", "BetaVAE"):
        hd = list(hidden_dims or DEFAULT_HIDDEN)
        mu, log_var = vanilla_encode(P, x, hd, training, stats)
        z = reparameterize(mu, log_var, eps)
        recon = vanilla_decode(P, z, hd, training, stats)
        if arch == "VanillaVAE":
            ld = vanilla_loss(recon, x, mu, log_var, M_N)
        else:
            ld = beta_loss(recon, x, mu, log_var, M_N, beta, gamma, loss_type, max_capacity,
                           Capacity_max_iter, num_iter)
        per_img = F.mse_loss(recon.detach(), x, reduction="none").mean(dim=[1, 2, 3])
        out.update(recon=recon.detach(), mu=mu.detach(), log_var=log_var.detach(), z=z.detach())
    elif arch == "IWAE":
        hd = list(hidden_dims or DEFAULT_HIDDEN)
        recon, mu_s, lv_s, z = iwae_forward(P, x, eps, hd, training, stats)
        ld, lw, w = iwae_loss(recon, x, mu_s, lv_s, M_N)
        per_img = ((recon.detach() - x.unsqueeze(1)) ** 2).flatten(2).mean(-1)  # [B,S]
        out.update(recon=recon.detach(), mu=mu_s[:, 0].detach(), log_var=lv_s[:, 0].detach(),
                   log_weight=lw.detach(), weight=w.detach())
    elif arch == "Autoencoder":
        hd = list(hidden_dims or DEFAULT_HIDDEN)
        z = ae_encode(P, x, hd, training, stats)
        recon = vanilla_decode(P, z, hd, training, stats)
        ld = ae_loss(recon, x, center_focus_sigma, use_mssim_loss)
        per_img = F.mse_loss(recon.detach(), x, reduction="none").mean(dim=[1, 2, 3])
        out.update(recon=recon.detach(), z=z.detach())
    elif arch == "VQVAE":
        hd = list(hidden_dims or VQ_HIDDEN)
        enc = vq_encode(P, x, hd)
        q, vq_loss, inds, gap = vq_quantize(enc, P["vq_layer.embedding.weight"], vq_beta, vq_indices)
        recon = vq_decode(P, q, hd)
        recons_loss = F.mse_loss(recon, x)
        ld = {"loss": recons_loss + vq_loss, "Reconstruction_Loss": recons_loss, "VQ_Loss": vq_loss}
        per_img = F.mse_loss(recon.detach(), x, reduction="none").mean(dim=[1, 2, 3])
        out.update(recon=recon.detach(), latents=enc.detach(), indices=inds, gap=gap)
    else:
        raise ValueError(arch)
    ld["loss"].backward()
    grads = OrderedDict((k, (P[k].grad.detach().clone() if P[k].grad is not None else torch.zeros_like(P[k])))
                        for k in P if spec_kinds[k] in TRAINABLE_KINDS)
    new_params = OrderedDict()
    if do_adam:
        for k, g in grads.items():
            p = P[k].detach().clone()
            adam_step(p, g, torch.zeros_like(p), torch.zeros_like(p), 1, lr)
            new_params[k] = p
    out.update(loss={k: float(v.detach()) for k, v in ld.items()}, per_img_mse=per_img, grads=grads,
               running=stats, new_params=new_params)
    return out


def _kinds_of(arch, sd, hidden_dims):
    if arch == "VQVAE":
        spec = vq_param_spec(hidden_dims=hidden_dims, embedding_dim=sd["vq_layer.embedding.weight"].shape[1],
                             num_embeddings=sd["vq_layer.embedding.weight"].shape[0])
    elif arch == "Autoencoder":
        spec = ae_param_spec(latent_dim=sd["fc.weight"].shape[0], hidden_dims=hidden_dims)
    else:
        spec = vanilla_param_spec(latent_dim=sd["fc_mu.weight"].shape[0], hidden_dims=hidden_dims)
    kinds = {n: k for n, _, k in spec}
    missing = set(sd) ^ set(kinds)
    if missing:
        raise KeyError(f"state dict does not match spec: {sorted(missing)[:5]}")
    return kinds
