"""Parameter layout of the VAE family: reference state-dict <-> native flat buffers.

The reference keeps PyTorch layouts (models/vanilla_vae.py:25-75): Conv2d [Co][Ci][R][S],
ConvTranspose2d [Ci][Co][R][S], Linear [Out][In] on an NCHW flatten of the [C,2,2] bottleneck
(torch.flatten at :85, view(-1,512,2,2) at :102).  Natively every tensor is stored for the
kernels that read it (include/vaehip.h):

  Conv2d           [Co][R][S][Ci]      (k-contiguous B operand of the implicit GEMM)
  ConvTranspose2d  [Ci][R][S][Co]
  fc_mu | fc_var   one [2D][4C] matrix, input index hw*C + c (NHWC flatten)
  decoder_input    [4C][D], output row hw*C + c (so its output *is* the NHWC map)

All trainable tensors live in one flat fp32 buffer (the optimizer and the gradient
all-reduce each see one contiguous range); the order is the order in which backward
finishes their gradients (decoder head first), so DDP buckets can be sent while the
encoder backward still runs.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

import torch

ALIGN = 64  # elements: every tensor starts 256-B aligned (fp32) / 128-B (bf16)


@dataclass
class PSpec:
    name: str                     # reference state-dict key
    ref_shape: Tuple[int, ...]
    kind: str                     # conv_w, convT_w, fc_w, fc_b, din_w, din_b, bias, bn_w, bn_b, codebook
    bottleneck_c: int = 0         # C of the [C,2,2] map for fc/decoder_input permutations
    offset: int = 0               # in the flat buffer
    numel: int = 0
    gemm_weight: bool = False     # read by an MFMA GEMM (needs a bf16 copy in bf16 mode)

    @property
    def native_shape(self) -> Tuple[int, ...]:
        s = self.ref_shape
        if self.kind in ("conv_w", "convT_w"):
            return (s[0], s[2], s[3], s[1])
        return s


def to_native(spec: PSpec, t: torch.Tensor) -> torch.Tensor:
    k = spec.kind
    if k in ("conv_w", "convT_w"):
        return t.permute(0, 2, 3, 1).contiguous()
    if k == "fc_w":                                    # [D][C*4] (c*4+hw) -> [D][hw*C+c]
        D, F = t.shape
        C = spec.bottleneck_c
        return t.reshape(D, C, F // C).permute(0, 2, 1).reshape(D, F).contiguous()
    if k == "din_w":                                   # [C*4][D] (row c*4+hw) -> row hw*C+c
        F, D = t.shape
        C = spec.bottleneck_c
        return t.reshape(C, F // C, D).permute(1, 0, 2).reshape(F, D).contiguous()
    if k == "din_b":
        C = spec.bottleneck_c
        return t.reshape(C, -1).t().reshape(-1).contiguous()
    return t.contiguous()


def from_native(spec: PSpec, t: torch.Tensor) -> torch.Tensor:
    k = spec.kind
    if k in ("conv_w", "convT_w"):
        return t.permute(0, 3, 1, 2).contiguous()
    if k == "fc_w":
        D, F = t.shape
        C = spec.bottleneck_c
        return t.reshape(D, F // C, C).permute(0, 2, 1).reshape(D, F).contiguous()
    if k == "din_w":
        F, D = t.shape
        C = spec.bottleneck_c
        return t.reshape(F // C, C, D).permute(1, 0, 2).reshape(F, D).contiguous()
    if k == "din_b":
        C = spec.bottleneck_c
        return t.reshape(-1, C).t().reshape(-1).contiguous()
    return t.contiguous()


@dataclass
class BNSpec:
    prefix: str                   # e.g. "encoder.0.1"
    channels: int
    offset: int = 0               # into the running-stat buffer ([mean | var] per layer)


@dataclass
class Layout:
    params: List[PSpec] = field(default_factory=list)
    bns: List[BNSpec] = field(default_factory=list)
    total: int = 0
    bn_total: int = 0

    def finalize(self):
        off = 0
        for p in self.params:
            p.numel = 1
            for d in p.ref_shape:
                p.numel *= d
            p.offset = off
            off += (p.numel + ALIGN - 1) // ALIGN * ALIGN
        self.total = off
        off = 0
        for b in self.bns:
            b.offset = off
            off += 2 * b.channels
        self.bn_total = off
        self.by_name: Dict[str, PSpec] = {p.name: p for p in self.params}
        self.bn_by_prefix: Dict[str, BNSpec] = {b.prefix: b for b in self.bns}
        return self

    def view(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        p = self.by_name[name]
        return flat[p.offset:p.offset + p.numel].view(p.native_shape)

    def span(self, flat: torch.Tensor, first: str, last: str) -> torch.Tensor:
        """Contiguous range from tensor `first` to the end of tensor `last` (fused views)."""
        a = self.by_name[first]
        b = self.by_name[last]
        return flat[a.offset:b.offset + b.numel]

    def load_reference(self, flat: torch.Tensor, running: torch.Tensor, sd: Dict[str, torch.Tensor]):
        """Copy a reference-layout state dict into the native buffers (keys must match)."""
        with torch.no_grad():
            for p in self.params:
                if p.name not in sd:
                    raise KeyError(f"missing key {p.name}")
                src = sd[p.name]
                if tuple(src.shape) != p.ref_shape:
                    raise ValueError(f"{p.name}: shape {tuple(src.shape)} != {p.ref_shape}")
                flat[p.offset:p.offset + p.numel].copy_(to_native(p, src.float()).reshape(-1))
            for b in self.bns:
                running[b.offset:b.offset + b.channels].copy_(sd[b.prefix + ".running_mean"].float())
                running[b.offset + b.channels:b.offset + 2 * b.channels].copy_(sd[b.prefix + ".running_var"].float())

    def export_reference(self, flat: torch.Tensor, running: Optional[torch.Tensor] = None,
                         num_batches: int = 0, order: Optional[List[str]] = None) -> Dict[str, torch.Tensor]:
        """Reference-layout state dict (in the reference's key order when `order` is given)."""
        out: Dict[str, torch.Tensor] = {}
        for p in self.params:
            out[p.name] = from_native(p, flat[p.offset:p.offset + p.numel].view(p.native_shape))
        if running is not None:
            for b in self.bns:
                out[b.prefix + ".running_mean"] = running[b.offset:b.offset + b.channels].clone()
                out[b.prefix + ".running_var"] = running[b.offset + b.channels:b.offset + 2 * b.channels].clone()
                out[b.prefix + ".num_batches_tracked"] = torch.tensor(num_batches, dtype=torch.long)
        if order is not None:
            out = {k: out[k] for k in order if k in out}
        return out


def vanilla_layout(in_channels: int, latent_dim: int, hidden_dims: List[int]) -> Layout:
    """VanillaVAE / BetaVAE / IWAE (models/vanilla_vae.py:20-75).  Flat order = backward
    completion order: head, final_layer, decoder (last block first), decoder_input, fc,
    encoder (last block first); each BatchNorm's (weight, bias) next to its conv."""
    h = list(hidden_dims)
    r = h[::-1]
    C = h[-1]
    L = Layout()
    L.params += [PSpec("final_layer.3.weight", (3, r[-1], 3, 3), "conv_w"),
                 PSpec("final_layer.3.bias", (3,), "bias")]
    L.params += [PSpec("final_layer.1.weight", (r[-1],), "bn_w"), PSpec("final_layer.1.bias", (r[-1],), "bn_b"),
                 PSpec("final_layer.0.weight", (r[-1], r[-1], 3, 3), "convT_w", gemm_weight=True),
                 PSpec("final_layer.0.bias", (r[-1],), "bias")]
    for i in reversed(range(len(r) - 1)):
        L.params += [PSpec(f"decoder.{i}.1.weight", (r[i + 1],), "bn_w"),
                     PSpec(f"decoder.{i}.1.bias", (r[i + 1],), "bn_b"),
                     PSpec(f"decoder.{i}.0.weight", (r[i], r[i + 1], 3, 3), "convT_w", gemm_weight=True),
                     PSpec(f"decoder.{i}.0.bias", (r[i + 1],), "bias")]
    L.params += [PSpec("decoder_input.weight", (4 * C, latent_dim), "din_w", C, gemm_weight=True),
                 PSpec("decoder_input.bias", (4 * C,), "din_b", C)]
    # fc_mu and fc_var adjacent: one fused [2D][4C] weight and one [2D] bias
    L.params += [PSpec("fc_mu.weight", (latent_dim, 4 * C), "fc_w", C, gemm_weight=True),
                 PSpec("fc_var.weight", (latent_dim, 4 * C), "fc_w", C, gemm_weight=True),
                 PSpec("fc_mu.bias", (latent_dim,), "bias"), PSpec("fc_var.bias", (latent_dim,), "bias")]
    cins = [in_channels] + h[:-1]
    for i in reversed(range(len(h))):
        L.params += [PSpec(f"encoder.{i}.1.weight", (h[i],), "bn_w"), PSpec(f"encoder.{i}.1.bias", (h[i],), "bn_b"),
                     PSpec(f"encoder.{i}.0.weight", (h[i], cins[i], 3, 3), "conv_w", gemm_weight=True),
                     PSpec(f"encoder.{i}.0.bias", (h[i],), "bias")]
    L.bns += [BNSpec(f"encoder.{i}.1", h[i]) for i in range(len(h))]
    L.bns += [BNSpec(f"decoder.{i}.1", r[i + 1]) for i in range(len(r) - 1)]
    L.bns += [BNSpec("final_layer.1", r[-1])]
    # fc_mu/fc_var weights must be exactly adjacent for the fused view: pad rule keeps them
    # adjacent only if latent_dim*4C is a multiple of ALIGN (always true for 4C % 64 == 0)
    L.finalize()
    mu, var = L.by_name["fc_mu.weight"], L.by_name["fc_var.weight"]
    if var.offset != mu.offset + mu.numel:
        raise ValueError("fc_mu/fc_var weights are not contiguous; latent_dim*4*C must be a multiple of 64")
    mb, vb = L.by_name["fc_mu.bias"], L.by_name["fc_var.bias"]
    if vb.offset != mb.offset + mb.numel:
        raise ValueError("fc biases are not contiguous; latent_dim must be a multiple of 64")
    return L


def vq_layout(in_channels: int, embedding_dim: int, num_embeddings: int, hidden_dims: List[int]) -> Layout:
    """VQVAE (models/vq_vae.py:73-166): the reference's parameters in backward completion order
    (decoder output layer first, codebook, encoder last), each weight followed by its bias.
    No BatchNorm.  The codebook stays fp32 for the VectorQuantizer kernels."""
    spec = vq_param_spec(in_channels, embedding_dim, num_embeddings, hidden_dims)
    L = Layout()
    groups: List[List[PSpec]] = []
    for name, shape, kind in spec:
        ps = PSpec(name, tuple(shape), kind, gemm_weight=kind in ("conv_w", "convT_w"))
        if kind == "bias":
            groups[-1].append(ps)
        else:
            groups.append([ps])
    dec = [g for g in groups if g[0].name.startswith("decoder.")]
    cb = [g for g in groups if g[0].name.startswith("vq_layer.")]
    enc = [g for g in groups if g[0].name.startswith("encoder.")]
    for g in dec[::-1] + cb + enc[::-1]:
        L.params += g
    return L.finalize()


def vq_param_spec(in_channels: int, embedding_dim: int, num_embeddings: int, hidden_dims: List[int]):
    """(name, reference shape, kind) of every VQVAE parameter in the reference's registration
    order (vq_vae.py:94-166; Sequential indices include the parameter-free LeakyReLUs)."""
    h = list(hidden_dims)
    spec = []
    cin, idx = in_channels, 0
    for hd in h:                                                    # :95-102 Conv k4 s2 p1
        spec += [(f"encoder.{idx}.0.weight", (hd, cin, 4, 4), "conv_w"), (f"encoder.{idx}.0.bias", (hd,), "bias")]
        cin, idx = hd, idx + 1
    spec += [(f"encoder.{idx}.0.weight", (cin, cin, 3, 3), "conv_w"), (f"encoder.{idx}.0.bias", (cin,), "bias")]
    idx += 1
    for _ in range(6):                                              # :111-112 ResidualLayer
        spec += [(f"encoder.{idx}.resblock.0.weight", (cin, cin, 3, 3), "conv_w"),
                 (f"encoder.{idx}.resblock.2.weight", (cin, cin, 1, 1), "conv_w")]
        idx += 1
    idx += 1                                                        # :113 LeakyReLU
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
    for i in range(len(r) - 1):                                     # :142-152 ConvT k4 s2 p1
        spec += [(f"decoder.{idx}.0.weight", (r[i], r[i + 1], 4, 4), "convT_w"),
                 (f"decoder.{idx}.0.bias", (r[i + 1],), "bias")]
        idx += 1
    spec += [(f"decoder.{idx}.0.weight", (r[-1], 3, 4, 4), "convT_w"), (f"decoder.{idx}.0.bias", (3,), "bias")]
    return spec


def reference_key_order(in_channels: int, latent_dim: int, hidden_dims: List[int]) -> List[str]:
    """The reference's state_dict key order (module registration order, vanilla_vae.py:20-75)."""
    h = list(hidden_dims)
    r = h[::-1]
    keys = []
    bn = lambda p: [f"{p}.weight", f"{p}.bias", f"{p}.running_mean", f"{p}.running_var", f"{p}.num_batches_tracked"]
    for i in range(len(h)):
        keys += [f"encoder.{i}.0.weight", f"encoder.{i}.0.bias"] + bn(f"encoder.{i}.1")
    keys += ["fc_mu.weight", "fc_mu.bias", "fc_var.weight", "fc_var.bias", "decoder_input.weight", "decoder_input.bias"]
    for i in range(len(r) - 1):
        keys += [f"decoder.{i}.0.weight", f"decoder.{i}.0.bias"] + bn(f"decoder.{i}.1")
    keys += ["final_layer.0.weight", "final_layer.0.bias"] + bn("final_layer.1")
    keys += ["final_layer.3.weight", "final_layer.3.bias"]
    return keys


def default_init(layout: Layout, flat: torch.Tensor, running: torch.Tensor, generator: torch.Generator = None):
    """PyTorch-default-equivalent init (kaiming_uniform(a=sqrt(5)) => U(±1/sqrt(fan_in)) for
    weights and biases, fan_in from dim 1 as torch computes it; BN weight 1, bias 0; running
    mean 0 / var 1).  Drawn in reference layout then converted."""
    import math
    with torch.no_grad():
        fan_in = 1
        for p in layout.params:
            if p.kind in ("conv_w", "convT_w", "fc_w", "din_w"):
                s = p.ref_shape
                fan_in = s[1] * (s[2] * s[3] if len(s) == 4 else 1)
                b = 1.0 / math.sqrt(fan_in)
                t = (torch.rand(s, generator=generator) * 2 - 1) * b
            elif p.kind in ("bias", "din_b", "fc_b"):
                b = 1.0 / math.sqrt(fan_in)
                t = (torch.rand(p.ref_shape, generator=generator) * 2 - 1) * b
            elif p.kind == "bn_w":
                t = torch.ones(p.ref_shape)
            elif p.kind == "bn_b":
                t = torch.zeros(p.ref_shape)
            elif p.kind == "codebook":
                k = p.ref_shape[0]
                t = (torch.rand(p.ref_shape, generator=generator) * 2 - 1) / k
            else:
                raise ValueError(p.kind)
            flat[p.offset:p.offset + p.numel].copy_(to_native(p, t).reshape(-1).to(flat.device))
        for b in layout.bns:
            running[b.offset:b.offset + b.channels].fill_(0.0)
            running[b.offset + b.channels:b.offset + 2 * b.channels].fill_(1.0)
