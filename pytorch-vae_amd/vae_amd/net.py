"""The VanillaVAE-family network on libvaehip (VanillaVAE, BetaVAE, IWAE share it).

Reference: models/vanilla_vae.py:11-146 (network, reparameterize, ELBO), beta_vae.py:129-152,
iwae.py:95-160, experiment.py:45-86 (the step that calls it), experiment.py:308-311 (Adam).

Design (MI355X-first):
  * weights live in one flat fp32 buffer in native layouts (layout.py); in bf16 mode a bf16
    copy of the GEMM weights is refreshed by the fused Adam kernel;
  * activations are NHWC and stored *pre-BatchNorm*: every BatchNorm+LeakyReLU is applied by
    the consuming kernel on load, the producing kernel accumulates Σ/Σ² per channel in its
    epilogue, and backward folds BN-backward into the next kernel's load the same way;
  * a `StepPlan` preallocates every buffer for one batch shape and prebuilds the ctypes
    argument blocks of the ~40 launches of a training step, so a step is a fixed launch
    sequence on one stream — capturable into a HIP graph (engine.py).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import torch

from . import _lib as L
from .layout import Layout, default_init, reference_key_order, vanilla_layout

SLOPE = 0.01         # nn.LeakyReLU default
# layers at least this large take materialised operands by default (StepPlan.big_layer,
# StepPlan(mat_min_flops=...))
MAT_MIN_FLOPS = 4e9
BN_EPS = 1e-5
BN_MOMENTUM = 0.1


class VAENet:
    """Parameters + BatchNorm state of the VanillaVAE conv stack on one device."""

    def __init__(self, in_channels: int = 3, latent_dim: int = 128, hidden_dims: Optional[List[int]] = None,
                 img_size: int = 64, dtype: torch.dtype = torch.float32, device=None,
                 generator: Optional[torch.Generator] = None):
        self.in_channels = in_channels
        self.latent_dim = latent_dim
        self.hidden_dims = list(hidden_dims or [32, 64, 128, 256, 512])
        self.img_size = img_size
        if img_size % (2 ** len(self.hidden_dims)) or img_size // (2 ** len(self.hidden_dims)) != 2:
            raise ValueError("the reference's bottleneck is a [C,2,2] map (fc_mu = hidden_dims[-1]*4, "
                             "models/vanilla_vae.py:36): need img_size == 2 * 2**len(hidden_dims)")
        if in_channels != 3:
            raise ValueError("the head reconstructs 3 channels (vanilla_vae.py:73); in_channels must be 3")
        self.dtype = dtype
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.layout: Layout = vanilla_layout(in_channels, latent_dim, self.hidden_dims)
        self.ref_order = reference_key_order(in_channels, latent_dim, self.hidden_dims)
        self.params = torch.zeros(self.layout.total, dtype=torch.float32, device=self.device)
        self.running = torch.zeros(self.layout.bn_total, dtype=torch.float32, device=self.device)
        cpu_p = torch.zeros(self.layout.total)
        cpu_r = torch.zeros(self.layout.bn_total)
        default_init(self.layout, cpu_p, cpu_r, generator)
        self.params.copy_(cpu_p)
        self.running.copy_(cpu_r)
        self.lowp = (torch.zeros(self.layout.total, dtype=torch.bfloat16, device=self.device)
                     if dtype == torch.bfloat16 else None)
        self.num_batches_tracked = 0
        self._init_swaps()
        self.sync_lowp()

    # ------------------------------------------------------------------ state
    def _init_swaps(self):
        """bf16 mode: swapped-axes copies (vaehip.h wt_t) of the weights the bf16 GEMMs read
        transposed — every ConvTranspose2d (its forward) and every Conv2d with a data gradient
        (encoder blocks 1..) — refreshed with the bf16 copy (sync_lowp / FusedAdam.apply)."""
        self.wt_t: Dict[str, int] = {}
        self.swap_descs = None
        if self.lowp is None:
            return
        names = ([f"encoder.{i}.0.weight" for i in range(1, len(self.hidden_dims))] +
                 [f"decoder.{i}.0.weight" for i in range(len(self.hidden_dims) - 1)] + ["final_layer.0.weight"])
        self.swap_descs, self.lowp_t = make_swaps(self.layout, self.params, names, self.device, self.wt_t, self.lowp)

    def refresh_swaps(self, stream=None):
        self.swaps_stale = False
        if self.swap_descs is not None:
            L.call("vae_swap_axes", len(self.swap_descs), ctypes.byref(self.swap_descs),
                   stream if stream is not None else L.stream_ptr())

    @property
    def dcode(self) -> int:
        return L.dtype_code(self.dtype)

    def sync_lowp(self):
        """Refresh the bf16 weight copy from the fp32 master (bf16 mode only)."""
        if self.lowp is not None:
            L.call("vae_cast_bf16", self.params.numel(), self.params.data_ptr(), self.lowp.data_ptr(), L.stream_ptr())
            self.refresh_swaps()

    def load_reference_state_dict(self, sd: Dict[str, torch.Tensor]):
        self.layout.load_reference(self.params, self.running, {k: v.to(self.device) for k, v in sd.items()})
        nbt = sd.get(self.layout.bns[0].prefix + ".num_batches_tracked")
        self.num_batches_tracked = int(nbt) if nbt is not None else 0
        self.sync_lowp()

    def reference_state_dict(self) -> Dict[str, torch.Tensor]:
        return self.layout.export_reference(self.params, self.running, self.num_batches_tracked, self.ref_order)

    # ------------------------------------------------------------------ pointers
    def p(self, name: str) -> int:
        """fp32 master pointer of a parameter."""
        s = self.layout.by_name[name]
        return self.params.data_ptr() + 4 * s.offset

    def w(self, name: str) -> int:
        """Pointer of the copy a GEMM reads (bf16 in bf16 mode)."""
        s = self.layout.by_name[name]
        if self.lowp is not None:
            return self.lowp.data_ptr() + 2 * s.offset
        return self.params.data_ptr() + 4 * s.offset

    def run_mean(self, prefix: str) -> int:
        b = self.layout.bn_by_prefix[prefix]
        return self.running.data_ptr() + 4 * b.offset

    def run_var(self, prefix: str) -> int:
        b = self.layout.bn_by_prefix[prefix]
        return self.running.data_ptr() + 4 * (b.offset + b.channels)


class StepPlan:
    """All buffers and prebuilt launches of one training step for a fixed batch shape.

    loss: 'vanilla' | 'betaH' | 'betaB' | 'iwae';  samples: IWAE S (decoder batch B*S).
    grads land in `self.grads` (same layout as net.params); `zero` (grads, BN sums, SSE,
    d[mu|logvar]) is cleared by `vae_step_begin` at the start of every step."""

    def __init__(self, net: VAENet, batch: int, *, loss: str = "vanilla", kld_weight: float = 1e-8,
                 samples: int = 1, beta: float = 4.0, gamma: float = 1000.0, max_capacity: float = 25.0,
                 capacity_max_iter: float = 1e5, fused_loss: bool = True, training: bool = True,
                 concurrent: bool = False, fuse_bn: bool = False, bn_in_consumer: bool = True,
                 wg_overlap: bool = False, recon_loss: Optional[dict] = None,
                 deterministic: Optional[bool] = None, latent_kernels: bool = True, head_kernels: bool = True,
                 pad_rgb: bool = True, materialise: bool = True, mat_min_flops: float = MAT_MIN_FLOPS,
                 batch_wgrads: bool = True):
        # Route options (explicit arguments; every non-default route has a GPU test,
        # tests/test_gpu_routes.py): latent_kernels / head_kernels / pad_rgb / materialise /
        # batch_wgrads = False keep the generic per-op calls in place of the dedicated bottleneck
        # kernels, the 64/128-channel head kernels, the 8-channel padded RGB ends, materialised
        # BatchNorm operands for layers >= mat_min_flops, and the batched weight gradients.
        self.net = net
        self.materialise, self.mat_min_flops = bool(materialise), float(mat_min_flops)
        self.batch_wgrads_on = bool(batch_wgrads)
        # deterministic: every cross-workgroup reduction of the step in a fixed order (vaehip.h
        # vae_conv_args.deterministic), so two runs of the same step give bit-identical gradients;
        # the default for fp32 (parity) plans, unsupported by the bf16 kernels.
        self.deterministic = (net.dtype == torch.float32) if deterministic is None else bool(deterministic)
        # recon_loss (the Autoencoder's other reconstruction losses, vaehip.h vae_recon_loss):
        # {"kind": "center", "mask": [H][W] device tensor} or {"kind": "mssim", "window": 1-D window}.
        # The loss runs inside the step in place of the ELBO and seeds the backward with its
        # dL/drecon (grad_recon), as the drop-in path does with autograd's.
        self.recon_loss = recon_loss if training else None
        self.seed_recon = (not fused_loss) or self.recon_loss is not None
        self.B = batch
        # training=False: eval-mode BatchNorm (running statistics, nothing updated; the
        # reference's validation_step / sample / generate under model.eval()) — forward only
        self.training = training
        # fused_loss: the ELBO runs on the GPU inside the step and seeds the backward itself.
        # False (the BaseVAE drop-in, vae_amd.models): the loss is computed by the caller from
        # recon/mu/log_var and the backward is seeded with dL/drecon (grad_recon) and
        # dL/d[mu|log_var] (written into dmulv) instead.
        self.fused_loss = fused_loss
        # bn_in_consumer: no vae_bn_finalize launches in training — every kernel that applies a
        # BatchNorm reduces the producer's replicated statistics itself (vae_common.hpp
        # tab_build); the forward consumer's first workgroup updates the running statistics and
        # the weight-gradient call's first workgroup writes dL/dgamma, dL/dbeta and the conv
        # bias gradient (closed form).  Eval mode keeps vae_bn_finalize (running statistics).
        self.bn_in_consumer = bn_in_consumer and training
        self.S = samples if loss == "iwae" else 1
        self.loss_kind = {"vanilla": L.LOSS_VANILLA, "betaH": L.LOSS_BETA_H, "betaB": L.LOSS_BETA_B,
                          "iwae": L.LOSS_IWAE}[loss]
        self.kld_weight, self.beta, self.gamma = kld_weight, beta, gamma
        self.c_max, self.c_stop = max_capacity, capacity_max_iter
        dev, T = net.device, net.dtype
        D, h, img = net.latent_dim, net.hidden_dims, net.img_size
        B, BS = self.B, self.B * self.S
        # latent: the bottleneck (fc_mu|fc_var, reparameterize, decoder_input and their backward) on
        # the vae_latent_* kernels — two launches each way instead of nine (vaehip.h).  bf16 training
        # plans with the fused loss (the TrainStep engine) and the shapes those kernels take;
        # latent_kernels=False keeps the per-op calls.
        C5, r0 = net.hidden_dims[-1], net.hidden_dims[::-1][0]
        self.latent_fused = (T == torch.bfloat16 and training and fused_loss and net.latent_dim in (64, 128)
                             and C5 % 128 == 0 and (4 * r0) % 128 == 0 and net.img_size == 64
                             and latent_kernels)
        self._keep = []            # ctypes structs referenced by the call lists
        # wide_head: a final layer wider than the head kernels take on MFMA (bf16, 64-wide images:
        # 32, 64 or 128 channels — configs/big_ae.yaml's 128 included) runs the head Conv2d(C->3)
        # on the conv-GEMM paths with its 3 outputs zero-padded to 8, then vae_recon_fwd (tanh, NCHW
        # reconstruction, SSE, backward seed) — the VQ-VAE output layer's route (the Autoencoder's
        # 256-512-channel final layers, and the fp32 parity mode above 32).  The reconstruction seed
        # is the mean-MSE one, so not for IWAE's per-sample weights (S > 1 keeps the head kernels).
        # head_kernels=False keeps the conv-GEMM route for 64/128 channels.
        head_mfma = T == torch.bfloat16 and img == 64 and h[0] in (64, 128) and head_kernels
        self.wide_head = h[0] > 32 and self.S == 1 and not head_mfma

        # -------- buffers
        f32 = dict(dtype=torch.float32, device=dev)
        self.x = torch.zeros(B, 3, img, img, **f32)                     # NCHW input (reference layout)
        # bf16: the image and the first conv's weights carried as 8 zero-padded channels (packed
        # GEMM operands; vae_nchw_to_nhwc_pad / vae_pad_channels at the start of every step)
        self.pad_rgb = T == torch.bfloat16 and pad_rgb
        if self.pad_rgb:
            self.x8 = torch.zeros(B, img, img, 8, dtype=T, device=dev)
            self.w8 = torch.zeros(h[0] * 9 * 8, dtype=T, device=dev)
        self.eps = torch.zeros(BS, D, **f32)
        self.enc = []
        sp = img
        for c in h:
            sp //= 2
            self.enc.append(torch.empty(B, sp, sp, c, dtype=T, device=dev))
        self.mulv = torch.empty(B, 2 * D, **f32)
        self.z = torch.empty(BS, D, dtype=T, device=dev)
        r = h[::-1]
        self.h0 = torch.empty(BS, 2, 2, r[0], dtype=T, device=dev)
        self.dec = []
        sp = 2
        for i in range(len(r) - 1):
            sp *= 2
            self.dec.append(torch.empty(BS, sp, sp, r[i + 1], dtype=T, device=dev))
        self.fin = torch.empty(BS, img, img, r[-1], dtype=T, device=dev)
        if self.wide_head:
            # the head's output (pre-tanh) and its gradient, 8 channels (3 real); the head weights
            # zero-padded to 8 output rows (vae_pad_channels at the step's head: rows 3..7 stay 0)
            self.y8 = torch.zeros(BS, img, img, 8, dtype=T, device=dev)
            self.g8 = torch.zeros(BS, img, img, 8, dtype=T, device=dev)
            self.w8h = torch.zeros(8 * 9 * r[-1], dtype=T, device=dev)
            self.b8h = torch.zeros(8, dtype=torch.float32, device=dev)   # bias padded alike (lanes 3..7 stay 0)
        self.recon = torch.empty(BS, 3, img, img, **f32)
        self.grad_recon = torch.zeros(BS, 3, img, img, **f32) if self.seed_recon else None
        self.out = torch.zeros(4, **f32)                                  # loss, recon, KLD(report), kld
        self.per_img = torch.zeros(BS, **f32)
        self.head_coef = torch.zeros(BS, **f32)
        self.kl_coef = torch.zeros(BS, **f32)
        self.num_iter = torch.zeros(1, **f32)                             # BetaVAE-B counter (beta_vae.py:132)
        # backward buffers (gradients w.r.t. pre-activation of each stored tensor)
        self.g_enc = [torch.empty_like(t) for t in self.enc]
        self.g_h0 = torch.empty_like(self.h0)
        self.g_dec = [torch.empty_like(t) for t in self.dec]
        self.g_fin = torch.empty_like(self.fin)
        # zero region: grads | BN statistics | sse | dmulv   (16-B aligned pieces).  Every
        # BatchNorm has forward sums (Σ, Σ²) and backward sums (Σg·x̂, Σg), each kept in
        # `bn_reps(C)` replicas so that the producing kernels' per-block atomics spread out.
        nbn = sum(4 * bn_reps(b.channels) * b.channels for b in net.layout.bns)
        nz = (_pad4(net.layout.total) + 4 + nbn + _pad4(BS) + _pad4(B * 2 * D) + _pad4(2 * len(net.layout.bns)) +
              (_pad4(B * 2 * D) if self.latent_fused else 0) +
              (_pad4(8 * 9 * r[-1]) + 8 if self.wide_head else 0))
        self.zero = torch.zeros(nz, **f32)
        o = 0
        self.grads = self.zero[o:o + net.layout.total]; o += _pad4(net.layout.total)
        # loss terms averaged over ranks (experiment.py:55 log_dict(sync_dist=True)): copied from
        # `out` after the forward and reduced together with the last gradient bucket (engine.py)
        self.metrics = self.zero[o:o + 4]; o += 4
        self.bnfwd: Dict[str, torch.Tensor] = {}     # [2][reps][C]: Σ(y-shift), Σ(y-shift)²
        self.bnbwd: Dict[str, torch.Tensor] = {}     # [2][reps][C]: Σg·x̂ (dγ), Σg (dβ)
        for b in net.layout.bns:
            n = 2 * bn_reps(b.channels) * b.channels
            self.bnfwd[b.prefix] = self.zero[o:o + n].view(2, bn_reps(b.channels), b.channels); o += n
            self.bnbwd[b.prefix] = self.zero[o:o + n].view(2, bn_reps(b.channels), b.channels); o += n
        self.sse = self.zero[o:o + BS]; o += _pad4(BS)
        self.dmulv = self.zero[o:o + B * 2 * D]; o += _pad4(B * 2 * D)
        self.counters = self.zero[o:o + 2 * len(net.layout.bns)].view(torch.int32); o += _pad4(2 * len(net.layout.bns))
        if self.latent_fused:       # vae_latent_fc_fwd accumulates mu|log_var: zero at every step
            self.mulv = self.zero[o:o + B * 2 * D].view(B, 2 * D); o += _pad4(B * 2 * D)
        if self.wide_head:          # the padded head's weight / bias gradients (vae_unpad_accumulate)
            self.dw8h = self.zero[o:o + 8 * 9 * r[-1]]; o += _pad4(8 * 9 * r[-1])
            self.db8h = self.zero[o:o + 8]; o += 8
        # per-BatchNorm coefficient tables, rewritten every step by vae_bn_finalize:
        # forward [4][C] (BN_ACT) then backward [3][C] (BN_DY)
        self.bntab: Dict[str, torch.Tensor] = {
            b.prefix: torch.zeros(7 * b.channels, **f32) for b in net.layout.bns}
        self.step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.fwd_calls: List = []
        self.bwd_calls: List = []
        # side stream for the weight gradients (run_calls); None: one stream
        self.side = torch.cuda.Stream(device=dev) if (concurrent and training) else None
        # wg_overlap: the decoder's weight gradients (one batch) on a side stream, beside the
        # encoder's data-gradient chain (batch_wgrads); one fork and one join per step.  Off by
        # default: measured 0.670 vs 0.648 ms/step (B=64, graph-replayed) — the graph's cross-stream
        # edges cost more than the overlap gains, as the per-call side stream of round 1 did
        self.wg_overlap = wg_overlap and training and not concurrent
        self._mat_a: Dict[str, torch.Tensor] = {}         # materialised lrelu(BN(y)) per BatchNorm
        self._mat_dz: Dict[str, torch.Tensor] = {}        # materialised BN-backward gradients
        self.side_all = self.side is not None            # concurrent: every weight-gradient call
        if self.wg_overlap:
            self.side = torch.cuda.Stream(device=dev)
        self._build()
        # the backward as built, one call per op; bwd_calls batches its weight gradients
        # (batch_wgrads: one vae_conv_bwd_filter_batch per backward segment)
        self.bwd_calls_raw = list(self.bwd_calls)
        if fuse_bn and training:
            # each BatchNorm finalisation carried by the call that produces its statistics
            # (vaehip.h bn_finalize).  The library runs it as its own launch right after the
            # producer: an in-kernel last-workgroup version measured 0.81 -> 1.26 ms/step (an
            # agent-scope release in every workgroup, and lower GEMM occupancy).
            self._fuse_finalize(self.fwd_calls)
            self._fuse_finalize(self.bwd_calls)
            self.bwd_calls_raw = list(self.bwd_calls)
        self.batch_wgrads([len(self.bwd_calls_raw)])

    def defer_reductions(self) -> bool:
        """Leave the step's weight-gradient slab reductions — the head backward's filter partials,
        the full-resolution ConvT backward's, the grouped weight gradients' K slices — and the loss
        fused into the head backward to the optimizer launch (vaehip.h defer_reduce,
        vae_adam_step_ex): three launches fewer per step.  For the one-rank fused step
        (engine.TrainStep), whose only reader of the gradients is its own Adam; each deferring call
        gets a workspace of its own, kept until the optimizer reads it.  bf16 training plans only;
        returns whether anything is deferred."""
        if self.net.dtype != torch.bfloat16 or not self.training:
            return False
        n = 0
        for fn, ref in self.bwd_calls:
            if fn == BATCH_FN:
                for a in ref.args:
                    a.defer_reduce = 1
                    n += 1
            elif fn in ("vae_convT2d_bwd", "vae_head_bwd") and ref is not None and not isinstance(ref, tuple):
                ref._obj.defer_reduce = 1
                n += 1
        if n:
            size_workspaces(self, [self.fwd_calls, self.bwd_calls])
        return n > 0

    def batch_wgrads(self, ends):
        """Rebuild bwd_calls from bwd_calls_raw with the conv / convT weight gradients of each
        backward segment (calls [ends[k-1], ends[k]) of the raw list) moved into one
        vae_conv_bwd_filter_batch call at the segment's end, and size the workspaces.  Returns the
        segment ends as indices into the new list.  batch_wgrads=False (constructor) keeps one call
        per layer.

        With one segment (one rank) and wg_overlap, the decoder's weight gradients form a batch of
        their own, issued on the side stream where the decoder's data-gradient chain ends: it runs
        beside the encoder's data gradients (the critical path) instead of after them."""
        splits = []
        if self.wg_overlap and len(ends) == 1:
            raw = self.bwd_calls_raw
            # the decoder's backward ends where the bottleneck's begins (the fused latent kernels
            # or the latent Linear layers)
            first_lin = next((i for i, (fn, _) in enumerate(raw)
                              if fn in ("vae_latent_dec_bwd", "vae_linear_bwd_data")), None)
            if first_lin is not None:
                splits = [first_lin]
        if self.deterministic:
            for fn, ref in list(self.fwd_calls) + list(self.bwd_calls_raw):
                obj = getattr(ref, "_obj", ref)
                if hasattr(obj, "deterministic"):
                    obj.deterministic = 1
        self.bwd_calls, new_ends = batch_filter_calls(self.bwd_calls_raw, ends, splits,
                                                      enabled=self.batch_wgrads_on)
        size_workspaces(self, [self.fwd_calls, self.bwd_calls])
        return new_ends

    # ------------------------------------------------------------------ helpers
    def g(self, name: str) -> int:
        s = self.net.layout.by_name[name]
        return self.grads.data_ptr() + 4 * s.offset

    def _bn_prod_bias(self, prefix: str) -> str:
        return prefix[:-2] + ".0.bias"          # "encoder.3.1" -> "encoder.3.0.bias"

    def bn_xf(self, prefix: str, kind: int, count: int, aux=None, running: bool = False,
              table: Optional[bool] = None) -> L.Xform:
        if table is None:
            table = not self.bn_in_consumer or self.wide_bn(prefix)
        net = self.net
        C = net.layout.bn_by_prefix[prefix].channels
        s = self.bnfwd[prefix]
        xf = L.Xform(kind=kind, channels=C, slope=SLOPE, count=float(count), eps=BN_EPS, momentum=BN_MOMENTUM)
        xf.sum = s[0].data_ptr()
        xf.sumsq = s[1].data_ptr()
        xf.reps = s.shape[1]
        xf.rstride = C
        xf.shift = net.p(self._bn_prod_bias(prefix))
        xf.gamma = net.p(prefix + ".weight")
        xf.beta = net.p(prefix + ".bias")
        if kind == L.X_BN_DY:
            xf.dgamma = self.bnbwd[prefix][0].data_ptr()
            xf.dbeta = self.bnbwd[prefix][1].data_ptr()
        if table:
            t = self.bntab[prefix]
            xf.table = t.data_ptr() + (4 * 4 * C if kind == L.X_BN_DY else 0)
        if aux is not None:
            xf.aux = aux.data_ptr()
        if running:
            xf.running_mean = net.run_mean(prefix)
            xf.running_var = net.run_var(prefix)
        return xf

    def wide_bn(self, prefix: str) -> bool:
        """A BatchNorm wider than 512 channels (the Autoencoder's 1024-4096): its coefficient table is
        built once per step by vae_bn_finalize instead of in every consumer workgroup (the in-kernel
        build reduces <= 512 channels in one round of loads; wider ones would loop per channel in each
        of thousands of workgroups)."""
        return self.bn_in_consumer and self.net.layout.bn_by_prefix[prefix].channels > 512

    def fwd_sums(self, arg, prefix: str):
        """Producer side of a BatchNorm's forward statistics (conv / convT fwd epilogue)."""
        s = self.bnfwd[prefix]
        arg.y_sum, arg.y_sumsq = s[0].data_ptr(), s[1].data_ptr()
        arg.sum_reps, arg.sum_rstride = s.shape[1], s.shape[2]

    def bwd_sums(self, arg, prefix: str):
        """Producer side of a BatchNorm's backward sums (bwd_data epilogue of the next layer)."""
        s = self.bnbwd[prefix]
        arg.dx_dgamma, arg.dx_dbeta = s[0].data_ptr(), s[1].data_ptr()
        arg.sum_reps, arg.sum_rstride = s.shape[1], s.shape[2]

    def bwd_extras(self, arg, prefix: str):
        """bn_in_consumer: the weight-gradient call of the conv feeding BatchNorm `prefix` also
        publishes that BatchNorm's dL/dgamma, dL/dbeta and the conv's bias gradient (what
        vae_bn_finalize mode 1 did)."""
        if not self.bn_in_consumer or self.wide_bn(prefix):
            return
        xf = arg.dy_xf
        xf.dgamma_out = self.g(prefix + ".weight")
        xf.dbeta_out = self.g(prefix + ".bias")
        arg.dy_xf = xf
        arg.db = self.g(self._bn_prod_bias(prefix))

    def bn_finalize(self, lst, prefix: str, mode: int, count: int):
        """Queue vae_bn_finalize for one BatchNorm: mode 0 after the conv producing its input
        (table + running statistics), mode 1 after the kernel producing its backward sums
        (table + dγ, dβ + the producing conv's bias gradient in closed form)."""
        if self.bn_in_consumer and mode in (0, 1) and not self.wide_bn(prefix):
            return
        C = self.net.layout.bn_by_prefix[prefix].channels
        a = L.BnArgs(mode=mode)
        a.xf = self.bn_xf(prefix, L.X_BN_DY if mode == 1 else L.X_BN_ACT, count, running=(mode != 1), table=False)
        a.table = self.bntab[prefix].data_ptr() + (4 * 4 * C if mode == 1 else 0)
        if mode == 1:
            a.xf.dgamma_out = self.g(prefix + ".weight")
            a.xf.dbeta_out = self.g(prefix + ".bias")
            a.db = self.g(self._bn_prod_bias(prefix))
        self._add(lst, "vae_bn_finalize", a)

    # ---- materialised transforms for the large layers (vaehip.h vae_bn_apply + vae_bgemm.hip)
    def big_layer(self, flops: float, cin: int, cout: int) -> bool:
        """A layer whose GEMMs take materialised (transform-free) operands: bf16 training, >= 4 GFLOP
        per pass and >= 128 channels on both sides (the Autoencoder's wide layers, whose GEMMs run on
        the 128 x 128 LDS-DMA tiles; the VanillaVAE's are 0.6 GFLOP, and IWAE's 32-channel final ConvT
        reaches 6 GFLOP at B*S = 320 but stays on its own kernels: materialised it measured 1.10 vs
        1.04 ms/step).  materialise=False keeps every transform fused into its consumers."""
        return (self.net.dtype == torch.bfloat16 and self.training and self.materialise
                and flops >= self.mat_min_flops and min(cin, cout) >= 128)

    def mat_act(self, F, prefix: str, t: torch.Tensor, count: int):
        """lrelu(BN(t)) written once (vae_bn_apply: running statistics updated there, the forward's
        first consumer of the BatchNorm); returns the tensor every later consumer reads plainly."""
        out = self._mat_a.get(prefix)
        if out is None:
            out = self._mat_a[prefix] = torch.empty_like(t)
            a = L.BnApplyArgs(dtype=self.net.dcode, rows=t.numel() // t.shape[-1], channels=t.shape[-1])
            a.x, a.out = t.data_ptr(), out.data_ptr()
            a.xf = self.bn_xf(prefix, L.X_BN_ACT, count, running=True)
            self._add(F, "vae_bn_apply", a)
        return out

    def mat_dz(self, Bw, prefix: str, g: torch.Tensor, y: torch.Tensor, count: int):
        """The BatchNorm-backward gradient A g + B y + C of a big layer's output written once
        (vae_bn_apply BN_DY, which also publishes dgamma, dbeta and the conv's closed-form bias
        gradient unless vae_bn_finalize did); the layer's data and weight gradients read it plainly."""
        out = self._mat_dz[prefix] = torch.empty_like(g)
        a = L.BnApplyArgs(dtype=self.net.dcode, rows=g.numel() // g.shape[-1], channels=g.shape[-1])
        a.x, a.out = g.data_ptr(), out.data_ptr()
        xf = self.bn_xf(prefix, L.X_BN_DY, count, aux=y)
        if self.bn_in_consumer and not self.wide_bn(prefix):
            xf.dgamma_out = self.g(prefix + ".weight")
            xf.dbeta_out = self.g(prefix + ".bias")
            a.db = self.g(self._bn_prod_bias(prefix))
        a.xf = xf
        self._add(Bw, "vae_bn_apply", a)
        return out

    def _fuse_finalize(self, calls):
        """Fold every vae_bn_finalize call (modes 0/1) into the call that produced its statistics
        (the GEMM whose epilogue wrote them): that call's last workgroup then builds the table
        (vaehip.h bn_finalize), saving a dependent launch per BatchNorm and direction."""
        out = []
        nctr = 0
        for fn, ref in calls:
            if fn == "vae_bn_finalize" and ref is not None and ref._obj.mode in (0, 1):
                bn = ref._obj
                key = bn.xf.sum if bn.mode == 0 else bn.xf.dgamma
                prod = None
                for pfn, pref in reversed(out):
                    a = pref._obj if pref is not None else None
                    if a is None or not hasattr(a, "bn_counter"):
                        continue
                    if bn.mode == 0 and getattr(a, "y_sum", None) == key:
                        prod = a
                    elif bn.mode == 1 and getattr(a, "dx_dgamma", None) == key:
                        prod = a
                    if prod is not None:
                        break
                if prod is not None and not prod.bn_finalize:
                    prod.bn_finalize = ctypes.pointer(bn)
                    prod.bn_counter = self.counters.data_ptr() + 4 * nctr
                    nctr += 1
                    continue
            out.append((fn, ref))
        calls[:] = out

    def _add(self, lst, fn, arg):
        self._keep.append(arg)
        lst.append((fn, ctypes.byref(arg)))

    # ------------------------------------------------------------------ plan
    def _build(self):
        net, T = self.net, self.net.dcode
        h = net.hidden_dims
        r = h[::-1]
        D = net.latent_dim
        B, BS = self.B, self.B * self.S
        img = net.img_size
        nenc = len(h)
        enc_pre = [f"encoder.{i}.1" for i in range(nenc)]
        dec_pre = [f"decoder.{i}.1" for i in range(len(r) - 1)] + ["final_layer.1"]
        dec_w = [f"decoder.{i}.0" for i in range(len(r) - 1)] + ["final_layer.0"]
        dec_out = self.dec + [self.fin]
        g_dec_out = self.g_dec + [self.g_fin]

        def cnt(t):   # BN reduction size of a stored NHWC map
            return t.shape[0] * t.shape[1] * t.shape[2]

        F = self.fwd_calls
        fmode = 0 if self.training else 2            # bn_finalize: batch statistics / running statistics
        if self.pad_rgb:
            F.append(("vae_nchw_to_nhwc_pad", (T, B, 3, img, img, 8, self.x.data_ptr(), self.x8.data_ptr())))
            F.append(("vae_pad_channels", (T, h[0] * 9, 3, 8, net.w("encoder.0.0.weight"), self.w8.data_ptr())))
        if self.wide_head:          # head weights [3][3][3][C] -> [8][3][3][C] (one row of 27C -> 72C)
            F.append(("vae_pad_channels", (T, 1, 27 * r[-1], 72 * r[-1], net.w("final_layer.3.weight"),
                                           self.w8h.data_ptr())))
            # the GEMM epilogue reads 8 bias values (its N): pad the 3-element bias too
            F.append(("vae_pad_channels", (L.F32, 1, 3, 8, net.p("final_layer.3.bias"), self.b8h.data_ptr())))
        # ---------------------------------------------------------------- encoder
        sp = img
        for i in range(nenc):
            a = L.ConvArgs(dtype=T, n=B, h=sp, w=sp, c=(3 if i == 0 else h[i - 1]), k=h[i], p=sp // 2, q=sp // 2,
                           r=3, stride=2, pad=1)
            if i == 0 and self.pad_rgb:
                a.c, a.x = 8, self.x8.data_ptr()
            elif i == 0:
                a.x_nchw_f32 = 1
                a.x = self.x.data_ptr()
            elif self.big_layer(2.0 * B * (sp // 2) ** 2 * h[i] * 9 * h[i - 1], h[i - 1], h[i]):
                a.x = self.mat_act(F, enc_pre[i - 1], self.enc[i - 1], cnt(self.enc[i - 1])).data_ptr()
            else:
                a.x = self.enc[i - 1].data_ptr()
                a.x_xf = self.bn_xf(enc_pre[i - 1], L.X_BN_ACT, cnt(self.enc[i - 1]), running=True)
            a.wt = self.w8.data_ptr() if (i == 0 and self.pad_rgb) else net.w(f"encoder.{i}.0.weight")
            a.bias = net.p(f"encoder.{i}.0.bias")
            a.y = self.enc[i].data_ptr()
            if self.training:
                self.fwd_sums(a, enc_pre[i])
            self._add(F, "vae_conv2d_fwd", a)
            self.bn_finalize(F, enc_pre[i], fmode, cnt(self.enc[i]))
            sp //= 2
        # ---------------------------------------------------------------- fc_mu | fc_var
        if self.latent_fused:
            la = self._latent = L.LatentArgs(dtype=T, batch=B, samples=self.S, latent=D, in_features=4 * h[-1],
                                              out_features=4 * r[0])
            la.x = self.enc[-1].data_ptr()
            la.x_xf = self.bn_xf(enc_pre[-1], L.X_BN_ACT, cnt(self.enc[-1]), running=True)
            la.w1, la.b1 = net.w("fc_mu.weight"), net.p("fc_mu.bias")
            la.mulv, la.eps, la.z = self.mulv.data_ptr(), self.eps.data_ptr(), self.z.data_ptr()
            la.w2, la.b2 = net.w("decoder_input.weight"), net.p("decoder_input.bias")
            la.h = self.h0.data_ptr()
            self._add(F, "vae_latent_fc_fwd", la)
            self.n_encode = len(F)
            self.n_decode0 = len(F)            # (decode() of a fused plan starts at the reparameterization)
            F.append(("vae_latent_dec_fwd", F[-1][1]))
        a = L.LinearArgs(dtype=T, m=B, n=2 * D, k=4 * h[-1])
        a.x = self.enc[-1].data_ptr()
        a.x_xf = self.bn_xf(enc_pre[-1], L.X_BN_ACT, cnt(self.enc[-1]), running=True)
        a.wt = net.w("fc_mu.weight")
        a.bias = net.p("fc_mu.bias")
        a.y = self.mulv.data_ptr()
        a.y_f32 = 1
        self._reparam = (T, BS, self.S, D, self.mulv.data_ptr(), self.eps.data_ptr(), self.z.data_ptr())
        if not self.latent_fused:
            self._add(F, "vae_linear_fwd", a)
            self.n_encode = len(F)             # calls of encode(): encoder + fc_mu|fc_var
            F.append(("vae_reparam_fwd", self._reparam))
            self.n_decode0 = len(F)            # decode(): decoder_input .. head
            # ------------------------------------------------------------ decoder_input
            a = L.LinearArgs(dtype=T, m=BS, n=4 * r[0], k=D)
            a.x = self.z.data_ptr()
            a.wt = net.w("decoder_input.weight")
            a.bias = net.p("decoder_input.bias")
            a.y = self.h0.data_ptr()
            self._add(F, "vae_linear_fwd", a)
        # ---------------------------------------------------------------- decoder (ConvT)
        sp = 2
        prev, prev_pre = self.h0, None
        for i in range(len(r)):
            cin = r[i] if i < len(r) - 1 else r[-1]
            cout = r[i + 1] if i < len(r) - 1 else r[-1]
            a = L.ConvArgs(dtype=T, n=BS, h=sp, w=sp, c=cin, k=cout, p=2 * sp, q=2 * sp, r=3, stride=2, pad=1)
            a.x = prev.data_ptr()
            if prev_pre is not None and self.big_layer(2.0 * BS * sp * sp * cin * cout * 9, cin, cout):
                a.x = self.mat_act(F, prev_pre, prev, cnt(prev)).data_ptr()
            elif prev_pre is not None:
                a.x_xf = self.bn_xf(prev_pre, L.X_BN_ACT, cnt(prev), running=True)
            a.wt = net.w(dec_w[i] + ".weight")
            a.wt_t = net.wt_t.get(dec_w[i] + ".weight")
            a.bias = net.p(dec_w[i] + ".bias")
            a.y = dec_out[i].data_ptr()
            if self.training:
                self.fwd_sums(a, dec_pre[i])
            self._add(F, "vae_convT2d_fwd", a)
            self.bn_finalize(F, dec_pre[i], fmode, cnt(dec_out[i]))
            prev, prev_pre = dec_out[i], dec_pre[i]
            sp *= 2
        # ---------------------------------------------------------------- head + SSE
        if self.wide_head:
            self._wide_head_fwd(F, cnt)
        hd = L.HeadArgs(dtype=T, n=BS, h=img, w=img, c=r[-1], samples=self.S)
        hd.x = self.fin.data_ptr()
        hd.x_xf = self.bn_xf("final_layer.1", L.X_BN_ACT, cnt(self.fin), running=True)
        hd.wt = net.p("final_layer.3.weight")
        hd.bias = net.p("final_layer.3.bias")
        hd.target = self.x.data_ptr()
        hd.recon = self.recon.data_ptr()
        hd.sse = self.sse.data_ptr()
        if not self.wide_head:
            self._add(F, "vae_head_fwd", hd)
        # ---------------------------------------------------------------- ELBO
        e = L.ElboArgs(kind=self.loss_kind, batch=B, samples=self.S, latent=D, img_elems=3 * img * img,
                       kld_weight=self.kld_weight, beta=self.beta, gamma=self.gamma, c_max=self.c_max,
                       c_stop_iter=self.c_stop)
        e.iter = self.num_iter.data_ptr()
        e.mulv = self.mulv.data_ptr()
        e.sse = self.sse.data_ptr()
        e.out = self.out.data_ptr()
        e.per_img = self.per_img.data_ptr()
        e.head_coef = self.head_coef.data_ptr()
        e.kl_coef = self.kl_coef.data_ptr()
        self.n_decode1 = len(F)
        self.elbo_args = e
        # elbo_in_head: the loss evaluated by the head backward (vaehip.h vae_head_args.elbo: one
        # extra workgroup of its filter-partial reduction, the seed coefficient a constant) instead
        # of a vae_elbo_fwd launch between the forward and the backward — the bf16 head kernels,
        # the vanilla / BetaVAE-H losses (their seeds do not depend on the batch), one sample
        self.elbo_in_head = (self.fused_loss and self.training and self.recon_loss is None and not self.wide_head
                             and self.S == 1 and T == L.BF16 and B <= 1024
                             and self.loss_kind in (L.LOSS_VANILLA, L.LOSS_BETA_H))
        # (with elbo_in_head, out / per_img / head_coef / kl_coef are written by the backward: they
        # are this step's only after backward() — loss_dict() raises in between)
        self._loss_pending = False
        if self.recon_loss is not None:
            self._add_recon_loss(F)
        elif self.fused_loss and not self.elbo_in_head:
            self._add(F, "vae_elbo_fwd", e)

        # ================================================================ backward
        if not self.training:
            return
        Bw = self.bwd_calls
        hb = L.HeadArgs(dtype=T, n=BS, h=img, w=img, c=r[-1], samples=self.S)
        hb.x = self.fin.data_ptr()
        hb.x_xf = self.bn_xf("final_layer.1", L.X_BN_ACT, cnt(self.fin))
        hb.wt = net.p("final_layer.3.weight")
        hb.bias = net.p("final_layer.3.bias")
        hb.target = self.x.data_ptr()
        hb.recon = self.recon.data_ptr()
        if self.seed_recon:
            hb.grad_recon = self.grad_recon.data_ptr()
        else:
            hb.coef = self.head_coef.data_ptr()
        hb.dx = self.g_fin.data_ptr()
        hb.dx_epi = self.bn_xf("final_layer.1", L.X_BN_ACT, cnt(self.fin))
        hb.dx_epi.aux = self.fin.data_ptr()
        self.bwd_sums(hb, "final_layer.1")
        hb.dw = self.g("final_layer.3.weight")
        hb.db = self.g("final_layer.3.bias")
        if self.elbo_in_head:
            hb.elbo = ctypes.addressof(e)
        if self.wide_head:
            self._wide_head_bwd(Bw, cnt)
            self._head_bwd = None
        else:
            self._add(Bw, "vae_head_bwd", hb)
            self._head_bwd = hb
        # decoder, last block first
        sps = [2 * 2 ** i for i in range(len(r))]          # input spatial of each ConvT
        for i in reversed(range(len(r))):
            sp = sps[i]
            cin = r[i] if i < len(r) - 1 else r[-1]
            cout = r[i + 1] if i < len(r) - 1 else r[-1]
            x_t = self.h0 if i == 0 else dec_out[i - 1]
            gx_t = self.g_h0 if i == 0 else g_dec_out[i - 1]
            self.bn_finalize(Bw, dec_pre[i], 1, cnt(dec_out[i]))
            dy_xf = self.bn_xf(dec_pre[i], L.X_BN_DY, cnt(dec_out[i]), aux=dec_out[i])
            dz = (self.mat_dz(Bw, dec_pre[i], g_dec_out[i], dec_out[i], cnt(dec_out[i]))
                  if self.big_layer(2.0 * BS * sp * sp * cin * cout * 9, cin, cout) else None)
            if dz is not None:
                dy_xf = L.Xform(kind=L.X_NONE, channels=cout)
            a = L.ConvArgs(dtype=T, n=BS, h=sp, w=sp, c=cin, k=cout, p=2 * sp, q=2 * sp, r=3, stride=2, pad=1)
            a.dy = (dz if dz is not None else g_dec_out[i]).data_ptr()
            a.dy_xf = dy_xf
            a.wt = net.w(dec_w[i] + ".weight")
            a.dx = gx_t.data_ptr()
            if i > 0:
                a.dx_epi = self.bn_xf(dec_pre[i - 1], L.X_BN_ACT, cnt(x_t), aux=x_t)
                self.bwd_sums(a, dec_pre[i - 1])
            f = a if i == len(r) - 1 else L.ConvArgs(dtype=T, n=BS, h=sp, w=sp, c=cin, k=cout, p=2 * sp, q=2 * sp,
                                                      r=3, stride=2, pad=1)
            f.x = x_t.data_ptr()
            if i > 0 and dec_pre[i - 1] in self._mat_a:
                f.x = self._mat_a[dec_pre[i - 1]].data_ptr()
            elif i > 0:
                f.x_xf = self.bn_xf(dec_pre[i - 1], L.X_BN_ACT, cnt(x_t))
            f.dy = (dz if dz is not None else g_dec_out[i]).data_ptr()
            f.dy_xf = dy_xf
            f.dw = self.g(dec_w[i] + ".weight")      # bias gradient: closed form (bn_finalize / bwd_extras)
            if dz is None:
                self.bwd_extras(f, dec_pre[i])
            if i == len(r) - 1:
                # the full-resolution last ConvTranspose2d: both gradients in one pass over dy
                # (vaehip.h vae_convT2d_bwd; other shapes run the two calls inside it)
                self._add(Bw, "vae_convT2d_bwd", a)
            else:
                self._add(Bw, "vae_convT2d_bwd_data", a)
                self._add(Bw, "vae_convT2d_bwd_filter", f)
        if self.latent_fused:
            la = self._latent
            la.dh, la.kl_coef, la.dmulv = self.g_h0.data_ptr(), self.kl_coef.data_ptr(), self.dmulv.data_ptr()
            la.dw2, la.db2 = self.g("decoder_input.weight"), self.g("decoder_input.bias")
            la.dx = self.g_enc[-1].data_ptr()
            la.dx_epi = self.bn_xf(enc_pre[-1], L.X_BN_ACT, cnt(self.enc[-1]), aux=self.enc[-1])
            s = self.bnbwd[enc_pre[-1]]
            la.dx_dgamma, la.dx_dbeta = s[0].data_ptr(), s[1].data_ptr()
            la.sum_reps, la.sum_rstride = s.shape[1], s.shape[2]
            la.dw1, la.db1 = self.g("fc_mu.weight"), self.g("fc_mu.bias")
            Bw.append(("vae_latent_dec_bwd", F[self.n_encode - 1][1]))
            Bw.append(("vae_latent_fc_bwd", F[self.n_encode - 1][1]))
            self._reparam_bwd = None
        # decoder_input: dz -> d[mu|logvar] (reparameterization + KL), and its weight grads
        a = L.LinearArgs(dtype=T, m=BS, n=4 * r[0], k=D)
        a.dy = self.g_h0.data_ptr()
        a.wt = net.w("decoder_input.weight")
        a.mulv = self.mulv.data_ptr()
        a.eps = self.eps.data_ptr()
        a.kl_coef = self.kl_coef.data_ptr() if self.fused_loss else None
        a.dmulv = self.dmulv.data_ptr()
        a.samples = self.S
        if not self.latent_fused:
            self._add(Bw, "vae_linear_bwd_data", a)
            self._reparam_bwd = a
        f = L.LinearArgs(dtype=T, m=BS, n=4 * r[0], k=D)
        f.dy = self.g_h0.data_ptr()
        f.x = self.z.data_ptr()
        f.dw = self.g("decoder_input.weight")
        f.db = self.g("decoder_input.bias")
        if not self.latent_fused:
            self._add(Bw, "vae_linear_bwd_filter", f)
        # fc_mu | fc_var
        a = L.LinearArgs(dtype=T, m=B, n=2 * D, k=4 * h[-1])
        a.dy = self.dmulv.data_ptr()
        a.dy_f32 = 1
        a.wt = net.w("fc_mu.weight")
        a.dx = self.g_enc[-1].data_ptr()
        a.dx_epi = self.bn_xf(enc_pre[-1], L.X_BN_ACT, cnt(self.enc[-1]), aux=self.enc[-1])
        self.bwd_sums(a, enc_pre[-1])
        if not self.latent_fused:
            self._add(Bw, "vae_linear_bwd_data", a)
        f = L.LinearArgs(dtype=T, m=B, n=2 * D, k=4 * h[-1])
        f.dy = self.dmulv.data_ptr()
        f.dy_f32 = 1
        f.x = self.enc[-1].data_ptr()
        f.x_xf = self.bn_xf(enc_pre[-1], L.X_BN_ACT, cnt(self.enc[-1]))
        f.dw = self.g("fc_mu.weight")
        f.db = self.g("fc_mu.bias")
        if not self.latent_fused:
            self._add(Bw, "vae_linear_bwd_filter", f)
        # encoder, last block first
        sps = [img // 2 ** i for i in range(nenc)]
        for i in reversed(range(nenc)):
            sp = sps[i]
            cin = 3 if i == 0 else h[i - 1]
            self.bn_finalize(Bw, enc_pre[i], 1, cnt(self.enc[i]))
            dy_xf = self.bn_xf(enc_pre[i], L.X_BN_DY, cnt(self.enc[i]), aux=self.enc[i])
            dz = (self.mat_dz(Bw, enc_pre[i], self.g_enc[i], self.enc[i], cnt(self.enc[i]))
                  if i > 0 and self.big_layer(2.0 * B * (sp // 2) ** 2 * h[i] * 9 * cin, cin, h[i]) else None)
            if dz is not None:
                dy_xf = L.Xform(kind=L.X_NONE, channels=h[i])
            f = L.ConvArgs(dtype=T, n=B, h=sp, w=sp, c=cin, k=h[i], p=sp // 2, q=sp // 2, r=3, stride=2, pad=1)
            f.dy = (dz if dz is not None else self.g_enc[i]).data_ptr()
            f.dy_xf = dy_xf
            if i == 0 and self.pad_rgb:
                # the 8-channel padded image; dW lands in the parameter's own [k][3][3][3] layout
                # (vaehip.h dw_inner: the weight-gradient GEMM drops the pad channels)
                f.c, f.x, f.dw, f.dw_inner = 8, self.x8.data_ptr(), self.g("encoder.0.0.weight"), 3
            elif i == 0:
                f.x_nchw_f32 = 1
                f.x = self.x.data_ptr()
            elif enc_pre[i - 1] in self._mat_a:
                f.x = self._mat_a[enc_pre[i - 1]].data_ptr()
            else:
                f.x = self.enc[i - 1].data_ptr()
                f.x_xf = self.bn_xf(enc_pre[i - 1], L.X_BN_ACT, cnt(self.enc[i - 1]))
            if not (i == 0 and self.pad_rgb):
                f.dw = self.g(f"encoder.{i}.0.weight")   # bias gradient: closed form (bn_finalize / bwd_extras)
            if dz is None:
                self.bwd_extras(f, enc_pre[i])
            self._add(Bw, "vae_conv2d_bwd_filter", f)
            if i > 0:
                a = L.ConvArgs(dtype=T, n=B, h=sp, w=sp, c=cin, k=h[i], p=sp // 2, q=sp // 2, r=3, stride=2, pad=1)
                a.dy = (dz if dz is not None else self.g_enc[i]).data_ptr()
                a.dy_xf = dy_xf
                a.wt = net.w(f"encoder.{i}.0.weight")
                a.wt_t = net.wt_t.get(f"encoder.{i}.0.weight")
                a.dx = self.g_enc[i - 1].data_ptr()
                a.dx_epi = self.bn_xf(enc_pre[i - 1], L.X_BN_ACT, cnt(self.enc[i - 1]), aux=self.enc[i - 1])
                self.bwd_sums(a, enc_pre[i - 1])
                self._add(Bw, "vae_conv2d_bwd_data", a)

    def _add_recon_loss(self, F):
        """The recon_loss call closing the forward (vae_recon_loss): loss terms into `out`, per-image
        MSE from the head's SSE, and dL/drecon into grad_recon for the backward."""
        img, BS = self.net.img_size, self.B * self.S
        cfg = self.recon_loss
        if cfg["kind"] == "center":
            self._rl_mask = cfg["mask"].to(self.net.device, torch.float32).contiguous().view(img, img)
            a = L.recon_loss_args(L.RLOSS_CENTER, BS, 3, img, img, mask=self._rl_mask)
        elif cfg["kind"] == "mssim":
            a = L.recon_loss_args(L.RLOSS_MSSIM, BS, 3, img, img, window=cfg["window"],
                                  levels=cfg.get("levels", 5), normalize=cfg.get("normalize", True))
        else:
            raise ValueError(f"recon_loss kind {cfg['kind']!r}")
        a.recon, a.target, a.grad, a.out = (self.recon.data_ptr(), self.x.data_ptr(), self.grad_recon.data_ptr(),
                                            self.out.data_ptr())
        a.sse, a.per_img = self.sse.data_ptr(), self.per_img.data_ptr()
        self._rl_ws = torch.zeros(max(1, L.recon_loss_workspace(a) // 4), dtype=torch.float32, device=self.net.device)
        a.workspace, a.workspace_bytes = self._rl_ws.data_ptr(), self._rl_ws.numel() * 4
        self._add(F, "vae_recon_loss", a)

    def _wide_head_fwd(self, F, cnt):
        """Head of a final layer wider than 32 channels: Conv2d(C -> 3 padded to 8, k3 s1 p1) on the
        conv-GEMM path with BatchNorm+LeakyReLU applied to its input on load, then vae_recon_fwd:
        tanh -> NCHW reconstruction, per-image SSE, and with the fused loss the backward seed
        dL/dy = 2(recon - x)(1 - recon^2) / (B*3*H*W) (the mean-MSE term of the ELBO)."""
        net, T, img, BS = self.net, self.net.dcode, self.net.img_size, self.B * self.S
        C = self.fin.shape[-1]
        a = L.ConvArgs(dtype=T, n=BS, h=img, w=img, c=C, k=8, p=img, q=img, r=3, stride=1, pad=1)
        a.x = self.fin.data_ptr()
        a.x_xf = self.bn_xf("final_layer.1", L.X_BN_ACT, cnt(self.fin), running=True)
        a.wt = self.w8h.data_ptr()
        a.bias = self.b8h.data_ptr()              # (channels 3..7 of y8 are never read)
        a.y = self.y8.data_ptr()
        self._add(F, "vae_conv2d_fwd", a)
        rc = L.ReconArgs(dtype=T, n=BS, h=img, w=img, c=3, ld=8)
        rc.y, rc.target, rc.recon, rc.sse = self.y8.data_ptr(), self.x.data_ptr(), self.recon.data_ptr(), self.sse.data_ptr()
        if self.fused_loss and self.training and self.recon_loss is None:
            rc.dy, rc.grad_scale = self.g8.data_ptr(), 1.0 / (self.B * 3 * img * img)
        self._add(F, "vae_recon_fwd", rc)

    def _wide_head_bwd(self, Bw, cnt):
        """Backward of _wide_head_fwd: [the seed from dL/drecon (drop-in)], data gradient into the final
        BatchNorm+LeakyReLU backward epilogue (its Σg, Σg·x̂), weight / bias gradient of the padded
        head, and the padded gradients' first 3 rows added into the parameter gradients."""
        net, T, img, BS = self.net, self.net.dcode, self.net.img_size, self.B * self.S
        C = self.fin.shape[-1]
        if self.seed_recon:
            rb = L.ReconArgs(dtype=T, n=BS, h=img, w=img, c=3, ld=8)
            rb.target, rb.recon = self.x.data_ptr(), self.recon.data_ptr()
            rb.dy, rb.grad_recon = self.g8.data_ptr(), self.grad_recon.data_ptr()
            self._add(Bw, "vae_recon_bwd", rb)
        a = L.ConvArgs(dtype=T, n=BS, h=img, w=img, c=C, k=8, p=img, q=img, r=3, stride=1, pad=1)
        a.dy = self.g8.data_ptr()
        a.wt = self.w8h.data_ptr()
        a.dx = self.g_fin.data_ptr()
        a.dx_epi = self.bn_xf("final_layer.1", L.X_BN_ACT, cnt(self.fin), aux=self.fin)
        self.bwd_sums(a, "final_layer.1")
        self._add(Bw, "vae_conv2d_bwd_data", a)
        f = L.ConvArgs(dtype=T, n=BS, h=img, w=img, c=C, k=8, p=img, q=img, r=3, stride=1, pad=1)
        f.dy = self.g8.data_ptr()
        f.x = self.fin.data_ptr()
        f.x_xf = self.bn_xf("final_layer.1", L.X_BN_ACT, cnt(self.fin))
        f.dw, f.db = self.dw8h.data_ptr(), self.db8h.data_ptr()
        self._add(Bw, "vae_conv2d_bwd_filter", f)
        Bw.append(("vae_unpad_accumulate", (1, 72 * C, 27 * C, self.dw8h.data_ptr(), self.g("final_layer.3.weight"))))
        Bw.append(("vae_unpad_accumulate", (1, 8, 3, self.db8h.data_ptr(), self.g("final_layer.3.bias"))))

    def use_device_eps(self, step: torch.Tensor, seed: int = 1265) -> bool:
        """Draw eps ~ N(0,1) on the device inside the forward, every step (the reference's
        torch.randn_like(std), vanilla_vae.py:116): vae_latent_dec_fwd runs Philox4x32-10 keyed by
        `seed` with the device step counter `step` (int32, advanced by vae_step_begin[_ex]) and writes
        the draw to self.eps for the backward.  Only the fused bf16 bottleneck (latent_fused) draws;
        returns False (eps stays an input) otherwise."""
        if not self.latent_fused:
            return False
        la = self._latent
        la.eps_gen, la.eps_step, la.eps_seed = 1, step.data_ptr(), seed & 0xFFFFFFFFFFFFFFFF
        self._eps_step = step                       # keep the counter alive with the plan
        return True

    # ------------------------------------------------------------------ execution
    def _run(self, calls, stream):
        run_calls(self, calls, stream)

    def begin(self, stream=None):
        stream = stream if stream is not None else L.stream_ptr()
        L.call("vae_step_begin", self.zero.data_ptr(), self.zero.numel() * 4, self.step.data_ptr(), stream)
        if self.loss_kind == L.LOSS_BETA_B:
            self.num_iter.add_(1.0)

    def forward(self, stream=None):
        self._run(self.fwd_calls, stream if stream is not None else L.stream_ptr())
        self._loss_pending = self.elbo_in_head

    def backward(self, stream=None):
        self._run(self.bwd_calls, stream if stream is not None else L.stream_ptr())
        self._loss_pending = False

    def encode(self, stream=None):
        """encoder + fc_mu|fc_var only (mu | log_var land in self.mulv)."""
        self._run(self.fwd_calls[:self.n_encode], stream if stream is not None else L.stream_ptr())

    def decode(self, stream=None):
        """decoder_input .. head from self.z (reconstruction lands in self.recon)."""
        self._run(self.fwd_calls[self.n_decode0:self.n_decode1], stream if stream is not None else L.stream_ptr())

    def loss_dict(self) -> Dict[str, float]:
        if self._loss_pending:
            raise RuntimeError("loss_dict(): this plan evaluates the ELBO in the head backward "
                               "(elbo_in_head); run backward() first")
        o = self.out.tolist()
        third = "KLD"
        return {"loss": o[0], "Reconstruction_Loss": o[1], third: o[2]}

    # ------------------------------------------------------------------ drop-in ELBO
    # A drop-in plan (fused_loss=False) can still take its loss on the GPU: the BaseVAE
    # loss_function of vae_amd.models runs vae_elbo_fwd on the forward's own buffers (run_elbo)
    # and seeds the backward from the kernel's coefficients (seed_fused) instead of autograd's
    # dL/drecon and dL/d[mu|log_var].
    LOSS_KINDS = {"vanilla": L.LOSS_VANILLA, "betaH": L.LOSS_BETA_H, "betaB": L.LOSS_BETA_B,
                  "iwae": L.LOSS_IWAE}

    def run_elbo(self, stream, loss: str, kld_weight: float, beta: float = 4.0, gamma: float = 1000.0,
                 c_max: float = 25.0, c_stop_iter: float = 1e5, num_iter: Optional[int] = None):
        """vae_elbo_fwd over this step's SSE and mu|log_var: out = [loss, Reconstruction_Loss, KLD
        as the reference reports it, raw KLD]; per_img; head_coef / kl_coef = dloss/dsse_i and the
        per-row KL gradient coefficient (the backward seeds)."""
        e = self.elbo_args
        e.kind = self.LOSS_KINDS[loss]
        if (e.kind == L.LOSS_IWAE) != (self.S > 1):
            raise ValueError(f"loss {loss!r} on a plan with {self.S} samples per image")
        e.kld_weight, e.beta, e.gamma, e.c_max, e.c_stop_iter = kld_weight, beta, gamma, c_max, c_stop_iter
        if num_iter is not None:
            self.num_iter.fill_(float(num_iter))
        L.call("vae_elbo_fwd", e, stream)

    def seed_fused(self, on: bool):
        """Backward seeding of a drop-in plan: on — from head_coef / kl_coef (run_elbo); off — from
        grad_recon and dmulv as written by autograd (the caller's own loss)."""
        if self.fused_loss or not self.training:
            return
        hb, rb = self._head_bwd, self._reparam_bwd
        if hb is None:               # wide head: its seed is vae_recon_bwd's, from grad_recon
            if on:                   # dL/drecon of the GPU ELBO: head_coef[n] * (recon - x)
                S = self.S
                torch.mul(self.head_coef.view(-1, 1, 1, 1),
                          self.recon - self.x.repeat_interleave(S, 0) if S > 1 else self.recon - self.x,
                          out=self.grad_recon)
                rb.kl_coef = self.kl_coef.data_ptr()
            else:
                rb.kl_coef = None
            return
        if on:
            hb.coef, hb.grad_recon = self.head_coef.data_ptr(), None
            rb.kl_coef = self.kl_coef.data_ptr()
        else:
            hb.coef, hb.grad_recon = None, self.grad_recon.data_ptr()
            rb.kl_coef = None

    def reset_backward(self):
        """Zero what the backward accumulates (gradients, BatchNorm-backward sums, d[mu|logvar],
        the padded head's dW) so the backward of the same forward can run again."""
        self.grads.zero_()
        for t in self.bnbwd.values():
            t.zero_()
        self.dmulv.zero_()
        if self.wide_head:
            self.dw8h.zero_()
            self.db8h.zero_()


BATCH_FN = "vae_conv_bwd_filter_batch"
DEFERRED_FNS = frozenset(("vae_conv2d_bwd_filter", "vae_convT2d_bwd_filter", "vae_unpad_accumulate"))


def batch_filter_calls(calls, ends, splits=(), enabled: bool = True):
    """Weight gradients are read only by the optimizer, so within a backward segment they can
    run after the segment's data-gradient chain and together: the conv / convT bwd_filter calls
    of each segment become one vae_conv_bwd_filter_batch call (grouped launches) at its end,
    followed by the calls that must follow them (vae_unpad_accumulate reads the padded first-layer
    weight gradient).  `splits`: raw call indices inside a segment where the weight gradients so
    far are emitted as a batch of their own that runs on the plan's side stream (run_calls).
    enabled=False: one call per layer, as built.  Returns (new call list, new segment ends)."""
    if not enabled:
        return list(calls), list(ends)
    out, new_ends, lo = [], [], 0

    def emit(deferred, side):
        wg = [(fn, ref) for fn, ref in deferred if fn != "vae_unpad_accumulate"]
        if len(wg) > 1 or (side and wg):
            b = L.FilterBatch(wg)
            b.side = side
            out.append((BATCH_FN, b))
            unpads = [(fn, ref) for fn, ref in deferred if fn == "vae_unpad_accumulate"]
            if side:
                # they read the batch's padded gradients: same (side) stream, right behind it
                b.after = unpads
            else:
                out.extend(unpads)
        else:
            out.extend(deferred)

    for end in ends:
        deferred = []
        for i in range(lo, end):
            if i in splits and deferred:
                emit(deferred, True)
                deferred = []
            fn, ref = calls[i]
            if fn in DEFERRED_FNS:
                deferred.append((fn, ref))
            else:
                out.append((fn, ref))
        emit(deferred, False)
        new_ends.append(len(out))
        lo = end
    return out, new_ends


def size_workspaces(plan, call_lists):
    """Give a plan's calls their workspace: each call's need is queried from the library
    (vaehip.h vae_*_workspace_size, which runs the call's own planning without launching), and
    the calls of the main chain share one buffer sized to the largest need, the weight-gradient
    calls of the side stream (run_calls) another — the two chains run concurrently.  A call
    whose need is 0 gets no workspace (the same plan).  Sets plan.workspace / plan.workspace_side
    and plan.workspace_need = {chain: bytes}."""
    dev = plan.net.device
    side_on = getattr(plan, "side", None) is not None
    need = {"main": 0, "side": 0}
    sized = []
    for calls in call_lists:
        for fn, ref in calls:
            if fn == BATCH_FN:
                arg = ref
                b = ref.workspace_size()
                deferred = any(getattr(a, "defer_reduce", 0) for a in ref.args)
            elif fn not in L.WS_QUERY:
                continue
            else:
                arg = ref._obj
                b = L.workspace_size(fn, arg)
                deferred = bool(getattr(arg, "defer_reduce", 0))
            on_side = (fn == BATCH_FN and getattr(ref, "side", False)) or (getattr(plan, "side_all", True) and fn in SIDE_FNS)
            chain = "side" if side_on and on_side else "main"
            if deferred and b > 0:
                # partial rows read later by the optimizer (vae_adam_step_ex): a buffer of its own
                chain = f"deferred{len(need)}"
                need[chain] = 0
            need[chain] = max(need[chain], b)
            sized.append((arg, b, chain))
    bufs = {c: torch.empty(max(1, (n + 3) // 4), dtype=torch.float32, device=dev) for c, n in need.items()}
    for arg, b, chain in sized:
        if b > 0:
            arg.workspace = bufs[chain].data_ptr()
            arg.workspace_bytes = bufs[chain].numel() * 4
        else:
            arg.workspace, arg.workspace_bytes = None, 0
    plan.workspace, plan.workspace_side, plan.workspace_need = bufs["main"], bufs["side"], need
    plan.workspace_deferred = [v for k, v in bufs.items() if k.startswith("deferred")]


SIDE_FNS = frozenset(("vae_conv2d_bwd_filter", "vae_convT2d_bwd_filter", "vae_linear_bwd_filter",
                      "vae_unpad_accumulate"))     # (follows its padded weight gradient)


def run_calls(plan, calls, stream):
    """Launch a call list on `stream`.  When the plan has a side stream (`plan.side`, and
    `stream` is the current torch stream), every weight-gradient call waits for the work queued
    on `stream` before it and runs on the side stream; the side stream is joined back into
    `stream` at the end of the list.  Recorded inside a HIP graph capture this becomes the
    graph's fork/join edges, so the replayed graph runs the two chains concurrently."""
    net = getattr(plan, "net", None)
    if getattr(net, "swaps_stale", False):
        # the swapped-axes weight copies trail the last optimizer step (a TrainStep refreshes them
        # inside its next step's head launch): bring them up to date before anything reads them
        net.refresh_swaps(stream)
    side = getattr(plan, "side", None)
    main = torch.cuda.current_stream() if side is not None else None
    if main is not None and main.cuda_stream != stream:
        side = None                          # an explicit foreign stream: keep everything on it
    forked = False
    for fn, arg in calls:
        on_side = (fn == BATCH_FN and getattr(arg, "side", False)) or (getattr(plan, "side_all", True) and fn in SIDE_FNS)
        if side is not None and on_side:
            side.wait_stream(main)
            call_one(fn, arg, side.cuda_stream)
            forked = True
        else:
            call_one(fn, arg, stream)
    if forked:
        main.wait_stream(side)


def call_one(fn, arg, stream):
    """One entry of a plan's call list (struct argument, scalar-argument tuple or a batch of
    weight-gradient calls) on `stream`."""
    if fn == BATCH_FN:
        arg(stream)
    elif isinstance(arg, tuple):
        L.call(fn, *arg, stream)
    else:
        L.call(fn, arg, stream)


def make_swaps(layout: Layout, params: torch.Tensor, names, device, out: Dict[str, int], lowp=None):
    """Descriptor array for vae_swap_axes over the named conv / convT weights (native
    [a][r][s][b] -> bf16 [b][r][s][a]) and the bf16 buffer holding the copies; `out` maps
    each name to its copy's device pointer.  lowp: the bf16 copy of `params` to read instead of
    the fp32 master (the same rounded values, half the bytes); it must be refreshed first."""
    specs = [layout.by_name[n] for n in names if n in layout.by_name]
    if len(specs) > L.SWAP_MAX:
        raise ValueError(f"{len(specs)} swapped weights > {L.SWAP_MAX} per vae_swap_axes launch")
    sizes = [(s.numel + 63) // 64 * 64 for s in specs]
    buf = torch.zeros(max(1, sum(sizes)), dtype=torch.bfloat16, device=device)
    descs = (L.SwapDesc * len(specs))()
    o = 0
    for i, (spec, n) in enumerate(zip(specs, sizes)):
        a, r, r2, b = spec.native_shape
        d = descs[i]
        if lowp is not None:
            d.src, d.src_dtype = lowp.data_ptr() + 2 * spec.offset, L.BF16
        else:
            d.src, d.src_dtype = params.data_ptr() + 4 * spec.offset, L.F32
        d.dst = buf.data_ptr() + 2 * o
        d.a, d.rs, d.b = a, r * r2, b
        out[spec.name] = d.dst
        o += n
    return descs, buf


def bn_reps(channels: int) -> int:
    """Replicas of a BatchNorm's statistics: enough that the ~1000 workgroups of a producing
    kernel do not all add into the same 2*C addresses, few enough (reps*C <= 256: one element per
    thread per statistic) that every consuming workgroup reduces them in one round of loads
    (vae_common.hpp tab_build) — thousands of consumer workgroups re-read them."""
    return max(1, min(32, 256 // max(1, channels)))


def _pad4(n: int) -> int:
    return (n + 3) // 4 * 4
