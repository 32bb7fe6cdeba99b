"""VQ-VAE on libvaehip: the reference's VQVAE (models/vq_vae.py:73-211) training step.

Network (hidden_dims default [128, 256], embedding_dim 64, num_embeddings 512, 64x64 images):
  encoder  Conv(k4,s2,p1)+LReLU per hidden dim (:95-102), Conv3x3+LReLU (:104-109),
           6 x ResidualLayer x + Conv1x1(ReLU(Conv3x3(x))) (:57-70, :111-112), LReLU (:113),
           Conv1x1 -> embedding_dim + LReLU (:115-121)
  vq_layer VectorQuantizer (:24-55): argmin over the codebook, straight-through estimator
  decoder  Conv3x3+LReLU (:128-135), 6 x ResidualLayer, LReLU, ConvT(k4,s2,p1)+LReLU per
           reversed hidden dim (:142-152), ConvT(k4,s2,p1) -> 3 + Tanh (:154-160)
  loss     mse(recon, x) + vq_loss (:194-211)

Same design as the VanillaVAE plan (net.py): NHWC activations stored before their activation
(every LeakyReLU / ReLU is applied by the consuming kernel on load, and its backward by the
producing kernel's epilogue); residual adds fused into the 1x1 conv epilogue forward and into
the 3x3 conv data-gradient epilogue backward; the VectorQuantizer, the Tanh output and the
loss are their own small kernels.  All convolutions are MFMA implicit GEMMs (vae_igemm.hpp).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import torch

from . import _lib as L
from .layout import Layout, default_init, vq_layout, vq_param_spec
from .net import MAT_MIN_FLOPS, SLOPE, _pad4, make_swaps, run_calls, size_workspaces

NRES = 6             # ResidualLayers per stack (vq_vae.py:111, :138)


class VQNet:
    """Parameters of the VQVAE on one device (flat fp32 master + bf16 GEMM copy)."""

    def __init__(self, in_channels: int = 3, embedding_dim: int = 64, num_embeddings: int = 512,
                 hidden_dims: Optional[List[int]] = None, img_size: int = 64, dtype: torch.dtype = torch.float32,
                 device=None, generator: Optional[torch.Generator] = None):
        if in_channels != 3:
            raise ValueError("the output layer reconstructs 3 channels (vq_vae.py:156); in_channels must be 3")
        self.in_channels = in_channels
        self.embedding_dim = embedding_dim
        self.num_embeddings = num_embeddings
        self.hidden_dims = list(hidden_dims or [128, 256])
        self.img_size = img_size
        if img_size % (2 ** len(self.hidden_dims)):
            raise ValueError("img_size must be divisible by 2**len(hidden_dims)")
        self.dtype = dtype
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.layout: Layout = vq_layout(in_channels, embedding_dim, num_embeddings, self.hidden_dims)
        self.ref_order = [n for n, _, _ in vq_param_spec(in_channels, embedding_dim, num_embeddings, self.hidden_dims)]
        cpu_p = torch.zeros(self.layout.total)
        default_init(self.layout, cpu_p, torch.zeros(0), generator)
        self.params = cpu_p.to(self.device)
        self.running = torch.zeros(1, dtype=torch.float32, device=self.device)   # no BatchNorm
        self.lowp = (torch.zeros(self.layout.total, dtype=torch.bfloat16, device=self.device)
                     if dtype == torch.bfloat16 else None)
        self.num_batches_tracked = 0
        self.wt_t: Dict[str, int] = {}
        self.swap_descs = None
        self.sync_lowp()

    @property
    def dcode(self) -> int:
        return L.dtype_code(self.dtype)

    def sync_lowp(self):
        if self.lowp is not None:
            L.call("vae_cast_bf16", self.params.numel(), self.params.data_ptr(), self.lowp.data_ptr(), L.stream_ptr())
            self.refresh_swaps()

    def ensure_swaps(self, names):
        """bf16 mode: swapped-axes copies (vaehip.h wt_t) of the named weights — the ones the bf16
        conv-GEMMs read transposed (every data gradient and transposed-conv forward) — refreshed
        with the bf16 copy (sync_lowp, FusedAdam.apply) in vae_swap_axes launches of SWAP_MAX
        weights, instead of one transposition per call per step."""
        if self.lowp is None:
            return
        new = sorted(set(names) - set(self.wt_t))
        if not new:
            return
        # copies already handed out stay where they are (plans built earlier point at them)
        chunks, bufs = list(self.swap_descs or ()), list(getattr(self, "lowp_t", ()))
        for i in range(0, len(new), L.SWAP_MAX):
            d, b = make_swaps(self.layout, self.params, new[i:i + L.SWAP_MAX], self.device, self.wt_t)
            chunks.append(d)
            bufs.append(b)
        self.swap_descs, self.lowp_t = chunks, bufs
        self.refresh_swaps()

    def refresh_swaps(self, stream=None):
        for d in self.swap_descs or ():
            L.call("vae_swap_axes", len(d), ctypes.byref(d), stream if stream is not None else L.stream_ptr())

    def name_of_lowp(self, ptr: int) -> Optional[str]:
        """Parameter name whose bf16 copy starts at device pointer `ptr` (None: not a bf16 weight)."""
        if self.lowp is None:
            return None
        off = (ptr - self.lowp.data_ptr()) // 2
        for s in self.layout.params:
            if s.offset == off:
                return s.name
        return None

    def load_reference_state_dict(self, sd: Dict[str, torch.Tensor]):
        self.layout.load_reference(self.params, self.running, {k: v.to(self.device) for k, v in sd.items()})
        self.sync_lowp()

    def reference_state_dict(self) -> Dict[str, torch.Tensor]:
        return self.layout.export_reference(self.params, None, 0, self.ref_order)

    def p(self, name: str) -> int:
        s = self.layout.by_name[name]
        return self.params.data_ptr() + 4 * s.offset

    def w(self, name: str) -> int:
        s = self.layout.by_name[name]
        if self.lowp is not None:
            return self.lowp.data_ptr() + 2 * s.offset
        return self.params.data_ptr() + 4 * s.offset


def _act(slope: float = SLOPE, aux: Optional[torch.Tensor] = None) -> L.Xform:
    xf = L.Xform(kind=L.X_ACT, channels=1, slope=slope)
    if aux is not None:
        xf.aux = aux.data_ptr()
    return xf


class VQStepPlan:
    """Buffers and prebuilt launches of one VQ-VAE training step for a fixed batch.

    grads land in `self.grads` (net.params layout); `zero` (grads, per-image SSE, the VQ SSE)
    is cleared by vae_step_begin.  fused_loss=False (the BaseVAE drop-in) seeds the backward
    from `grad_recon` (dL/drecon) and `vq_grad` (dL/dvq_loss) instead of the fixed loss."""

    loss_kind = L.LOSS_VQ

    def __init__(self, net: VQNet, batch: int, *, beta: float = 0.25, fused_loss: bool = True, concurrent: bool = False,
                 materialise: bool = True, mat_min_flops: float = MAT_MIN_FLOPS):
        # materialise=False: the large strided layers keep their LeakyReLU fused into the GEMM's
        # operand load instead of one vae_bn_apply pass (tests/test_gpu_routes.py)
        self.net, self.B, self.beta, self.fused_loss = net, batch, beta, fused_loss
        self.materialise, self.mat_min_flops = bool(materialise), float(mat_min_flops)
        dev, T = net.device, net.dtype
        h, E, img = net.hidden_dims, net.embedding_dim, net.img_size
        B = batch
        self._keep = []
        f32 = dict(dtype=torch.float32, device=dev)
        act = dict(dtype=T, device=dev)
        self.x = torch.zeros(B, 3, img, img, **f32)
        sp = img
        self.enc = []
        for c in h:
            sp //= 2
            self.enc.append(torch.empty(B, sp, sp, c, **act))
        self.s, C = sp, h[-1]
        self.lat_hw = sp
        m = (B, sp, sp, C)
        self.e_in = torch.empty(*m, **act)                          # encoder Conv3x3 output
        self.e_t = [torch.empty(*m, **act) for _ in range(NRES)]    # residual Conv3x3 outputs
        self.e_h = [torch.empty(*m, **act) for _ in range(NRES)]    # residual layer outputs
        self.latpre = torch.empty(B, sp, sp, E, **act)
        self.q = torch.empty(B, sp, sp, E, **act)
        self.indices = torch.zeros(B * sp * sp, dtype=torch.int64, device=dev)
        self.d_in = torch.empty(*m, **act)
        self.d_t = [torch.empty(*m, **act) for _ in range(NRES)]
        self.d_h = [torch.empty(*m, **act) for _ in range(NRES)]
        r = h[::-1]
        self.up = []
        s2 = sp
        for i in range(len(r) - 1):
            s2 *= 2
            self.up.append(torch.empty(B, s2, s2, r[i + 1], **act))
        # bf16: the 3-channel ends (image, output conv) carried as 8 zero-padded channels so every
        # GEMM operand stays on the packed path (vae_pad_channels / vae_unpad_accumulate)
        self.pad_rgb = T == torch.bfloat16
        self.cy = 8 if self.pad_rgb else 3
        r_ = h[::-1]
        if self.pad_rgb:
            self.x8 = torch.zeros(B, img, img, 8, **act)
            self.w8e = torch.zeros(h[0] * 16 * 8, **act)            # encoder.0 [Co][4][4][8]
            self.w8d = torch.zeros(r_[-1] * 16 * 8, **act)          # output ConvT [Ci][4][4][8]
            self.b8d = torch.zeros(8, **f32)
        self.y = torch.empty(B, img, img, self.cy, **act)           # pre-Tanh output
        self.recon = torch.empty(B, 3, img, img, **f32)
        self.grad_recon = None if fused_loss else torch.zeros(B, 3, img, img, **f32)
        self.vq_grad = torch.ones(1, **f32)
        self.out = torch.zeros(4, **f32)
        self.per_img = torch.zeros(B, **f32)
        self.num_iter = torch.zeros(1, **f32)
        # backward buffers
        self.g_y = torch.empty_like(self.y)
        self.g_up = [torch.empty_like(t) for t in self.up]
        # residual-stream gradients: a buffer per layer and stack (nothing is reused inside a
        # backward, so the weight gradients on the side stream never race the data gradients)
        self.g_h = {st: [torch.empty(*m, **act) for _ in range(NRES + 1)] for st in ("encoder", "decoder")}
        self.g_t = {st: [torch.empty(*m, **act) for _ in range(NRES)] for st in ("encoder", "decoder")}
        self.g_q = torch.empty_like(self.q)
        self.g_lat = torch.empty_like(self.latpre)
        self.g_enc = [torch.empty_like(t) for t in self.enc]
        nz = _pad4(net.layout.total) + 4 + _pad4(B) + 4
        self.zero = torch.zeros(nz, **f32)
        o = 0
        self.grads = self.zero[o:o + net.layout.total]; o += _pad4(net.layout.total)
        self.metrics = self.zero[o:o + 4]; o += 4                  # rank-averaged loss terms (engine.py)
        self.sse = self.zero[o:o + B]; o += _pad4(B)
        self.vq_sse = self.zero[o:o + 1]; o += 4
        self.step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.fwd_calls: List = []
        self.bwd_calls: List = []
        self._mat: Dict[int, torch.Tensor] = {}     # materialised lrelu(t) of large layers' inputs (by t)
        self.side = torch.cuda.Stream(device=dev) if concurrent else None     # weight gradients (run_calls)
        self._build()
        self._attach_swaps()
        size_workspaces(self, [self.fwd_calls, self.bwd_calls])

    def _attach_swaps(self):
        """Point every data gradient and transposed-conv forward at the net's swapped-axes weight
        copy (vaehip.h wt_t: read by the bf16 conv-GEMM as k-contiguous rows), so no call
        transposes its weights itself (one vae_swap_axes pass per SWAP_MAX weights per step)."""
        net = self.net
        if net.lowp is None:
            return
        use = []
        for fn, ref in self.fwd_calls + self.bwd_calls:
            if fn in ("vae_conv2d_bwd_data", "vae_convT2d_fwd") and not isinstance(ref, tuple):
                name = net.name_of_lowp(ref._obj.wt or 0)
                if name is not None:
                    use.append((ref._obj, name))
        net.ensure_swaps([n for _, n in use])
        for arg, name in use:
            arg.wt_t = net.wt_t[name]

    # ------------------------------------------------------------------ helpers
    def g(self, name: str) -> int:
        s = self.net.layout.by_name[name]
        return self.grads.data_ptr() + 4 * s.offset

    def _add(self, lst, fn, arg):
        self._keep.append(arg)
        lst.append((fn, ctypes.byref(arg)))

    def _conv(self, t_in, cin, cout, r, stride, pad, transposed=False):
        n, hh, ww = t_in.shape[0], t_in.shape[1], t_in.shape[2]
        if transposed:
            p = q = hh * stride
        else:
            p = q = (hh + 2 * pad - r) // stride + 1
        return L.ConvArgs(dtype=self.net.dcode, n=n, h=hh, w=ww, c=cin, k=cout, p=p, q=q, r=r, stride=stride, pad=pad)

    def _res_stack(self, pre: str, first_idx: int, x0: torch.Tensor, ts, hs):
        """Forward of the 6 ResidualLayers on input lrelu(x0): t_j = Conv3x3(h_j),
        h_{j+1} = h_j + Conv1x1(relu(t_j)) (vq_vae.py:57-70)."""
        F, net = self.fwd_calls, self.net
        C = x0.shape[3]
        for j in range(NRES):
            idx = first_idx + j
            hin, hin_xf = (x0, _act()) if j == 0 else (hs[j - 1], L.Xform())
            a = self._conv(hin, C, C, 3, 1, 1)
            a.x, a.x_xf = hin.data_ptr(), hin_xf
            a.wt = net.w(f"{pre}.{idx}.resblock.0.weight")
            a.y = ts[j].data_ptr()
            self._add(F, "vae_conv2d_fwd", a)
            b = self._conv(ts[j], C, C, 1, 1, 0)
            b.x, b.x_xf = ts[j].data_ptr(), _act(0.0)                       # ReLU(True), :66
            b.wt = net.w(f"{pre}.{idx}.resblock.2.weight")
            b.residual, b.residual_xf = hin.data_ptr(), (_act() if j == 0 else L.Xform())
            b.y = hs[j].data_ptr()
            self._add(F, "vae_conv2d_fwd", b)

    def _res_stack_bwd(self, pre: str, first_idx: int, x0: torch.Tensor, ts, hs) -> torch.Tensor:
        """Backward of the residual stack.  g_h[pre][NRES] holds dL/dh_6 on entry; returns the
        buffer holding dL/dx0 (the gradient w.r.t. the stored pre-activation x0)."""
        Bw, net = self.bwd_calls, self.net
        C = x0.shape[3]
        gh, gt_ = self.g_h[pre], self.g_t[pre]
        for j in reversed(range(NRES)):
            idx = first_idx + j
            dh, dnext, gt = gh[j + 1], gh[j], gt_[j]
            hin, hin_xf = (x0, _act()) if j == 0 else (hs[j - 1], L.Xform())
            # Conv1x1: dt = W1^T dh * relu'(t)
            a = self._conv(ts[j], C, C, 1, 1, 0)
            a.dy, a.wt = dh.data_ptr(), net.w(f"{pre}.{idx}.resblock.2.weight")
            a.dx, a.dx_epi = gt.data_ptr(), _act(0.0, ts[j])
            self._add(Bw, "vae_conv2d_bwd_data", a)
            f = self._conv(ts[j], C, C, 1, 1, 0)
            f.x, f.x_xf = ts[j].data_ptr(), _act(0.0)
            f.dy, f.dw = dh.data_ptr(), self.g(f"{pre}.{idx}.resblock.2.weight")
            self._add(Bw, "vae_conv2d_bwd_filter", f)
            # Conv3x3: dh_j = W3^T * dt + dh (skip connection) [* lrelu'(x0) for j == 0]
            a = self._conv(hin, C, C, 3, 1, 1)
            a.dy, a.wt = gt.data_ptr(), net.w(f"{pre}.{idx}.resblock.0.weight")
            a.dx, a.residual = dnext.data_ptr(), dh.data_ptr()
            if j == 0:
                a.dx_epi = _act(SLOPE, x0)
            self._add(Bw, "vae_conv2d_bwd_data", a)
            f = self._conv(hin, C, C, 3, 1, 1)
            f.x, f.x_xf = hin.data_ptr(), hin_xf
            f.dy, f.dw = gt.data_ptr(), self.g(f"{pre}.{idx}.resblock.0.weight")
            self._add(Bw, "vae_conv2d_bwd_filter", f)
        return gh[0]

    def _mat_lrelu(self, F, t: torch.Tensor) -> torch.Tensor:
        """lrelu(t) written once (vaehip.h vae_bn_apply, ACT) for a large strided layer, so its GEMM
        runs transform-free on the LDS-DMA pipeline (vae_bgemm.hip); its weight gradient reads the
        same tensor.  bf16 only (the fp32 parity mode keeps the fused transform)."""
        key = t.data_ptr()
        out = self._mat.get(key)
        if out is None:
            out = self._mat[key] = torch.empty_like(t)
            a = L.BnApplyArgs(dtype=self.net.dcode, rows=t.numel() // t.shape[-1], channels=t.shape[-1])
            a.x, a.out, a.xf = t.data_ptr(), out.data_ptr(), _act()
            self._add(F, "vae_bn_apply", a)
        return out

    def _mat_ok(self, flops: float) -> bool:
        return self.net.dtype == torch.bfloat16 and self.materialise and flops >= self.mat_min_flops

    # ------------------------------------------------------------------ plan
    def _build(self):
        net = self.net
        h, E, K = net.hidden_dims, net.embedding_dim, net.num_embeddings
        nh = len(h)
        B, img = self.B, net.img_size
        C = h[-1]
        F = self.fwd_calls
        T = net.dcode
        r = h[::-1]
        iup = 1 + NRES + 1
        wout = f"decoder.{iup + len(r) - 1}.0"                      # output ConvT (-> 3 channels)
        if self.pad_rgb:
            F.append(("vae_nchw_to_nhwc_pad", (T, B, 3, img, img, 8, self.x.data_ptr(), self.x8.data_ptr())))
            F.append(("vae_pad_channels", (T, h[0] * 16, 3, 8, net.w("encoder.0.0.weight"), self.w8e.data_ptr())))
            F.append(("vae_pad_channels", (T, r[-1] * 16, 3, 8, net.w(wout + ".weight"), self.w8d.data_ptr())))
            F.append(("vae_pad_channels", (L.F32, 1, 3, 8, net.p(wout + ".bias"), self.b8d.data_ptr())))
        # ---------------------------------------------------------------- encoder
        for i in range(nh):
            src = self.x if i == 0 else self.enc[i - 1]
            cin = 3 if i == 0 else h[i - 1]
            a = L.ConvArgs(dtype=net.dcode, n=B, h=src.shape[2], w=src.shape[3] if i == 0 else src.shape[2], c=cin,
                           k=h[i], p=self.enc[i].shape[1], q=self.enc[i].shape[2], r=4, stride=2, pad=1)
            if i == 0:
                a.h = a.w = img
                if self.pad_rgb:
                    a.c, a.x = 8, self.x8.data_ptr()
                else:
                    a.x_nchw_f32, a.x = 1, self.x.data_ptr()
            elif self._mat_ok(2.0 * B * a.p * a.q * h[i] * 16 * cin):
                a.x = self._mat_lrelu(F, src).data_ptr()
            else:
                a.x, a.x_xf = src.data_ptr(), _act()
            a.wt, a.bias = net.w(f"encoder.{i}.0.weight"), net.p(f"encoder.{i}.0.bias")
            if i == 0 and self.pad_rgb:
                a.wt = self.w8e.data_ptr()
            a.y = self.enc[i].data_ptr()
            self._add(F, "vae_conv2d_fwd", a)
        a = self._conv(self.enc[-1], C, C, 3, 1, 1)
        a.x, a.x_xf = self.enc[-1].data_ptr(), _act()
        a.wt, a.bias = net.w(f"encoder.{nh}.0.weight"), net.p(f"encoder.{nh}.0.bias")
        a.y = self.e_in.data_ptr()
        self._add(F, "vae_conv2d_fwd", a)
        self._res_stack("encoder", nh + 1, self.e_in, self.e_t, self.e_h)
        ilat = nh + 1 + NRES + 1
        a = self._conv(self.e_h[-1], C, E, 1, 1, 0)
        a.x, a.x_xf = self.e_h[-1].data_ptr(), _act()
        a.wt, a.bias = net.w(f"encoder.{ilat}.0.weight"), net.p(f"encoder.{ilat}.0.bias")
        a.y = self.latpre.data_ptr()
        self._add(F, "vae_conv2d_fwd", a)
        self.n_encode = len(F)
        # ---------------------------------------------------------------- vector quantizer
        v = L.VqArgs(dtype=net.dcode, rows=B * self.s * self.s, dim=E, codes=K, beta=self.beta)
        v.lat, v.lat_xf = self.latpre.data_ptr(), _act()
        v.codebook = net.p("vq_layer.embedding.weight")
        v.indices, v.q, v.sse = self.indices.data_ptr(), self.q.data_ptr(), self.vq_sse.data_ptr()
        v.dq, v.dlat = self.g_q.data_ptr(), self.g_lat.data_ptr()
        v.loss_grad = None if self.fused_loss else self.vq_grad.data_ptr()
        v.dcodebook = self.g("vq_layer.embedding.weight")
        self._add(F, "vae_vq_fwd", v)
        self.n_decode0 = len(F)
        # ---------------------------------------------------------------- decoder
        a = self._conv(self.q, E, C, 3, 1, 1)
        a.x = self.q.data_ptr()
        a.wt, a.bias = net.w("decoder.0.0.weight"), net.p("decoder.0.0.bias")
        a.y = self.d_in.data_ptr()
        self._add(F, "vae_conv2d_fwd", a)
        self._res_stack("decoder", 1, self.d_in, self.d_t, self.d_h)
        src = self.d_h[-1]
        for i in range(len(r)):
            last = i == len(r) - 1
            dst = self.y if last else self.up[i]
            cout = self.cy if last else r[i + 1]
            a = self._conv(src, r[i], cout, 4, 2, 1, transposed=True)
            a.x, a.x_xf = src.data_ptr(), _act()
            if not last and self._mat_ok(2.0 * B * src.shape[1] * src.shape[2] * r[i] * cout * 16):
                a.x, a.x_xf = self._mat_lrelu(F, src).data_ptr(), L.Xform()
            a.wt, a.bias = net.w(f"decoder.{iup + i}.0.weight"), net.p(f"decoder.{iup + i}.0.bias")
            if last and self.pad_rgb:
                a.wt, a.bias = self.w8d.data_ptr(), self.b8d.data_ptr()
            a.y = dst.data_ptr()
            if not (last and self.pad_rgb):
                self._add(F, "vae_convT2d_fwd", a)
            src = dst
        # ---------------------------------------------------------------- Tanh + SSE + loss
        rc = L.ReconArgs(dtype=net.dcode, n=B, h=img, w=img, c=3, ld=self.cy)
        rc.y, rc.target, rc.recon, rc.sse = self.y.data_ptr(), self.x.data_ptr(), self.recon.data_ptr(), self.sse.data_ptr()
        if self.fused_loss:
            rc.dy, rc.grad_scale = self.g_y.data_ptr(), 1.0 / (B * 3 * img * img)
        if self.pad_rgb:
            # the output ConvT(128 -> 3) and Tanh + reconstruction + SSE + seed as one call
            # (vaehip.h vae_convT2d_fwd_recon: an input-centric kernel, no pre-tanh tensor in HBM)
            self._keep += [a, rc]
            F.append(("vae_convT2d_fwd_recon", (ctypes.byref(a), ctypes.byref(rc))))
        else:
            self._add(F, "vae_recon_fwd", rc)
        self.n_decode1 = len(F)
        e = L.ElboArgs(kind=L.LOSS_VQ, batch=B, samples=1, latent=1, img_elems=3 * img * img,
                       vq_beta=self.beta, vq_elems=float(B * self.s * self.s * E))
        e.sse, e.out, e.per_img, e.vq_sse = self.sse.data_ptr(), self.out.data_ptr(), self.per_img.data_ptr(), self.vq_sse.data_ptr()
        if self.fused_loss:
            self._add(F, "vae_elbo_fwd", e)

        # ================================================================ backward
        Bw = self.bwd_calls
        if not self.fused_loss:
            rb = L.ReconArgs(dtype=net.dcode, n=B, h=img, w=img, c=3, ld=self.cy)
            rb.target, rb.recon = self.x.data_ptr(), self.recon.data_ptr()
            rb.dy, rb.grad_recon = self.g_y.data_ptr(), self.grad_recon.data_ptr()
            self._add(Bw, "vae_recon_bwd", rb)
        ups = [self.d_h[-1]] + self.up                      # inputs of the ConvTs
        gups = [self.g_h["decoder"][NRES]] + self.g_up     # their gradients (pre-activation)
        gouts = self.g_up + [self.g_y]
        for i in reversed(range(len(r))):
            last = i == len(r) - 1
            cout = self.cy if last else r[i + 1]
            xin = ups[i]
            name = f"decoder.{iup + i}.0"
            padded = last and self.pad_rgb
            a = self._conv(xin, r[i], cout, 4, 2, 1, transposed=True)
            a.dy, a.wt = gouts[i].data_ptr(), (self.w8d.data_ptr() if padded else net.w(name + ".weight"))
            a.dx, a.dx_epi = gups[i].data_ptr(), _act(SLOPE, xin)
            if padded:
                # the output ConvT's data, weight and bias gradients in one call (vae_convT2d_bwd: one
                # pass over dy and x on the RGB-end kernel), dW / db straight into the parameters'
                # own [128][4][4][3] / [3] (dw_inner = 3: no padded gradient, no unpad launches)
                a.x, a.x_xf = xin.data_ptr(), _act()
                a.dw, a.db, a.dw_inner = self.g(name + ".weight"), self.g(name + ".bias"), 3
                self._add(Bw, "vae_convT2d_bwd", a)
                continue
            self._add(Bw, "vae_convT2d_bwd_data", a)
            f = self._conv(xin, r[i], cout, 4, 2, 1, transposed=True)
            f.x, f.x_xf = xin.data_ptr(), _act()
            if xin.data_ptr() in self._mat:
                f.x, f.x_xf = self._mat[xin.data_ptr()].data_ptr(), L.Xform()
            f.dy, f.dw, f.db = gouts[i].data_ptr(), self.g(name + ".weight"), self.g(name + ".bias")
            self._add(Bw, "vae_convT2d_bwd_filter", f)
        g_din = self._res_stack_bwd("decoder", 1, self.d_in, self.d_t, self.d_h)
        a = self._conv(self.q, E, C, 3, 1, 1)
        a.dy, a.wt, a.dx = g_din.data_ptr(), net.w("decoder.0.0.weight"), self.g_q.data_ptr()
        self._add(Bw, "vae_conv2d_bwd_data", a)
        f = self._conv(self.q, E, C, 3, 1, 1)
        f.x, f.dy = self.q.data_ptr(), g_din.data_ptr()
        f.dw, f.db = self.g("decoder.0.0.weight"), self.g("decoder.0.0.bias")
        self._add(Bw, "vae_conv2d_bwd_filter", f)
        self._add(Bw, "vae_vq_bwd", v)
        # encoder: Conv1x1 -> latents, residual stack, Conv3x3, strided convs
        a = self._conv(self.e_h[-1], C, E, 1, 1, 0)
        a.dy, a.wt = self.g_lat.data_ptr(), net.w(f"encoder.{ilat}.0.weight")
        a.dx, a.dx_epi = self.g_h["encoder"][NRES].data_ptr(), _act(SLOPE, self.e_h[-1])
        self._add(Bw, "vae_conv2d_bwd_data", a)
        f = self._conv(self.e_h[-1], C, E, 1, 1, 0)
        f.x, f.x_xf = self.e_h[-1].data_ptr(), _act()
        f.dy, f.dw, f.db = self.g_lat.data_ptr(), self.g(f"encoder.{ilat}.0.weight"), self.g(f"encoder.{ilat}.0.bias")
        self._add(Bw, "vae_conv2d_bwd_filter", f)
        g_ein = self._res_stack_bwd("encoder", nh + 1, self.e_in, self.e_t, self.e_h)
        a = self._conv(self.enc[-1], C, C, 3, 1, 1)
        a.dy, a.wt = g_ein.data_ptr(), net.w(f"encoder.{nh}.0.weight")
        a.dx, a.dx_epi = self.g_enc[-1].data_ptr(), _act(SLOPE, self.enc[-1])
        self._add(Bw, "vae_conv2d_bwd_data", a)
        f = self._conv(self.enc[-1], C, C, 3, 1, 1)
        f.x, f.x_xf = self.enc[-1].data_ptr(), _act()
        f.dy, f.dw, f.db = g_ein.data_ptr(), self.g(f"encoder.{nh}.0.weight"), self.g(f"encoder.{nh}.0.bias")
        self._add(Bw, "vae_conv2d_bwd_filter", f)
        for i in reversed(range(nh)):
            cin = 3 if i == 0 else h[i - 1]
            hin = img if i == 0 else self.enc[i - 1].shape[1]
            mk = lambda: L.ConvArgs(dtype=net.dcode, n=B, h=hin, w=hin, c=cin, k=h[i], p=self.enc[i].shape[1],
                                    q=self.enc[i].shape[2], r=4, stride=2, pad=1)
            f = mk()
            if i == 0 and self.pad_rgb:
                f.c, f.x = 8, self.x8.data_ptr()
            elif i == 0:
                f.x_nchw_f32, f.x = 1, self.x.data_ptr()
            elif self.enc[i - 1].data_ptr() in self._mat:
                f.x = self._mat[self.enc[i - 1].data_ptr()].data_ptr()
            else:
                f.x, f.x_xf = self.enc[i - 1].data_ptr(), _act()
            f.dy, f.dw, f.db = self.g_enc[i].data_ptr(), self.g(f"encoder.{i}.0.weight"), self.g(f"encoder.{i}.0.bias")
            if i == 0 and self.pad_rgb:
                f.dw_inner = 3          # dW straight into [128][4][4][3] from the 8-channel image
            self._add(Bw, "vae_conv2d_bwd_filter", f)
            if i > 0:
                a = mk()
                a.dy, a.wt = self.g_enc[i].data_ptr(), net.w(f"encoder.{i}.0.weight")
                a.dx, a.dx_epi = self.g_enc[i - 1].data_ptr(), _act(SLOPE, self.enc[i - 1])
                self._add(Bw, "vae_conv2d_bwd_data", a)

    # ------------------------------------------------------------------ execution
    def _run(self, calls, stream):
        run_calls(self, calls, stream)

    def begin(self, stream=None):
        stream = stream if stream is not None else L.stream_ptr()
        L.call("vae_step_begin", self.zero.data_ptr(), self.zero.numel() * 4, self.step.data_ptr(), stream)

    def forward(self, stream=None):
        self._run(self.fwd_calls, stream if stream is not None else L.stream_ptr())

    def backward(self, stream=None):
        self._run(self.bwd_calls, stream if stream is not None else L.stream_ptr())

    def loss_dict(self) -> Dict[str, float]:
        o = self.out.tolist()
        return {"loss": o[0], "Reconstruction_Loss": o[1], "VQ_Loss": o[2]}
