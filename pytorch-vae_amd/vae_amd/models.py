"""BaseVAE-compatible models on the MI355X kernels — the drop-in for the reference's
`models` package on the training hot path.

Mirrors the reference interface (paths relative to the reference root):
  BaseVAE                 models/base.py:5-28       encode/decode/sample/generate/forward/loss_function
  VanillaVAE              models/vanilla_vae.py:8-173
  BetaVAE                 models/beta_vae.py:8-179  (loss_type 'H' / 'B', per-instance num_iter)
  IWAE                    models/iwae.py:8-188      (num_samples; row-major b*S+s latent order)
  VQVAE                   models/vq_vae.py:73-219   (VectorQuantizer, residual stacks; vae_amd/vq.py)
  vae_models registry     models/__init__.py:35-56

`forward(x)` runs the HIP encoder/decoder (libvaehip.so) and returns the reference's list
([recons, input, mu, log_var], IWAE: [recons, input, mu, log_var, z, eps]).  `loss_function`
called on that list (what experiment.VAEXperiment.training_step does) runs the ELBO on the GPU
(vae_elbo_fwd, `_HipELBO`) and returns the reference's dict; its backward is the fused HIP
backward seeded by the kernel's coefficients — no dL/drecon tensor is materialised.  On any
other tensors (eval mode, a caller's own loss, no grad) it is the reference formula in torch and
`loss.backward()` reaches `_VAEStep.backward`, which seeds the same fused backward with autograd's
dL/drecon and dL/d[mu, log_var].  Optimizers see one flat nn.Parameter (`model.flat`);
`reference_state_dict()` / `load_reference_state_dict()` convert to the reference's keys and
layouts (vae_amd/layout.py).

model.train(): train-mode BatchNorm (batch statistics, running-stat update) and the fused HIP
backward; model.eval(): eval-mode BatchNorm from the running statistics, forward only
(validation_step, sample, generate).
"""
from __future__ import annotations

import math
from abc import abstractmethod
from typing import Any, Dict, List, Optional, Union

import torch
from torch import nn
from torch.nn import functional as F

from . import _lib as L
from .net import StepPlan, VAENet

Tensor = torch.Tensor


class BaseVAE(nn.Module):
    """models/base.py:5-28.

    state_dict() / load_state_dict() speak the reference's keys and PyTorch layouts (the one
    flat nn.Parameter the optimizers see is an implementation detail): a Lightning checkpoint of
    the experiment (`model.`-prefixed keys, run.py:80-84) has exactly the reference's entries,
    and a reference-trained checkpoint loads unchanged (checkpoint interop)."""

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        net = getattr(self, "net", None)
        if net is None:
            return super()._save_to_state_dict(destination, prefix, keep_vars)
        for k, v in self.reference_state_dict().items():
            destination[prefix + k] = v

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        net = getattr(self, "net", None)
        if net is None:
            return super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                                 unexpected_keys, error_msgs)
        expected = list(self._ref_keys()) if hasattr(self, "_ref_keys") else list(net.ref_order)
        mine = {k[len(prefix):]: v for k, v in state_dict.items() if k.startswith(prefix)}
        for k in expected:
            if k not in mine:
                missing_keys.append(prefix + k)
        for k in mine:
            if k not in expected and "." in k:
                unexpected_keys.append(prefix + k)
        if all(k in mine for k in expected):
            with torch.no_grad():
                self.load_reference_state_dict({k: mine[k] for k in expected})

    def __init__(self) -> None:
        super().__init__()

    def encode(self, input: Tensor) -> List[Tensor]:
        raise NotImplementedError

    def decode(self, input: Tensor) -> Any:
        raise NotImplementedError

    def sample(self, batch_size: int, current_device: int, **kwargs) -> Tensor:
        raise NotImplementedError

    def generate(self, x: Tensor, **kwargs) -> Tensor:
        raise NotImplementedError

    @abstractmethod
    def forward(self, *inputs: Tensor) -> Tensor:
        pass

    @abstractmethod
    def loss_function(self, *inputs: Any, **kwargs) -> Tensor:
        pass


class _VAEStep(torch.autograd.Function):
    """Forward of the HIP network; backward = the fused HIP backward of the whole network."""

    @staticmethod
    def forward(ctx, flat: Tensor, x: Tensor, eps: Tensor, model: "_HipVAE"):
        plan = model._plan(x.shape[0])
        st = L.stream_ptr()
        model.net.sync_lowp()                          # optimizer may have moved the fp32 master
        plan.x.copy_(x.detach().to(plan.x.dtype))
        plan.eps.copy_(eps.detach().reshape(plan.eps.shape))
        L.call("vae_step_begin", plan.zero.data_ptr(), plan.zero.numel() * 4, plan.step.data_ptr(), st)
        plan.forward(st)
        plan.backward_done = False
        model.net.num_batches_tracked += 1
        ctx.plan = plan
        ctx.set_materialize_grads(False)
        D = model.latent_dim
        recon = plan.recon.clone()
        mu = plan.mulv[:, :D].clone()
        log_var = plan.mulv[:, D:].clone()
        return recon, mu, log_var

    @staticmethod
    def backward(ctx, g_recon: Optional[Tensor], g_mu: Optional[Tensor], g_lv: Optional[Tensor]):
        plan = ctx.plan
        if g_recon is None and g_mu is None and g_lv is None:
            return None, None, None, None          # the loss came through _HipELBO (already done)
        if plan.backward_done:                     # a second backward of the same forward
            plan.reset_backward()
        plan.backward_done = True
        D = plan.net.latent_dim
        if g_recon is None:
            plan.grad_recon.zero_()
        else:
            plan.grad_recon.copy_(g_recon.reshape(plan.grad_recon.shape))
        dm = plan.dmulv.view(plan.B, 2 * D)
        dm[:, :D].copy_(g_mu if g_mu is not None else torch.zeros_like(dm[:, :D]))
        dm[:, D:].copy_(g_lv if g_lv is not None else torch.zeros_like(dm[:, D:]))
        plan.backward(L.stream_ptr())
        return plan.grads.clone(), None, None, None


class _HipELBO(torch.autograd.Function):
    """loss_function of a VanillaVAE-family model on its own forward's outputs, on the GPU:
    vae_elbo_fwd evaluates the reference's loss terms (vanilla_vae.py:124-146, beta_vae.py:129-152,
    iwae.py:129-160) from the per-image SSE the head kernel accumulated and mu|log_var, and writes
    the backward seeds; backward scales them by dL/dloss and runs the fused HIP backward from them,
    returning the flat parameter gradient (recons / mu / log_var get none, so `_VAEStep.backward`
    has nothing left to do)."""

    @staticmethod
    def forward(ctx, flat: Tensor, recons: Tensor, mu: Tensor, log_var: Tensor, plan, loss_kw: dict):
        plan.run_elbo(L.stream_ptr(), **loss_kw)
        ctx.plan = plan
        # the unscaled backward seeds of this loss (a repeated backward rescales from these)
        ctx.seeds = (plan.head_coef.clone(), plan.kl_coef.clone())
        loss, rl, kld = plan.out[0].clone(), plan.out[1].clone(), plan.out[2].clone()
        ctx.mark_non_differentiable(rl, kld)
        return loss, rl, kld

    @staticmethod
    def backward(ctx, g_loss: Optional[Tensor], g_rl, g_kld):
        plan = ctx.plan
        if g_loss is None:
            return None, None, None, None, None, None
        if plan.backward_done:
            plan.reset_backward()
        plan.backward_done = True
        torch.mul(ctx.seeds[0], g_loss, out=plan.head_coef)
        torch.mul(ctx.seeds[1], g_loss, out=plan.kl_coef)
        plan.seed_fused(True)
        try:
            plan.backward(L.stream_ptr())
        finally:
            plan.seed_fused(False)
        return plan.grads.clone(), None, None, None, None, None


class _HipReconLoss(torch.autograd.Function):
    """The Autoencoder's centre-weighted MSE / MS-SSIM on the GPU (vaehip.h vae_recon_loss): forward
    evaluates the loss and dL/drecons in one call; backward scales that seed by dL/dloss.  `cfg` is a
    StepPlan recon_loss dict."""

    @staticmethod
    def forward(ctx, recons: Tensor, target: Tensor, cfg: dict):
        n, c, h, w = recons.shape
        recons, target = recons.detach().float().contiguous(), target.detach().float().contiguous()
        if cfg["kind"] == "center":
            mask = cfg["mask"].to(recons.device, torch.float32).contiguous()
            a = L.recon_loss_args(L.RLOSS_CENTER, n, c, h, w, mask=mask)
        else:
            a = L.recon_loss_args(L.RLOSS_MSSIM, n, c, h, w, window=cfg["window"], levels=cfg.get("levels", 5),
                                  normalize=cfg.get("normalize", True))
        grad = torch.empty_like(recons)
        out = torch.zeros(3, dtype=torch.float32, device=recons.device)
        ws = torch.empty(max(1, L.recon_loss_workspace(a) // 4), dtype=torch.float32, device=recons.device)
        a.recon, a.target, a.grad, a.out = recons.data_ptr(), target.data_ptr(), grad.data_ptr(), out.data_ptr()
        a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel() * 4
        L.call("vae_recon_loss", a, L.stream_ptr())
        ctx.save_for_backward(grad)
        return out[0].clone()

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return grad * g, None, None


class _HipVAE(BaseVAE):
    """Shared machinery of the VanillaVAE-family models on libvaehip."""

    samples = 1

    def __init__(self, in_channels: int, latent_dim: int, hidden_dims: List = None, *,
                 dtype: torch.dtype = torch.float32, device=None, img_size: int = 64, seed: Optional[int] = None,
                 **kwargs) -> None:
        super().__init__()
        self.latent_dim = latent_dim
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        self.net = VAENet(in_channels=in_channels, latent_dim=latent_dim, hidden_dims=hidden_dims,
                          img_size=img_size, dtype=dtype, device=device, generator=gen)
        self.flat = nn.Parameter(self.net.params)      # shares storage with the kernels' buffer
        self._plans: Dict[int, StepPlan] = {}
        self._last = None                              # (plan, input, recon, mu, log_var) of forward

    def _loss_config(self) -> dict:
        """StepPlan loss arguments of this model's loss_function."""
        return dict(loss="iwae" if self.samples > 1 else "vanilla", samples=self.samples)

    def fused_train_step(self, batch: int, kld_weight: float, lr: float, weight_decay: float = 0.0,
                         betas=(0.9, 0.999), graph: bool = True, process_group=None, opt=None,
                         plan_options: Optional[dict] = None):
        """The whole training step of this model — forward, loss_function (vae_elbo_fwd), backward,
        [gradient all-reduce], Adam — as one engine.TrainStep on the model's own parameters,
        replayed from HIP graphs: the graph path of VAEXperiment.training_step + backward +
        optimizer.step (experiment.fit(..., engine="graph")).  `opt`: an engine.FusedAdam to share
        (one Adam state for the steps of every batch size, as the reference's single optimizer).
        `plan_options`: StepPlan route options (latent_kernels, head_kernels, pad_rgb, materialise,
        mat_min_flops, batch_wgrads, wg_overlap)."""
        from .engine import FusedAdam, TrainStep
        plan = StepPlan(self.net, batch, kld_weight=kld_weight, **self._loss_config(), **(plan_options or {}))
        if opt is None:
            opt = FusedAdam(self.net, lr=lr, betas=betas, weight_decay=weight_decay)
        return TrainStep(self.net, plan, opt, graph=graph, process_group=process_group)

    def _gpu_loss(self, args, loss: str, **kw):
        """The loss dict terms from vae_elbo_fwd when `args` are exactly what this model's last
        training forward returned (so its buffers hold them), else None (torch formula)."""
        last = self._last
        if last is None or not self.training or not torch.is_grad_enabled() or len(args) < 4:
            return None
        plan, inp, recon, mu, lv = last
        if args[0] is not recon or args[1] is not inp or args[2] is not mu or args[3] is not lv:
            return None
        return _HipELBO.apply(self.flat, recon, mu, lv, plan, dict(loss=loss, **kw))

    def _plan(self, batch: int, training: Optional[bool] = None) -> StepPlan:
        """Launch plan for a batch size: train-mode BatchNorm (batch statistics, running-stat
        update, backward) or, under model.eval(), eval-mode BatchNorm from the running statistics
        (forward only)."""
        training = self.training if training is None else training
        key = (batch, training)
        if key not in self._plans:
            self._plans[key] = StepPlan(self.net, batch, loss="iwae" if self.samples > 1 else "vanilla",
                                        samples=self.samples, fused_loss=False, training=training)
        return self._plans[key]

    def _eval_forward(self, input: Tensor, eps: Optional[Tensor]):
        """model.eval() forward (no autograd): encoder, reparameterization, decoder with running
        BatchNorm statistics (vanilla_vae.py:119-122 under eval())."""
        B = input.shape[0]
        if eps is None:
            eps = torch.randn(B * self.samples, self.latent_dim, device=input.device)
        plan = self._plan(B, False)
        st = L.stream_ptr()
        self.net.sync_lowp()
        plan.x.copy_(input.detach().to(plan.x.dtype))
        plan.eps.copy_(eps.detach().reshape(plan.eps.shape))
        L.call("vae_step_begin", plan.zero.data_ptr(), plan.zero.numel() * 4, plan.step.data_ptr(), st)
        plan._run(plan.fwd_calls[:plan.n_decode1], st)
        D = self.latent_dim
        return plan.recon.clone(), plan.mulv[:, :D].clone(), plan.mulv[:, D:].clone(), eps

    # ---- reference state dict interop (models/vanilla_vae.py parameter names and layouts)
    def reference_state_dict(self) -> Dict[str, Tensor]:
        return self.net.reference_state_dict()

    def load_reference_state_dict(self, sd: Dict[str, Tensor]):
        with torch.no_grad():
            self.net.load_reference_state_dict(sd)

    # ---- BaseVAE
    def reparameterize(self, mu: Tensor, logvar: Tensor) -> Tensor:
        """vanilla_vae.py:107-117 (torch ops; the fused path runs it on the GPU inside forward)."""
        std = torch.exp(0.5 * logvar)
        eps = torch.randn_like(std)
        return eps * std + mu

    def encode(self, input: Tensor) -> List[Tensor]:
        plan = self._plan(input.shape[0])
        st = L.stream_ptr()
        self.net.sync_lowp()
        plan.x.copy_(input.detach())
        L.call("vae_step_begin", plan.zero.data_ptr(), plan.zero.numel() * 4, plan.step.data_ptr(), st)
        plan.encode(st)
        D = self.latent_dim
        return [plan.mulv[:, :D].clone(), plan.mulv[:, D:].clone()]

    def decode(self, z: Tensor) -> Tensor:
        rows = z.reshape(-1, self.latent_dim).shape[0]
        plan = self._plan(rows // self.samples)
        st = L.stream_ptr()
        self.net.sync_lowp()
        plan.z.copy_(z.detach().reshape(plan.z.shape))
        L.call("vae_step_begin", plan.zero.data_ptr(), plan.zero.numel() * 4, plan.step.data_ptr(), st)
        plan.decode(st)
        return plan.recon.clone()

    def _remember(self, out):
        """Keep the identity of a training forward's outputs for _gpu_loss (eval: forget)."""
        if self.training and torch.is_grad_enabled() and out[0].grad_fn is not None:
            self._last = (self._plan(out[1].shape[0]), out[1], out[0], out[2], out[3])
        else:
            self._last = None

    def _run(self, input: Tensor, eps: Optional[Tensor] = None):
        if not self.training:
            return self._eval_forward(input, eps)
        B = input.shape[0]
        if eps is None:                                 # torch.randn_like(std), vanilla_vae.py:116
            eps = torch.randn(B * self.samples, self.latent_dim, device=input.device)
        return _VAEStep.apply(self.flat, input, eps, self) + (eps,)

    def sample(self, num_samples: int, current_device: int, **kwargs) -> Tensor:
        """vanilla_vae.py:148-161."""
        z = torch.randn(num_samples, self.latent_dim, device=current_device)
        return self.decode(z)

    def generate(self, x: Tensor, **kwargs) -> Tensor:
        """vanilla_vae.py:163-173."""
        return self.forward(x)[0]


class VanillaVAE(_HipVAE):
    """models/vanilla_vae.py:8-173 on libvaehip."""

    def forward(self, input: Tensor, **kwargs) -> List[Tensor]:
        recon, mu, log_var, _ = self._run(input, kwargs.get("eps"))
        out = [recon, input, mu, log_var]
        self._remember(out)
        return out

    def loss_function(self, *args, **kwargs) -> dict:
        """vanilla_vae.py:124-146."""
        kld_weight = kwargs['M_N']
        g = self._gpu_loss(args, "vanilla", kld_weight=kld_weight)
        if g is not None:
            return {'loss': g[0], 'Reconstruction_Loss': g[1], 'KLD': g[2]}
        recons, input, mu, log_var = args[0], args[1], args[2], args[3]
        recons_loss = F.mse_loss(recons, input)
        kld_loss = torch.mean(-0.5 * torch.sum(1 + log_var - mu ** 2 - log_var.exp(), dim=1), dim=0)
        loss = recons_loss + kld_weight * kld_loss
        return {'loss': loss, 'Reconstruction_Loss': recons_loss.detach(), 'KLD': -kld_loss.detach()}


class BetaVAE(_HipVAE):
    """models/beta_vae.py:8-179 on libvaehip."""

    num_iter = 0  # beta_vae.py:10 (class attribute, shared like the reference's)

    def __init__(self, in_channels: int, latent_dim: int, hidden_dims: List = None, beta: int = 4,
                 gamma: float = 1000., max_capacity: int = 25, Capacity_max_iter: int = 1e5, loss_type: str = 'B',
                 **kwargs) -> None:
        super().__init__(in_channels, latent_dim, hidden_dims, **kwargs)
        self.beta = beta
        self.gamma = gamma
        self.loss_type = loss_type
        self.C_max = torch.Tensor([max_capacity])
        self.C_stop_iter = Capacity_max_iter

    def forward(self, input: Tensor, **kwargs) -> List[Tensor]:
        recon, mu, log_var, _ = self._run(input, kwargs.get("eps"))
        out = [recon, input, mu, log_var]
        self._remember(out)
        return out

    def _loss_config(self) -> dict:
        if self.loss_type not in ('H', 'B'):
            raise ValueError('Undefined loss type.')
        return dict(loss="betaH" if self.loss_type == 'H' else "betaB", beta=float(self.beta), gamma=float(self.gamma),
                    max_capacity=float(self.C_max[0]), capacity_max_iter=float(self.C_stop_iter))

    def fused_train_step(self, *args, **kwargs):
        step = super().fused_train_step(*args, **kwargs)
        step.plan.num_iter.fill_(float(self.num_iter))       # the capacity schedule continues
        return step

    def loss_function(self, *args, **kwargs) -> dict:
        """beta_vae.py:129-152."""
        self.num_iter += 1
        kld_weight = kwargs['M_N']
        if self.loss_type in ('H', 'B'):
            g = self._gpu_loss(args, "betaH" if self.loss_type == 'H' else "betaB", kld_weight=kld_weight,
                               beta=float(self.beta), gamma=float(self.gamma), c_max=float(self.C_max[0]),
                               c_stop_iter=float(self.C_stop_iter), num_iter=self.num_iter)
            if g is not None:
                return {'loss': g[0], 'Reconstruction_Loss': g[1], 'KLD': g[2]}
        recons, input, mu, log_var = args[0], args[1], args[2], args[3]
        recons_loss = F.mse_loss(recons, input)
        kld_loss = torch.mean(-0.5 * torch.sum(1 + log_var - mu ** 2 - log_var.exp(), dim=1), dim=0)
        if self.loss_type == 'H':
            loss = recons_loss + self.beta * kld_weight * kld_loss
        elif self.loss_type == 'B':
            self.C_max = self.C_max.to(input.device)
            C = torch.clamp(self.C_max / self.C_stop_iter * self.num_iter, 0, self.C_max.data[0])
            loss = recons_loss + self.gamma * kld_weight * (kld_loss - C).abs()
        else:
            raise ValueError('Undefined loss type.')
        return {'loss': loss, 'Reconstruction_Loss': recons_loss, 'KLD': kld_loss}


class IWAE(_HipVAE):
    """models/iwae.py:8-188 on libvaehip (decoder batched at B*S; latents in row-major b*S+s
    order — the semantics of iwae.py:103 on torch < 1.5)."""

    def __init__(self, in_channels: int, latent_dim: int, hidden_dims: List = None, num_samples: int = 5,
                 **kwargs) -> None:
        self.samples = num_samples
        super().__init__(in_channels, latent_dim, hidden_dims, **kwargs)
        self.num_samples = num_samples

    def forward(self, input: Tensor, **kwargs) -> List[Tensor]:
        B, S, D = input.shape[0], self.num_samples, self.latent_dim
        recon, mu, log_var, eps = self._run(input, kwargs.get("eps"))
        mu_r = mu.repeat(S, 1, 1).permute(1, 0, 2)          # [B x S x D], iwae.py:123-124
        lv_r = log_var.repeat(S, 1, 1).permute(1, 0, 2)
        eps_r = eps.reshape(B, S, D)
        z = eps_r * torch.exp(0.5 * lv_r) + mu_r
        eps_ret = (z - mu_r) / lv_r                         # iwae.py:126 (returned, unused by the loss)
        out = [recon.view(B, S, *recon.shape[1:]), input, mu_r, lv_r, z, eps_ret]
        self._remember(out)
        return out

    def loss_function(self, *args, **kwargs) -> dict:
        """iwae.py:129-160."""
        g = self._gpu_loss(args, "iwae", kld_weight=kwargs['M_N'])
        if g is not None:
            return {'loss': g[0], 'Reconstruction_Loss': g[1], 'KLD': g[2]}
        recons, input, mu, log_var = args[0], args[1], args[2], args[3]
        input = input.repeat(self.num_samples, 1, 1, 1, 1).permute(1, 0, 2, 3, 4)
        kld_weight = kwargs['M_N']
        log_p_x_z = ((recons - input) ** 2).flatten(2).mean(-1)
        kld_loss = -0.5 * torch.sum(1 + log_var - mu ** 2 - log_var.exp(), dim=2)
        log_weight = (log_p_x_z + kld_weight * kld_loss)
        weight = F.softmax(log_weight, dim=-1)
        loss = torch.mean(torch.sum(weight * log_weight, dim=-1), dim=0)
        return {'loss': loss, 'Reconstruction_Loss': log_p_x_z.mean(), 'KLD': -kld_loss.mean()}


class MSSIM(nn.Module):
    """models/mssim_vae.py:182-282: the differentiable MS-SSIM loss 1 - Π cs_l^w_l · ssim_L^w_L over five
    levels (11x11 window, avg-pool 2x2 between levels, size_average, dynamic range 1, normalised
    (s+1)/2).  The window is built as the reference builds it — its Gaussian has a POSITIVE
    exponent, exp(+(x - 5)^2 / 4.5) (mssim_vae.py:205-209), an inverted bell the reference's
    trained models depend on, so it is kept."""

    WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)

    def __init__(self, in_channels: int = 3, window_size: int = 11, normalize: bool = True,
                 size_average: bool = True) -> None:
        super().__init__()
        self.in_channels, self.window_size = in_channels, window_size
        self.normalize, self.size_average = normalize, size_average
        k = torch.tensor([math.exp((i - window_size // 2) ** 2 / (2 * 1.5 ** 2)) for i in range(window_size)])
        k = k / k.sum()
        self.window_1d = k.tolist()             # the separable factor the HIP kernel takes (vae_recon_loss)
        k = k.unsqueeze(1)
        self._window = k.mm(k.t()).float().unsqueeze(0).unsqueeze(0).expand(
            in_channels, 1, window_size, window_size).contiguous()

    def ssim(self, img1: Tensor, img2: Tensor):
        """mssim_vae.py:217-250: (ssim, contrast sensitivity) at one level."""
        C, pad = self.in_channels, self.window_size // 2
        w = self._window.to(img1)
        mu1 = F.conv2d(img1, w, padding=pad, groups=C)
        mu2 = F.conv2d(img2, w, padding=pad, groups=C)
        mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
        sigma1_sq = F.conv2d(img1 * img1, w, padding=pad, groups=C) - mu1_sq
        sigma2_sq = F.conv2d(img2 * img2, w, padding=pad, groups=C) - mu2_sq
        sigma12 = F.conv2d(img1 * img2, w, padding=pad, groups=C) - mu1_mu2
        C1, C2 = 0.01 ** 2, 0.03 ** 2
        v1 = 2.0 * sigma12 + C2
        v2 = sigma1_sq + sigma2_sq + C2
        cs = torch.mean(v1 / v2)
        ssim_map = ((2 * mu1_mu2 + C1) * v1) / ((mu1_sq + mu2_sq + C1) * v2)
        ret = ssim_map.mean() if self.size_average else ssim_map.mean(1).mean(1).mean(1)
        return ret, cs

    def forward(self, img1: Tensor, img2: Tensor) -> Tensor:
        """mssim_vae.py:252-282."""
        weights = torch.tensor(self.WEIGHTS, device=img1.device)
        ms, mcs = [], []
        for _ in range(len(self.WEIGHTS)):
            sim, cs = self.ssim(img1, img2)
            ms.append(sim)
            mcs.append(cs)
            img1, img2 = F.avg_pool2d(img1, (2, 2)), F.avg_pool2d(img2, (2, 2))
        ms, mcs = torch.stack(ms), torch.stack(mcs)
        if self.normalize:
            ms, mcs = (ms + 1) / 2, (mcs + 1) / 2
        return 1 - torch.prod((mcs ** weights)[:-1] * (ms ** weights)[-1])


class Autoencoder(_HipVAE):
    """models/autoencoder.py:9-305 (the fork's main model) on libvaehip.

    The reference's network is the VanillaVAE stack with one `fc` (Linear 4C -> D, :50) and no
    reparameterization: z = fc(h), recons = decode(z).  Here it runs the VanillaVAE plan with the
    log-variance half of the fused fc_mu|fc_var GEMM pinned at zero and eps = 0, so
    z = mu + exp(0) * 0 = fc(h) exactly, the log-variance weights receive exactly zero gradient
    (dlogvar = dz * eps * std / 2 = 0) and stay zero under Adam, and `fc` is fc_mu.  The loss is
    the reference's: MSE on the GPU ELBO kernel (kind vanilla, M_N = 0 — no KL term), or the
    centre-weighted MSE (center_focus_sigma, :95-146) in torch on the HIP forward's output, whose
    autograd gradient seeds the fused HIP backward.  forward returns [recons, input, zeros, zeros]
    (the VGG-feature placeholders, :224-227); the dict adds KLD = 0 and feature_loss = 0.

    The MSSIM loss (use_mssim_loss, :32, :266-267) is the reference's MSSIM module restated in torch
    (class MSSIM below) on the HIP forward's reconstruction; its autograd gradient seeds the fused
    HIP backward, as the centre-weighted MSE's does.

    Not on this path (raise): the VGG feature loss (needs pretrained vgg19_bn weights, a network
    download) and hidden_dims other than five stride-2 layers (the stride-1 extra layers, :39; no
    reference config uses them).  Every width of the reference's configs runs, up to
    patient_vvbig_ae.yaml's [512, 1024, 2048, 4096, 4096]: the per-channel BatchNorm tables are sized
    by the real channel count in LDS (vae_launch.hpp lds budget)."""

    def __init__(self, in_channels: int, latent_dim: int, hidden_dims: List = None, use_vgg: bool = False,
                 center_focus_sigma: float = None, use_skip_connections: bool = False,
                 use_mssim_loss: bool = False, **kwargs) -> None:
        if use_vgg:
            raise NotImplementedError("Autoencoder(use_vgg=True) needs pretrained vgg19_bn weights (network "
                                      "download) — not on the MI355X path")
        hd = list(hidden_dims) if hidden_dims is not None else [32, 64, 128, 256, 512]
        if len(hd) != 5:
            raise NotImplementedError(f"Autoencoder with {len(hd)} layers (stride-1 extra layers, "
                                      "autoencoder.py:39) is not on the MI355X path; five stride-2 layers are")
        if max(hd) > 4096 or hd[0] > 512:
            raise NotImplementedError(f"Autoencoder hidden widths {hd}: the kernels take BatchNorm widths up to "
                                      "4096 and a final layer of up to 512 channels (every reference config)")
        super().__init__(in_channels, latent_dim, hd, **kwargs)
        self.center_focus_sigma = center_focus_sigma
        self.center_weight_mask = None
        self.mssim = MSSIM(in_channels) if use_mssim_loss else None
        # with five stride-2 layers no decoder output matches an encoder output's spatial size
        # (autoencoder.py:205-210 compares shapes), so the skip connections never fire
        self.use_skip_connections = use_skip_connections
        self.use_vgg = False
        self._zero_logvar()

    # ---- the fc_var half held at zero
    def _zero_logvar(self):
        lay = self.net.layout
        with torch.no_grad():
            for n in ("fc_var.weight", "fc_var.bias"):
                sp = lay.by_name[n]
                self.net.params[sp.offset:sp.offset + sp.numel].zero_()
        self.net.sync_lowp()

    def _ref_keys(self) -> List[str]:
        out = []
        for k in self.net.ref_order:
            if k in ("fc_mu.weight", "fc_mu.bias"):
                out.append("fc." + k.split(".")[1])
            elif not k.startswith("fc_var."):
                out.append(k)
        return out

    def reference_state_dict(self) -> Dict[str, Tensor]:
        sd = self.net.reference_state_dict()
        out = {}
        for k in self._ref_keys():
            src = "fc_mu." + k[3:] if k.startswith("fc.") else k
            out[k] = sd[src]
        return out

    def load_reference_state_dict(self, sd: Dict[str, Tensor]):
        full = dict(sd)
        for part in ("weight", "bias"):
            t = full.pop("fc." + part)
            full["fc_mu." + part] = t
            full["fc_var." + part] = torch.zeros_like(t)
        with torch.no_grad():
            self.net.load_reference_state_dict(full)

    def _recon_loss_cfg(self, device) -> Optional[dict]:
        """StepPlan / vae_recon_loss configuration of this model's reconstruction loss (None: MSE)."""
        if self.center_focus_sigma is not None:
            if self.center_weight_mask is None:
                self.center_weight_mask = self.create_center_weight_mask(self.net.img_size, self.net.img_size, device)
            return {"kind": "center", "mask": self.center_weight_mask.view(self.net.img_size, self.net.img_size)}
        if self.mssim is not None:
            if not (self.mssim.size_average and self.mssim.window_size <= 15):
                return None
            return {"kind": "mssim", "window": self.mssim.window_1d, "normalize": self.mssim.normalize}
        return None

    def _loss_config(self) -> dict:
        return dict(loss="vanilla", samples=1, recon_loss=self._recon_loss_cfg(self.net.device))

    def fused_train_step(self, batch: int, kld_weight: float, lr: float, weight_decay: float = 0.0,
                         betas=(0.9, 0.999), graph: bool = True, process_group=None, opt=None,
                         plan_options: Optional[dict] = None):
        """The whole Autoencoder step in one graph, whichever reconstruction loss the model has: the
        plain MSE on the ELBO kernel (M_N = 0), or the centre-weighted MSE / MS-SSIM on vae_recon_loss
        (loss terms, per-image MSE and the dL/drecon seed of the fused backward)."""
        step = super().fused_train_step(batch, 0.0, lr, weight_decay, betas, graph, process_group, opt,
                                        plan_options=plan_options)
        step.plan.eps.zero_()
        step.zero_eps = True
        return step

    # ---- BaseVAE
    def encode(self, input: Tensor) -> List[Tensor]:
        """autoencoder.py:147-163: [z]."""
        return [super().encode(input)[0]]

    def forward(self, input: Tensor, **kwargs) -> List[Tensor]:
        B = input.shape[0]
        recon, z, lv, _ = self._run(input, torch.zeros(B, self.latent_dim, device=input.device))
        zeros = torch.zeros(B, self.latent_dim, device=input.device)
        out = [recon, input, zeros, zeros.clone()]
        if self.training and torch.is_grad_enabled() and recon.grad_fn is not None:
            self._last = (self._plan(B), input, recon, z, lv)
        else:
            self._last = None
        return out

    def loss_function(self, *args, **kwargs) -> dict:
        """autoencoder.py:230-262."""
        recons, input = args[0], args[1]
        zero = torch.tensor(0.0, device=recons.device)
        last = self._last
        if (self.center_focus_sigma is None and self.mssim is None and last is not None and self.training
                and torch.is_grad_enabled() and recons is last[2] and input is last[1]):
            g = _HipELBO.apply(self.flat, last[2], last[3], last[4], last[0], dict(loss="vanilla", kld_weight=0.0))
            return {'loss': g[0], 'Reconstruction_Loss': g[1], 'KLD': zero, 'feature_loss': zero}
        cfg = (self._recon_loss_cfg(recons.device) if recons.is_cuda and recons.dim() == 4
               and recons.shape[2] * recons.shape[3] <= 4096 and recons.shape[2:] == input.shape[2:] else None)
        if cfg is not None and cfg["kind"] == "mssim":
            # the kernel's pyramid halves exactly (vaehip.h vae_recon_loss); other plane sizes (the
            # reference's avg_pool2d floors them, mssim_vae.py) take the torch MS-SSIM below
            step = 1 << (cfg.get("levels", 5) - 1)
            if recons.shape[2] % step or recons.shape[3] % step:
                cfg = None
        if cfg is not None and (cfg["kind"] != "center" or tuple(cfg["mask"].shape) == tuple(recons.shape[2:])):
            recons_loss = _HipReconLoss.apply(recons, input, cfg)  # vae_recon_loss (HIP forward + seed)
        elif self.center_focus_sigma is not None:
            if self.center_weight_mask is None:
                self.center_weight_mask = self.create_center_weight_mask(input.shape[2], input.shape[3], input.device)
            recons_loss = self.weighted_mse_loss(recons, input, self.center_weight_mask)
        elif self.mssim is not None:
            recons_loss = self.mssim(recons, input)               # autoencoder.py:266-267
        else:
            recons_loss = F.mse_loss(recons, input)
        return {'loss': recons_loss, 'Reconstruction_Loss': recons_loss, 'KLD': zero, 'feature_loss': zero}

    def create_center_weight_mask(self, height, width, device):
        """autoencoder.py:95-125."""
        y, x = torch.meshgrid(torch.arange(height, device=device).float(), torch.arange(width, device=device).float(),
                              indexing='ij')
        d2 = (y - (height - 1) / 2) ** 2 + (x - (width - 1) / 2) ** 2
        w = torch.exp(-d2 / (2 * self.center_focus_sigma ** 2))
        return (w * (height * width / w.sum())).unsqueeze(0).unsqueeze(0)

    @staticmethod
    def weighted_mse_loss(input, target, weight_mask):
        """autoencoder.py:127-145."""
        return ((input - target) ** 2 * weight_mask.expand(input.size(0), input.size(1), -1, -1)).mean()

    def sample(self, num_samples: int, current_device: int, **kwargs) -> Tensor:
        """autoencoder.py:264-279: z ~ U(-1, 1)."""
        z = torch.rand(num_samples, self.latent_dim, device=current_device) * 2 - 1
        return self.decode(z)


class _VQStep(torch.autograd.Function):
    """VQ-VAE forward on the HIP network; backward = the fused HIP backward seeded with
    dL/drecon and dL/dvq_loss (straight-through estimator inside, vq_vae.py:53)."""

    @staticmethod
    def forward(ctx, flat: Tensor, x: Tensor, model: "VQVAE"):
        plan = model._plan(x.shape[0])
        st = L.stream_ptr()
        model.net.sync_lowp()
        plan.x.copy_(x.detach().to(plan.x.dtype))
        L.call("vae_step_begin", plan.zero.data_ptr(), plan.zero.numel() * 4, plan.step.data_ptr(), st)
        plan.forward(st)
        ctx.plan = plan
        n = plan.q.numel()
        vq_loss = plan.vq_sse[0] * ((1.0 + plan.beta) / n)      # commitment*beta + embedding (:47-50)
        return plan.recon.clone(), vq_loss.clone()

    @staticmethod
    def backward(ctx, g_recon: Optional[Tensor], g_vq: Optional[Tensor]):
        plan = ctx.plan
        if g_recon is None:
            plan.grad_recon.zero_()
        else:
            plan.grad_recon.copy_(g_recon.reshape(plan.grad_recon.shape))
        if g_vq is None:
            plan.vq_grad.zero_()
        else:
            plan.vq_grad.copy_(g_vq.reshape(1))
        plan.backward(L.stream_ptr())
        return plan.grads.clone(), None, None


class VQVAE(BaseVAE):
    """models/vq_vae.py:73-219 on libvaehip (vae_amd/vq.py)."""

    def __init__(self, in_channels: int, embedding_dim: int, num_embeddings: int, hidden_dims: List = None,
                 beta: float = 0.25, img_size: int = 64, *, dtype: torch.dtype = torch.float32, device=None,
                 seed: Optional[int] = None, **kwargs) -> None:
        super().__init__()
        from .vq import VQNet
        self.embedding_dim = embedding_dim
        self.num_embeddings = num_embeddings
        self.img_size = img_size
        self.beta = beta
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        self.net = VQNet(in_channels, embedding_dim, num_embeddings, hidden_dims, img_size, dtype, device, gen)
        self.flat = nn.Parameter(self.net.params)
        self._plans: Dict[int, Any] = {}

    def _plan(self, batch: int):
        from .vq import VQStepPlan
        if batch not in self._plans:
            self._plans[batch] = VQStepPlan(self.net, batch, beta=self.beta, fused_loss=False)
        return self._plans[batch]

    def reference_state_dict(self) -> Dict[str, Tensor]:
        return self.net.reference_state_dict()

    def load_reference_state_dict(self, sd: Dict[str, Tensor]):
        with torch.no_grad():
            self.net.load_reference_state_dict(sd)

    def encode(self, input: Tensor) -> List[Tensor]:
        """vq_vae.py:168-176: the encoder output (after its final LeakyReLU), NCHW."""
        plan = self._plan(input.shape[0])
        st = L.stream_ptr()
        self.net.sync_lowp()
        plan.x.copy_(input.detach())
        plan.begin(st)
        plan._run(plan.fwd_calls[:plan.n_encode], st)
        return [F.leaky_relu(plan.latpre.float(), 0.01).permute(0, 3, 1, 2).contiguous()]

    def decode(self, z: Tensor) -> Tensor:
        """vq_vae.py:178-187: decoder on (quantized) latents [B x D x H x W]."""
        plan = self._plan(z.shape[0])
        st = L.stream_ptr()
        self.net.sync_lowp()
        plan.q.copy_(z.detach().permute(0, 2, 3, 1))
        plan.begin(st)
        plan._run(plan.fwd_calls[plan.n_decode0:plan.n_decode1], st)
        return plan.recon.clone()

    def forward(self, input: Tensor, **kwargs) -> List[Tensor]:
        recon, vq_loss = _VQStep.apply(self.flat, input, self)
        return [recon, input, vq_loss]

    def fused_train_step(self, batch: int, kld_weight: float, lr: float, weight_decay: float = 0.0,
                         betas=(0.9, 0.999), graph: bool = True, process_group=None, opt=None,
                         plan_options: Optional[dict] = None):
        """See _HipVAE.fused_train_step (the VQ-VAE loss ignores kld_weight, vq_vae.py:194-211)."""
        from .engine import FusedAdam, TrainStep
        from .vq import VQStepPlan
        plan = VQStepPlan(self.net, batch, beta=self.beta, **(plan_options or {}))
        if opt is None:
            opt = FusedAdam(self.net, lr=lr, betas=betas, weight_decay=weight_decay)
        return TrainStep(self.net, plan, opt, graph=graph, process_group=process_group)

    def loss_function(self, *args, **kwargs) -> dict:
        """vq_vae.py:194-211."""
        recons, input, vq_loss = args[0], args[1], args[2]
        recons_loss = F.mse_loss(recons, input)
        loss = recons_loss + vq_loss
        return {'loss': loss, 'Reconstruction_Loss': recons_loss, 'VQ_Loss': vq_loss}

    def sample(self, num_samples: int, current_device: Union[int, str], **kwargs) -> Tensor:
        raise Warning('VQVAE sampler is not implemented.')              # vq_vae.py:216

    def generate(self, x: Tensor, **kwargs) -> Tensor:
        return self.forward(x)[0]


# models/__init__.py:35-56: the families on the MI355X path; the others raise on use.
_ON_PATH = {'VanillaVAE': VanillaVAE, 'BetaVAE': BetaVAE, 'IWAE': IWAE, 'VQVAE': VQVAE, 'Autoencoder': Autoencoder}
_REFERENCE_NAMES = ['HVAE', 'LVAE', 'IWAE', 'SWAE', 'MIWAE', 'VQVAE', 'DFCVAE', 'DIPVAE', 'BetaVAE', 'InfoVAE',
                    'WAE_MMD', 'VampVAE', 'GammaVAE', 'MSSIMVAE', 'JointVAE', 'BetaTCVAE', 'FactorVAE',
                    'LogCoshVAE', 'VanillaVAE', 'ConditionalVAE', 'CategoricalVAE', 'Autoencoder']


def _not_on_path(name):
    def ctor(*args, **kwargs):
        raise NotImplementedError(f"{name} is not on the MI355X training path of this build "
                                  f"(VanillaVAE, BetaVAE, IWAE, VQVAE, Autoencoder are; DESIGN.md §7)")
    return ctor


vae_models = {name: _ON_PATH.get(name) or _not_on_path(name) for name in _REFERENCE_NAMES}
VAE = VanillaVAE      # models/__init__.py:29-33 aliases
GaussianVAE = VanillaVAE
CVAE = _not_on_path('ConditionalVAE')
GumbelVAE = _not_on_path('CategoricalVAE')
