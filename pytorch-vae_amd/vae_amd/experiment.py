"""VAEXperiment counterpart (experiment.py:16-391 of the reference) without PyTorch Lightning.

The reference drives the hot path through a LightningModule: `training_step` (experiment.py:45-86)
calls the model, its `loss_function` with M_N = kld_weight, logs every loss term with
`.item()` + sync_dist, records per-image MSE for the difficulty sampler and tracks the
extreme-loss images with 64 more `.item()` calls; `configure_optimizers` (:304-357) builds Adam
(lr, weight_decay) with ExponentialLR per epoch (or ReduceLROnPlateau when adaptive_lr).

Here the same methods take the same arguments and return the same values, but the step keeps
everything on the device: the loss terms are returned as tensors (`logged` holds them; the
caller decides when to synchronise), per-image losses move to the host in one copy, and the
extreme-image update is a single argmax/argmin.  Lightning (1.5.6 pinned by the reference,
absent here) is optional: `VAEXperiment` is a plain object whose hooks a Trainer-like loop —
or `fit()` below — calls.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional

import torch
import torch.nn.functional as F
from torch import optim

Tensor = torch.Tensor


class VAEXperiment:
    """experiment.py:16 VAEXperiment(vae_model, params) — params are the YAML `exp_params`."""

    def __init__(self, vae_model, params: dict) -> None:
        self.model = vae_model
        self.params = params
        self.curr_device = None
        self.hold_graph = bool(params.get('retain_first_backpass', False))
        self.test_output_size = (256, 256)
        self.datamodule = None                 # optional: .record_img_losses(names, losses)
        self.logged: Dict[str, Tensor] = {}
        self.reset_extreme_image_tracking()

    def forward(self, input: Tensor, **kwargs) -> List[Tensor]:
        return self.model(input, **kwargs)

    __call__ = forward

    def reset_extreme_image_tracking(self):
        """experiment.py:38-43."""
        self.extreme_images = {
            'highest': {'loss': float('-inf'), 'img': None, 'recon': None, 'name': None},
            'lowest': {'loss': float('inf'), 'img': None, 'recon': None, 'name': None},
        }

    def log_dict(self, d: Dict[str, Tensor]):
        """Lightning's log_dict(..., sync_dist=True) without the per-term host sync: values stay
        device tensors (detached); averaged over ranks when torch.distributed is initialised."""
        for k, v in d.items():
            v = v.detach() if torch.is_tensor(v) else torch.tensor(float(v))
            if torch.distributed.is_available() and torch.distributed.is_initialized():
                v = v.clone().float()
                torch.distributed.all_reduce(v)
                v /= torch.distributed.get_world_size()
            self.logged[k] = v

    @staticmethod
    def per_image_mse(recon: Tensor, input: Tensor) -> Tensor:
        """experiment.py:58-62: mse(recon, input, reduction='none').mean([1,2,3]).  IWAE's
        [B,S,C,H,W] reconstructions (where the reference's broadcast fails)
        are scored per image averaged over the samples."""
        if recon.dim() == 5:
            return ((recon - input.unsqueeze(1)) ** 2).mean(dim=[1, 2, 3, 4])
        return F.mse_loss(recon, input, reduction='none').mean(dim=[1, 2, 3])

    def training_step(self, batch, batch_idx, optimizer_idx=0):
        """experiment.py:45-86."""
        imgs, labels, img_names = batch
        self.curr_device = imgs.device
        results = self.forward(imgs, labels=labels)
        train_loss = self.model.loss_function(*results, M_N=self.params['kld_weight'],
                                              optimizer_idx=optimizer_idx, batch_idx=batch_idx)
        self.log_dict(train_loss)
        per_img = self.per_image_mse(results[0].detach(), results[1]).cpu()     # one host copy
        if self.datamodule is not None and hasattr(self.datamodule, "record_img_losses"):
            self.datamodule.record_img_losses(img_names, per_img)
        self._track_extremes(per_img, imgs, results[0], img_names)
        return train_loss['loss']

    def _track_extremes(self, per_img: Tensor, imgs: Tensor, recon: Tensor, names):
        """experiment.py:65-84 with one argmax / argmin instead of a per-image loop (the first
        index wins ties, as the reference's strict comparisons do)."""
        if per_img.numel() == 0:
            return
        hi, lo = int(torch.argmax(per_img)), int(torch.argmin(per_img))
        for key, i, better in (('highest', hi, lambda a, b: a > b), ('lowest', lo, lambda a, b: a < b)):
            v = float(per_img[i])
            if better(v, self.extreme_images[key]['loss']):
                self.extreme_images[key] = {'loss': v, 'img': imgs[i:i + 1].detach().cpu(),
                                            'recon': recon[i:i + 1].detach().cpu(), 'name': names[i]}

    def validation_step(self, batch, batch_idx, optimizer_idx=0):
        """experiment.py:122-132.  Lightning calls it with the model in eval mode (BatchNorm on the
        running statistics, nothing updated); fit() below does the same."""
        imgs, labels, _ = batch
        self.curr_device = imgs.device
        with torch.no_grad():
            results = self.forward(imgs, labels=labels)
            val_loss = self.model.loss_function(*results, M_N=self.params['kld_weight'],
                                                optimizer_idx=optimizer_idx, batch_idx=batch_idx)
        self.log_dict({f"val_{k}": v for k, v in val_loss.items()})
        return val_loss

    # ------------------------------------------------------------------ test
    def test_step(self, batch, batch_idx):
        """experiment.py:155-217: the batch's loss terms (logged as test_*), then for every image
        the loss of that image alone (x1000, with running min/max in loss_stats) and the original
        and reconstruction resized to 256x256 (bilinear, align_corners=False) into test_data.

        The reference runs one extra forward per image at batch 1.  Under model.eval() BatchNorm
        uses the running statistics, so an image's outputs do not depend on the rest of its batch:
        here one batched forward serves all images and each image's loss is loss_function on its
        slice of the outputs (the same formula on the same values).  VQ-VAE's vq_loss is a batch
        scalar in the forward's outputs, so it keeps the per-image forwards."""
        imgs, labels, img_names = batch
        self.curr_device = imgs.device
        if not hasattr(self, 'test_data'):
            self.test_data = []
            self.loss_stats = {k: {'min': float('inf'), 'max': float('-inf')}
                               for k in ('total_loss', 'recon_loss', 'feature_loss')}
        kw = dict(M_N=self.params['kld_weight'], optimizer_idx=0, batch_idx=batch_idx)
        B = imgs.shape[0]
        with torch.no_grad():
            results = self.forward(imgs, labels=labels)
            test_loss = self.model.loss_function(*results, **kw)
            self.log_dict({f"test_{k}": v for k, v in test_loss.items()})
            sliceable = all(torch.is_tensor(r) and r.dim() > 0 and r.shape[0] == B for r in results)
            for i in range(B):
                if sliceable:
                    single_results = [r[i:i + 1] for r in results]
                else:
                    single_results = self.forward(imgs[i:i + 1], labels=labels[i:i + 1] if labels is not None else None)
                single_loss = self.model.loss_function(*single_results, **kw)
                recons = self.ensure_4_dims(single_results[0])
                total = float(single_loss['loss']) * 1000
                recon = float(single_loss['Reconstruction_Loss']) * 1000
                feat = float(single_loss['feature_loss']) * 1000 if 'feature_loss' in single_loss else None
                for key, v in (('total_loss', total), ('recon_loss', recon), ('feature_loss', feat)):
                    if v is not None:
                        st = self.loss_stats[key]
                        st['min'], st['max'] = min(st['min'], v), max(st['max'], v)
                orig = F.interpolate(imgs[i:i + 1], size=self.test_output_size, mode='bilinear', align_corners=False)
                rec = F.interpolate(recons, size=self.test_output_size, mode='bilinear', align_corners=False)
                self.test_data.append({'name': img_names[i], 'original': orig.cpu(), 'reconstruction': rec.cpu(),
                                       'total_loss': total, 'recon_loss': recon, 'feature_loss': feat})
        return test_loss

    def normalize_loss(self, loss_value, loss_type):
        """experiment.py:359-374: the fraction of test images whose loss is <= loss_value."""
        key = {'total_loss': 'total_loss', 'recon_loss': 'recon_loss', 'feature_loss': 'feature_loss'}[loss_type]
        vals = [d[key] for d in self.test_data if d[key] is not None]
        return sum(1 for x in vals if x <= loss_value) / len(vals)

    def ensure_4_dims(self, t: Tensor) -> Tensor:
        """experiment.py:376-392: [B,S,C,H,W] -> the first sample; [B,_,S,C,H,W] -> [:, 0, 0]."""
        if t.dim() == 6:
            return t[:, 0, 0]
        if t.dim() == 5:
            return t[:, 0]
        if t.dim() == 3:
            return t.unsqueeze(0)
        return t

    def configure_optimizers(self):
        """experiment.py:304-357: Adam(lr, weight_decay); ReduceLROnPlateau on val_loss when
        adaptive_lr, else ExponentialLR(scheduler_gamma) stepped per epoch; a second optimizer
        for `submodel` when LR_2 is set."""
        p = self.params
        optims, scheds = [], []
        optimizer = optim.Adam(self.model.parameters(), lr=p['LR'], weight_decay=p['weight_decay'])
        optims.append(optimizer)
        if p.get('LR_2') is not None and p.get('submodel'):
            optims.append(optim.Adam(getattr(self.model, p['submodel']).parameters(), lr=p['LR_2']))
        if p.get('adaptive_lr'):
            scheduler = optim.lr_scheduler.ReduceLROnPlateau(optimizer, mode='min', factor=0.5, patience=5,
                                                             threshold=0.00003, threshold_mode='abs', min_lr=1e-7)
            return {"optimizer": optimizer,
                    "lr_scheduler": {"scheduler": scheduler, "monitor": "val_loss", "interval": "epoch",
                                     "frequency": 1}}
        if p.get('scheduler_gamma') is not None:
            scheds.append({"scheduler": optim.lr_scheduler.ExponentialLR(optims[0], gamma=p['scheduler_gamma']),
                           "interval": "epoch"})
            if p.get('scheduler_gamma_2') is not None and len(optims) > 1:
                scheds.append({"scheduler": optim.lr_scheduler.ExponentialLR(optims[1], gamma=p['scheduler_gamma_2']),
                               "interval": "epoch"})
            return optims, scheds
        return optims


class GraphedSteps:
    """The graph path of VAEXperiment.training_step + loss.backward() + optimizer.step(): one
    engine.TrainStep per batch size (HIP graphs of forward, vae_elbo_fwd, backward, Adam on the
    model's own parameters, model.fused_train_step), with the experiment's logging — the loss
    terms as device tensors in experiment.logged, per-image MSE to the data module and the
    extreme-image tracking — and the torch optimizer's learning rate (so its schedulers keep
    their semantics) copied into the fused Adam before every step."""

    def __init__(self, experiment: VAEXperiment, optimizer):
        self.exp, self.opt = experiment, optimizer
        self.steps: Dict[int, Any] = {}
        p = experiment.params
        self.kw = dict(kld_weight=p['kld_weight'], lr=optimizer.param_groups[0]['lr'],
                       weight_decay=p.get('weight_decay', 0.0), betas=optimizer.param_groups[0]['betas'])

    def __call__(self, batch, batch_idx):
        imgs, labels, names = batch
        exp, model = self.exp, self.exp.model
        B = imgs.shape[0]
        step = self.steps.get(B)
        if step is None:
            step = self.steps[B] = model.fused_train_step(B, **self.kw)
        step.opt.set_lr(self.opt.param_groups[0]['lr'])
        exp.curr_device = imgs.device
        plan = step.plan
        eps = None
        if hasattr(plan, "eps"):
            eps = (torch.zeros(plan.eps.shape, device=imgs.device) if getattr(step, "zero_eps", False)
                   else torch.randn(plan.eps.shape, device=imgs.device))
        step(imgs, eps)
        if hasattr(model, "num_iter"):
            model.num_iter += 1                       # BetaVAE: the loss_function's counter
        out = plan.out
        third = "VQ_Loss" if not hasattr(plan, "eps") else "KLD"
        terms = {'loss': out[0], 'Reconstruction_Loss': out[1], third: out[2]}
        if getattr(step, "zero_eps", False):                  # Autoencoder: no KL, no feature loss
            terms.update(KLD=torch.zeros_like(out[2]), feature_loss=torch.zeros_like(out[2]))
        exp.log_dict(terms)
        per = plan.per_img.view(B, -1).mean(dim=1).cpu()
        if exp.datamodule is not None and hasattr(exp.datamodule, "record_img_losses"):
            exp.datamodule.record_img_losses(names, per)
        recon = plan.recon.view(B, -1, *plan.recon.shape[1:])[:, 0]
        exp._track_extremes(per, imgs, recon, names)
        return exp.logged['loss']


def fit(experiment: VAEXperiment, train_batches, epochs: int = 1, val_batches=None,
        engine: str = "eager") -> List[Dict[str, float]]:
    """Minimal Trainer loop over an iterable of (imgs, labels, names) batches: the reference's
    Lightning fit() for one optimizer (zero_grad, training_step, backward, step, epoch-interval
    schedulers).  Returns the per-epoch mean of each logged term (host values, synced once per
    epoch).  engine="graph": each training step is one GraphedSteps replay (models with
    fused_train_step; plain Adam on model.parameters())."""
    opt_cfg = experiment.configure_optimizers()
    sched, plateau = [], None
    if isinstance(opt_cfg, dict):
        optims = [opt_cfg["optimizer"]]
        plateau = opt_cfg["lr_scheduler"]["scheduler"]
    elif isinstance(opt_cfg, tuple):
        optims, sched = opt_cfg
    else:
        optims = opt_cfg
    graphed = None
    if engine == "graph":
        if not hasattr(experiment.model, "fused_train_step") or len(optims) != 1:
            raise ValueError("engine='graph' needs a vae_amd model and a single optimizer")
        graphed = GraphedSteps(experiment, optims[0])
    elif engine != "eager":
        raise ValueError(f"engine {engine!r}")
    history = []
    for _ in range(epochs):
        sums: Dict[str, Tensor] = {}
        cnt: Dict[str, int] = {}

        def acc():
            for k, v in experiment.logged.items():
                sums[k] = sums.get(k, 0) + v.float()
                cnt[k] = cnt.get(k, 0) + 1
        for i, batch in enumerate(train_batches):
            if graphed is not None:
                graphed(batch, i)
                acc()
                continue
            for o in optims:
                o.zero_grad(set_to_none=True)
            loss = experiment.training_step(batch, i)
            loss.backward()
            optims[0].step()
            acc()
        if val_batches is not None:
            was_training = getattr(experiment.model, "training", True)
            if hasattr(experiment.model, "eval"):
                experiment.model.eval()            # Lightning's validation loop: model.eval()
            try:
                for i, batch in enumerate(val_batches):
                    experiment.validation_step(batch, i)
                    acc()
            finally:
                if was_training and hasattr(experiment.model, "train"):
                    experiment.model.train()
        rec = {k: float(v) / cnt[k] for k, v in sums.items()}
        for s in sched:
            s["scheduler"].step()
        if plateau is not None and "val_loss" in rec and math.isfinite(rec["val_loss"]):
            plateau.step(rec["val_loss"])
        experiment.reset_extreme_image_tracking()
        history.append(rec)
    return history
