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

import ctypes
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
        device tensors (detached); averaged over ranks when torch.distributed is initialised — all
        terms of the dict in ONE all-reduce (a stacked vector), not one collective per term."""
        keys = list(d)
        vals = [d[k].detach() if torch.is_tensor(d[k]) else torch.tensor(float(d[k])) for k in keys]
        if keys and torch.distributed.is_available() and torch.distributed.is_initialized():
            dev = vals[0].device
            vec = torch.stack([v.to(dev).float().reshape(()) for v in vals])
            torch.distributed.all_reduce(vec)
            vec /= torch.distributed.get_world_size()
            vals = list(vec.unbind(0))
        for k, v in zip(keys, vals):
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
    model's own parameters, model.fused_train_step), with the experiment's logging.

    One optimizer state, as the reference's single torch.optim.Adam: every batch size's step
    shares ONE FusedAdam, whose first / second moments are the torch optimizer's own exp_avg /
    exp_avg_sq tensors of the model's flat parameter (its `step` is kept in the torch state too),
    so a checkpoint's optimizer_states and a resumed run see the state the fused steps built.
    The torch optimizer's learning rate (its schedulers keep their semantics) is copied in before
    every step.

    No host synchronisation per step: the loss terms stay device tensors in experiment.logged;
    per-image MSE and the extreme-image candidates are kept on the device and handed to the data
    module / experiment.extreme_images by flush() (fit() calls it once per epoch)."""

    def __init__(self, experiment: VAEXperiment, optimizer):
        self.exp, self.opt = experiment, optimizer
        self.steps: Dict[int, Any] = {}
        p = experiment.params
        g = optimizer.param_groups[0]
        self.kw = dict(kld_weight=p['kld_weight'], lr=g['lr'], weight_decay=p.get('weight_decay', 0.0),
                       betas=g['betas'])
        self.fused = None
        self.nstep = 0
        self._per: List[Any] = []                    # (offset, batch) of each step in _per_buf
        self._names: List[Any] = []
        self._ext = None                             # device extreme-image state
        self._terms: Dict[str, Tensor] = {}
        self._img_shape = None
        self._lr = None

    def _shared_adam(self):
        from .engine import FusedAdam
        model = self.exp.model
        flat = model.flat
        g = self.opt.param_groups[0]
        if not any(q is flat for q in g['params']):
            raise ValueError("engine='graph' needs the optimizer over model.parameters() (the flat parameter)")
        st = self.opt.state[flat]
        if 'exp_avg' not in st:
            st['step'] = torch.tensor(0.0)
            st['exp_avg'] = torch.zeros_like(flat, memory_format=torch.preserve_format)
            st['exp_avg_sq'] = torch.zeros_like(flat, memory_format=torch.preserve_format)
        fused = FusedAdam(model.net, lr=g['lr'], betas=g['betas'], eps=g['eps'], weight_decay=g['weight_decay'],
                          m=st['exp_avg'].data, v=st['exp_avg_sq'].data)
        self.nstep = int(float(st['step']))
        fused.step.fill_(self.nstep)
        return fused

    def __call__(self, batch, batch_idx):
        imgs, labels, names = batch
        exp, model = self.exp, self.exp.model
        B = imgs.shape[0]
        step = self.steps.get(B)
        if step is None:
            if self.fused is None:
                self.fused = self._shared_adam()
            step = self.steps[B] = model.fused_train_step(B, opt=self.fused, **self.kw)
            # eps drawn inside the step on the device (Philox keyed by a seed from torch's generator,
            # so manual_seed still fixes the run) where the fused bottleneck can; else plan.eps below
            if hasattr(step.plan, "use_device_eps") and not getattr(step, "zero_eps", False):
                step.device_eps = step.plan.use_device_eps(self.fused.step, int(torch.randint(0, 2 ** 62, (1,))))
        lr = self.opt.param_groups[0]['lr']
        if lr != self._lr:                            # (a device scalar: written only on change)
            self.fused.set_lr(lr)
            self._lr = lr
        self._img_shape = tuple(imgs.shape[1:])
        exp.curr_device = imgs.device
        plan = step.plan
        if hasattr(plan, "eps") and not getattr(step, "zero_eps", False) and not getattr(step, "device_eps", False):
            plan.eps.normal_()                        # torch.randn_like(std), vanilla_vae.py:116
        step(imgs)
        self.nstep += 1
        self.opt.state[model.flat]['step'] = torch.tensor(float(self.nstep))
        if hasattr(model, "num_iter"):
            model.num_iter += 1                       # BetaVAE: the loss_function's counter
        self._record(step, imgs)
        exp.logged.update(self._terms)
        self._names.append(names)
        return exp.logged['loss']

    def _record(self, step, imgs):
        """The per-step bookkeeping of training_step on the device in ONE launch
        (vaehip.h vae_step_record): the logged loss terms, the per-image losses (experiment.py:58-62,
        kept for the data module until flush()) and the running extreme images (:65-84)."""
        from . import _lib as L
        plan = step.plan
        B = plan.x.shape[0]
        S = plan.recon.shape[0] // B
        dev = imgs.device
        if self._ext is None:
            ie = plan.x[0].numel()
            third = "VQ_Loss" if not hasattr(plan, "eps") else "KLD"
            self._terms_buf = torch.zeros(3, device=dev)
            self._terms = {'loss': self._terms_buf[0], 'Reconstruction_Loss': self._terms_buf[1],
                           third: self._terms_buf[2]}
            if getattr(step, "zero_eps", False):                                # Autoencoder
                z = torch.zeros((), device=dev)
                self._terms.update(KLD=z, feature_loss=z)
            self._ext = {'best': torch.tensor([float('-inf'), float('inf')], device=dev),
                         'at': torch.full((4,), -1, dtype=torch.int32, device=dev),
                         'img': torch.zeros(2, ie, device=dev), 'recon': torch.zeros(2, ie, device=dev)}
            self._per_buf = torch.zeros(1024 * 64, device=dev)              # grows in flush-sized chunks
            self._per_off = 0
        if self._per_off + B > self._per_buf.numel():                       # keep the epoch's records
            self._per_buf = torch.cat([self._per_buf, torch.zeros_like(self._per_buf)])
        e = self._ext
        out = plan.metrics if step.world > 1 else plan.out
        a = L.RecordArgs(batch=B, samples=S, img_elems=plan.x[0].numel(), nterms=3, step=len(self._names))
        a.src_terms, a.terms = out.data_ptr(), self._terms_buf.data_ptr()
        a.per_img, a.per = plan.per_img.data_ptr(), self._per_buf.data_ptr() + 4 * self._per_off
        a.img, a.recon = plan.x.data_ptr(), plan.recon.data_ptr()
        a.best, a.at = e['best'].data_ptr(), e['at'].data_ptr()
        a.hi_img, a.lo_img = e['img'][0].data_ptr(), e['img'][1].data_ptr()
        a.hi_recon, a.lo_recon = e['recon'][0].data_ptr(), e['recon'][1].data_ptr()
        L.call("vae_step_record", ctypes.byref(a), L.stream_ptr())
        self._per.append((self._per_off, B))
        self._per_off += B

    def flush(self):
        """Hand the epoch's device-side records to the host (one synchronisation): per-image
        losses to the data module (dataset.py:130-136), extreme images to the experiment."""
        exp = self.exp
        if self._per:
            per = self._per_buf[:self._per_off].cpu().tolist()
            if exp.datamodule is not None and hasattr(exp.datamodule, "record_img_losses"):
                for (o, b), names in zip(self._per, self._names):
                    exp.datamodule.record_img_losses(names, per[o:o + b])
        if self._ext is not None:
            e = self._ext
            best, at = e['best'].tolist(), e['at'].tolist()
            shape = self._img_shape
            for k, key in enumerate(('highest', 'lowest')):
                step_i, i = at[2 * k], at[2 * k + 1]
                if step_i < 0:
                    continue
                v = best[k]
                better = v > exp.extreme_images[key]['loss'] if key == 'highest' else v < exp.extreme_images[key]['loss']
                if better:
                    exp.extreme_images[key] = {'loss': v, 'img': e['img'][k].view(1, *shape).cpu(),
                                               'recon': e['recon'][k].view(1, *shape).cpu(),
                                               'name': self._names[step_i][i]}
            e['best'].copy_(torch.tensor([float('-inf'), float('inf')]))
            e['at'].fill_(-1)
        self._per, self._names, self._per_off = [], [], 0


def _fusable(model) -> bool:
    """Models whose whole step the fused engine computes: every model with fused_train_step — the
    Autoencoder's centre-weighted MSE and MS-SSIM included (vae_recon_loss inside the step), except
    an MS-SSIM configured outside the kernel's range (size_average=False, windows > 15)."""
    m = getattr(model, "mssim", None)
    return m is None or (m.size_average and m.window_size <= 15)


def _owns_flat(opt, model) -> bool:
    """A torch.optim.Adam with one parameter group holding model.flat (what GraphedSteps can share)."""
    flat = getattr(model, "flat", None)
    return (flat is not None and type(opt) is torch.optim.Adam and len(opt.param_groups) == 1
            and any(q is flat for q in opt.param_groups[0]["params"]))


def fit(experiment: VAEXperiment, train_batches, epochs: int = 1, val_batches=None,
        engine: str = "graph") -> List[Dict[str, float]]:
    """Minimal Trainer loop over an iterable of (imgs, labels, names) batches: the reference's
    Lightning fit() for one optimizer (zero_grad, training_step, backward, step, epoch-interval
    schedulers).  Returns the per-epoch mean of each logged term (host values, synced once per
    epoch).  engine="graph" (default): each training step is one GraphedSteps replay (models with
    fused_train_step; plain Adam on model.parameters()); models without it (or several optimizers)
    run the eager path.  engine="eager": training_step + loss.backward() + optimizer.step()."""
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
        # the fused step shares the torch optimizer's state: only a plain Adam over model.flat
        # (configure_optimizers' own); any other setup keeps the eager path instead of raising
        if (hasattr(experiment.model, "fused_train_step") and len(optims) == 1 and _fusable(experiment.model)
                and _owns_flat(optims[0], experiment.model)):
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
        if graphed is not None:
            graphed.flush()
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
