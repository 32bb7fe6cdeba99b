"""VAEXperiment counterpart (vae_amd/experiment.py) on CPU with a stand-in model that follows the
BaseVAE contract (forward -> [recons, input, ...], loss_function(*results, M_N=...) -> dict):
training_step / validation_step / configure_optimizers / fit semantics of experiment.py."""
import torch
import torch.nn.functional as F
from torch import nn

from vae_amd.experiment import VAEXperiment, fit


class TinyAE(nn.Module):
    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(0)
        self.enc = nn.Linear(3 * 8 * 8, 16)
        self.dec = nn.Linear(16, 3 * 8 * 8)
        with torch.no_grad():
            for p in self.parameters():
                p.copy_(torch.randn(p.shape, generator=g) * 0.05)

    def forward(self, x, **kwargs):
        h = self.enc(x.flatten(1))
        return [torch.tanh(self.dec(h)).view_as(x), x, h]

    def loss_function(self, *args, **kwargs):
        recons, x, h = args
        r = F.mse_loss(recons, x)
        k = (h ** 2).mean()
        loss = r + kwargs['M_N'] * k
        return {'loss': loss, 'Reconstruction_Loss': r.detach(), 'KLD': -k.detach()}


class Recorder:
    def __init__(self):
        self.calls = []

    def record_img_losses(self, names, losses):
        self.calls.append((list(names), losses.clone()))


def _batch(seed, B=6):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(B, 3, 8, 8, generator=g), torch.zeros(B, dtype=torch.float64), [f"img{seed}_{i}.png" for i in range(B)]


PARAMS = {'LR': 0.005, 'weight_decay': 0.0, 'scheduler_gamma': 0.95, 'kld_weight': 0.5, 'manual_seed': 1265}


def test_training_step_matches_reference_semantics():
    m = TinyAE()
    exp = VAEXperiment(m, dict(PARAMS))
    rec = Recorder()
    exp.datamodule = rec
    batch = _batch(1)
    loss = exp.training_step(batch, 0)
    res = m(batch[0])
    want = m.loss_function(*res, M_N=0.5)
    assert torch.allclose(loss, want['loss'])
    assert set(exp.logged) == {'loss', 'Reconstruction_Loss', 'KLD'}
    per_img = F.mse_loss(res[0], batch[0], reduction='none').mean(dim=[1, 2, 3]).detach()
    names, got = rec.calls[0]
    assert names == batch[2] and torch.allclose(got, per_img)
    i_hi, i_lo = int(per_img.argmax()), int(per_img.argmin())
    assert exp.extreme_images['highest']['name'] == batch[2][i_hi]
    assert exp.extreme_images['lowest']['name'] == batch[2][i_lo]
    assert abs(exp.extreme_images['highest']['loss'] - float(per_img[i_hi])) < 1e-7


def test_iwae_shaped_recon_per_image():
    x = torch.rand(2, 3, 4, 4)
    r = torch.rand(2, 5, 3, 4, 4)
    got = VAEXperiment.per_image_mse(r, x)
    want = ((r - x.unsqueeze(1)) ** 2).mean(dim=[1, 2, 3, 4])
    assert torch.allclose(got, want)


def test_configure_optimizers_variants():
    m = TinyAE()
    optims, scheds = VAEXperiment(m, dict(PARAMS)).configure_optimizers()
    assert isinstance(optims[0], torch.optim.Adam) and optims[0].defaults['lr'] == 0.005
    assert isinstance(scheds[0]['scheduler'], torch.optim.lr_scheduler.ExponentialLR) and scheds[0]['interval'] == 'epoch'
    d = VAEXperiment(m, dict(PARAMS, adaptive_lr=True)).configure_optimizers()
    assert isinstance(d['lr_scheduler']['scheduler'], torch.optim.lr_scheduler.ReduceLROnPlateau)
    assert d['lr_scheduler']['monitor'] == 'val_loss'
    p = dict(PARAMS)
    p['scheduler_gamma'] = None
    o = VAEXperiment(m, p).configure_optimizers()
    assert isinstance(o, list) and len(o) == 1


def test_fit_steps_and_exponential_lr():
    m = TinyAE()
    exp = VAEXperiment(m, dict(PARAMS))
    batches = [_batch(s) for s in range(3)]
    before = [p.detach().clone() for p in m.parameters()]
    hist = fit(exp, batches, epochs=2, val_batches=[_batch(9)])
    assert len(hist) == 2 and 'val_loss' in hist[0] and 'loss' in hist[0]
    assert any(not torch.equal(a, b) for a, b in zip(before, m.parameters()))
    assert hist[1]['loss'] < hist[0]['loss']


class TinyBN(TinyAE):
    """TinyAE with a BatchNorm on the code (running statistics change only in train mode)."""

    def __init__(self):
        super().__init__()
        self.bn = nn.BatchNorm1d(16)
        self.modes = []

    def forward(self, x, **kwargs):
        self.modes.append(self.training)
        h = self.bn(self.enc(x.flatten(1)))
        return [torch.tanh(self.dec(h)).view_as(x), x, h]


def test_fit_validates_in_eval_mode():
    """Lightning's validation loop runs the model under eval(): BatchNorm uses its running
    statistics and does not update them (the reference's val_loss, experiment.py:122-132)."""
    m = TinyBN()
    exp = VAEXperiment(m, dict(PARAMS))
    fit(exp, [_batch(0)], epochs=1)
    rm, rv = m.bn.running_mean.clone(), m.bn.running_var.clone()
    m.modes.clear()
    fit(exp, [], epochs=1, val_batches=[_batch(5), _batch(6)])
    assert m.modes == [False, False]
    assert torch.equal(rm, m.bn.running_mean) and torch.equal(rv, m.bn.running_var)
    assert m.training                           # back in train mode afterwards


def test_test_step_per_image_losses_match_per_image_forwards():
    """test_step (experiment.py:155-217): the per-image losses from one batched forward equal the
    reference's per-image forwards (the stand-in has no cross-sample coupling, as eval-mode BN),
    x1000, min/max tracked, 256x256 bilinear resizes, batch terms logged as test_*."""
    m = TinyAE()
    exp = VAEXperiment(m, dict(PARAMS))
    batch = _batch(3, B=5)
    out = exp.test_step(batch, 0)
    assert set(exp.logged) == {'test_loss', 'test_Reconstruction_Loss', 'test_KLD'}
    assert len(exp.test_data) == 5
    imgs = batch[0]
    for i, d in enumerate(exp.test_data):
        single = m(imgs[i:i + 1])
        want = m.loss_function(*single, M_N=0.5)
        assert abs(d['total_loss'] - float(want['loss']) * 1000) < 1e-3
        assert abs(d['recon_loss'] - float(want['Reconstruction_Loss']) * 1000) < 1e-3
        assert d['feature_loss'] is None and d['name'] == batch[2][i]
        assert tuple(d['original'].shape) == (1, 3, 256, 256)
        ref = F.interpolate(single[0].detach(), size=(256, 256), mode='bilinear', align_corners=False)
        assert torch.allclose(d['reconstruction'], ref, atol=1e-6)
    tl = [d['total_loss'] for d in exp.test_data]
    assert exp.loss_stats['total_loss'] == {'min': min(tl), 'max': max(tl)}
    assert abs(exp.normalize_loss(max(tl), 'total_loss') - 1.0) < 1e-12
    assert float(out['loss']) > 0
    # IWAE-shaped reconstructions: the first sample
    assert exp.ensure_4_dims(torch.zeros(2, 5, 3, 4, 4)).shape == (2, 3, 4, 4)
