"""eps drawn on the device inside the fused step (StepPlan.use_device_eps: Philox4x32-10 + Box-Muller
in vae_latent_dec_fwd) — the reference's torch.randn_like(std) of reparameterize, drawn every step
(models/vanilla_vae.py:107-117, beta_vae.py:112-122, iwae.py:111-119).

The draw cannot equal torch's CPU generator bit for bit (nor does the reference promise a stream),
so parity is checked the way the injected-eps tests do it, teacher-forced: the noise the kernel drew
(written to plan.eps) is fed to the oracle, and the bf16 step must then meet the autocast bar of
tests/test_gpu_bf16_shapes.py.  The draw itself: N(0,1) moments and a Kolmogorov-Smirnov test,
fresh noise every step, the same noise for the same (seed, step)."""
import numpy as np
import pytest
import torch

from test_gpu_bf16_shapes import _grad_bar, _loss_bar, _oracles, _pre_bn_bias

pytestmark = pytest.mark.gpu


def _plan(batch=64, samples=1, loss="vanilla", M_N=2.5e-4, seed=99):
    from oracle import vae_oracle as O
    from vae_amd.engine import FusedAdam
    from vae_amd.net import StepPlan, VAENet
    sd = O.make_params(O.vanilla_param_spec(), 1265)
    x, _ = O.make_inputs(batch, 128, 23)
    net = VAENet(latent_dim=128, dtype=torch.bfloat16, device="cuda")
    net.load_reference_state_dict(sd)
    plan = StepPlan(net, batch, loss=loss, kld_weight=M_N, samples=samples)
    opt = FusedAdam(net, lr=0.005)
    assert plan.use_device_eps(opt.step, seed)
    plan.x.copy_(x)
    return sd, x, plan, opt


def _fwd_bwd(plan, opt, backward=True):
    from vae_amd import _lib as L
    st = L.stream_ptr()
    L.call("vae_step_begin", plan.zero.data_ptr(), plan.zero.numel() * 4, opt.step.data_ptr(), st)
    plan.forward(st)
    if backward:
        plan.backward(st)
    torch.cuda.synchronize()


def test_device_eps_is_standard_normal_and_fresh_every_step():
    from scipy import stats
    _, _, plan, opt = _plan(batch=64, samples=5, loss="iwae")
    draws = []
    for _ in range(3):
        _fwd_bwd(plan, opt, backward=False)
        draws.append(plan.eps.cpu().double().flatten())
    for e in draws:
        assert e.numel() == 64 * 5 * 128
        assert abs(float(e.mean())) < 0.03 and abs(float(e.std()) - 1) < 0.03, (float(e.mean()), float(e.std()))
        assert stats.kstest(e.numpy(), "norm").pvalue > 1e-4
        assert float(e.abs().max()) < 7.0 and bool(torch.isfinite(e).all())
    # a fresh draw every step, uncorrelated with the previous one
    for a, b in zip(draws, draws[1:]):
        assert not torch.equal(a, b)
        assert abs(float(np.corrcoef(a.numpy(), b.numpy())[0, 1])) < 0.03
    # the same (seed, step) draws the same noise
    _, _, plan2, opt2 = _plan(batch=64, samples=5, loss="iwae")
    _fwd_bwd(plan2, opt2, backward=False)
    assert torch.equal(plan2.eps.cpu().double().flatten(), draws[0])


def test_device_eps_step_is_the_reparameterization_of_its_own_draw():
    """z = mu + eps * exp(logvar / 2) with the drawn eps (bf16 z), and the whole bf16 step
    teacher-forced on that eps meets the autocast-oracle bar (loss terms and every gradient)."""
    sd, x, plan, opt = _plan(batch=64)
    _fwd_bwd(plan, opt)
    eps = plan.eps.cpu()
    mulv = plan.mulv.cpu()
    z_ref = mulv[:, :128] + eps * torch.exp(0.5 * mulv[:, 128:])
    torch.testing.assert_close(plan.z.float().cpu(), z_ref, rtol=1e-2, atol=1e-2)
    o32, oac = _oracles("VanillaVAE", sd, x, eps, M_N=2.5e-4)
    _loss_bar(plan.out.cpu().tolist(), o32, oac, ("loss", "Reconstruction_Loss", "KLD"))
    g16 = {k: v.cpu() for k, v in plan.net.layout.export_reference(plan.grads).items()}
    assert _grad_bar(g16, o32, oac, "VanillaVAE B=64 device eps", _pre_bn_bias) >= 30


def test_graphed_train_step_draws_per_replay():
    """TrainStep(device_eps=seed) — what bench.py times: every graph replay draws new noise."""
    from vae_amd.engine import FusedAdam, TrainStep
    from vae_amd.net import StepPlan, VAENet
    net = VAENet(latent_dim=128, dtype=torch.bfloat16, device="cuda")
    plan = StepPlan(net, 64, loss="vanilla", kld_weight=1e-8)
    step = TrainStep(net, plan, FusedAdam(net, lr=0.005), graph=True, device_eps=7)
    assert step.device_eps
    plan.x.uniform_()
    seen = []
    for _ in range(3):
        step()
        torch.cuda.synchronize()
        seen.append(plan.eps.clone())
    assert not torch.equal(seen[0], seen[1]) and not torch.equal(seen[1], seen[2])
    assert all(np.isfinite(v) for v in step.loss_terms())
