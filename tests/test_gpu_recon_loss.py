"""The Autoencoder's centre-weighted MSE and MS-SSIM losses on the GPU (vaehip.h vae_recon_loss;
models/autoencoder.py:95-146, :259-267; models/mssim_vae.py:182-282):

  * the kernels against the reference formulas in torch (vae_amd.models.MSSIM / the weighted MSE,
    restated from the reference and pinned by the golden tests) with autograd for dL/drecon;
  * the fused graph-replayed Autoencoder step (fused_train_step: the loss inside the step, its seed
    driving the HIP backward) against the reference's own golden vectors ae_center_b8 / ae_mssim_b8 —
    loss within 1e-4 relative and every gradient's norm within 1e-3 (BN affine 3e-3), the drop-in
    path's bars."""
import numpy as np
import pytest
import torch

from golden_util import case_inputs, load_case, summary

pytestmark = pytest.mark.gpu


def _hip_loss(cfg, recon, target):
    from vae_amd import _lib as L
    from vae_amd.models import _HipReconLoss
    r = recon.clone().cuda().requires_grad_(True)
    loss = _HipReconLoss.apply(r, target.cuda(), cfg)
    loss.backward()
    torch.cuda.synchronize()
    return float(loss), r.grad.cpu()


def _inputs(B, seed):
    g = torch.Generator().manual_seed(seed)
    target = torch.rand(B, 3, 64, 64, generator=g)
    recon = (target + 0.2 * torch.randn(B, 3, 64, 64, generator=g)).clamp(-1, 1)
    return recon, target


@pytest.mark.parametrize("B", [2, 16, 64])
def test_mssim_kernel_matches_reference_formula(B):
    from vae_amd.models import MSSIM
    m = MSSIM(3)
    recon, target = _inputs(B, 100 + B)
    r = recon.double().requires_grad_(True)
    ref = m(r, target.double())                      # the reference formula in fp64 (CPU autograd)
    ref.backward()
    got, grad = _hip_loss({"kind": "mssim", "window": m.window_1d}, recon, target)
    assert abs(got - float(ref)) <= 1e-5 * abs(float(ref)) + 1e-7, (got, float(ref))
    g_ref = r.grad.float()
    rel = float((grad - g_ref).norm() / g_ref.norm())
    assert rel < 1e-4, rel
    # and the reference's fp32 formula (what the golden vectors were made with) is as close
    r32 = recon.clone().requires_grad_(True)
    ref32 = m(r32, target)
    assert abs(got - float(ref32)) <= 1e-5 * abs(float(ref32)) + 1e-7


@pytest.mark.parametrize("sigma", [8.0, 16.0, 32.0])
def test_center_weighted_mse_kernel_matches_reference_formula(sigma):
    from vae_amd.models import Autoencoder
    recon, target = _inputs(8, 7)
    model = Autoencoder(3, 128, center_focus_sigma=sigma, dtype=torch.float32, device="cuda")
    mask = model.create_center_weight_mask(64, 64, "cpu").double()
    r = recon.double().requires_grad_(True)
    ref = Autoencoder.weighted_mse_loss(r, target.double(), mask)
    ref.backward()
    got, grad = _hip_loss({"kind": "center", "mask": mask.float().view(64, 64).cuda()}, recon, target)
    assert abs(got - float(ref)) <= 1e-5 * float(ref)
    assert float((grad - r.grad.float()).norm() / r.grad.norm()) < 1e-5


@pytest.mark.parametrize("case", ["ae_center_b8", "ae_mssim_b8"])
def test_fused_graph_step_with_recon_loss_matches_reference(case):
    """configs/center_*focused_ae.yaml / mssim_ae.yaml on the fused step (fused_train_step, HIP graph)
    against the reference's golden vectors."""
    from vae_amd.models import vae_models
    meta, ref = load_case(case)
    sd, x, _ = case_inputs(meta)
    model = vae_models["Autoencoder"](**meta["ctor"], dtype=torch.float32, device="cuda")
    model.load_reference_state_dict(sd)
    model.train()
    step = model.fused_train_step(x.shape[0], 0.0, lr=meta["lr"], graph=True)
    assert any(fn == "vae_recon_loss" for fn, _ in step.plan.fwd_calls)
    assert not any(fn == "vae_elbo_fwd" for fn, _ in step.plan.fwd_calls)
    step(x.cuda())
    torch.cuda.synchronize()
    got = step.loss_terms()
    for i, k in enumerate(("loss", "Reconstruction_Loss")):
        v = meta["loss"][k]
        assert abs(got[i] - v) <= 1e-4 * abs(v), (k, got[i], v)
    n_head = ref["recon_head"].shape[0]
    np.testing.assert_allclose(step.plan.recon[:n_head].cpu().numpy(), ref["recon_head"], rtol=0, atol=1e-4)
    g_all = model.net.layout.export_reference(step.plan.grads)
    checked = 0
    for name in meta["param_names"]:
        if name.endswith(".0.bias") and not name.startswith("final_layer.3"):
            continue
        src = "fc_mu." + name[3:] if name.startswith("fc.") else name
        rs = ref[f"grad_stats/{name}"]
        st = summary(g_all[src])
        bound = 3e-3 if name.endswith(".1.weight") or name.endswith(".1.bias") else 1e-3
        assert abs(st[1] - rs[1]) / max(rs[1], 1e-12) < bound, (name, st, rs)
        checked += 1
    assert checked >= 20
    # per-image MSE of the step (experiment.py:60-62) from the head's SSE
    per = step.plan.per_img.cpu()
    want = ((step.plan.recon.cpu() - x) ** 2).mean(dim=[1, 2, 3])
    torch.testing.assert_close(per, want, rtol=1e-4, atol=1e-7)


def test_experiment_fit_runs_mssim_config_on_the_graph_engine():
    """experiment.fit(engine='graph') takes the MS-SSIM Autoencoder onto GraphedSteps (no eager
    fallback), and its loss follows the eager drop-in path's on the same batches."""
    from vae_amd.experiment import VAEXperiment, _fusable, fit
    from vae_amd.models import vae_models
    g = torch.Generator(device="cuda").manual_seed(3)
    batches = [(torch.rand(8, 3, 64, 64, generator=g, device="cuda"), torch.zeros(8, device="cuda"),
                [f"{i}.png" for i in range(8)]) for _ in range(3)]
    out = {}
    for engine in ("graph", "eager"):
        torch.manual_seed(0)
        model = vae_models["Autoencoder"](in_channels=3, latent_dim=128, use_mssim_loss=True, dtype=torch.float32,
                                          device="cuda", seed=5)
        assert _fusable(model)
        exp = VAEXperiment(model, {"LR": 0.001, "weight_decay": 0.0, "kld_weight": 0.0})
        out[engine] = fit(exp, batches, epochs=1, engine=engine)[0]["loss"]
    assert np.isfinite(out["graph"]) and 0.0 < out["graph"] < 1.0
    assert abs(out["graph"] - out["eager"]) <= 1e-3 * abs(out["eager"]), out
