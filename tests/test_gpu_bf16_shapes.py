"""The bf16 throughput step at the shapes bench.py times, against the CPU oracle under
torch.autocast(bfloat16) (the precision contract of a bf16 PyTorch run of the reference), both
measured against the fp32 oracle on the same inputs and parameters.

The bf16 step runs kernels the fp32 parity mode does not (vae_c3.hip c3 / c3w / c1w, vae_p1.hip,
vae_latent.hip, vae_hires.hip, vae_wgrad_batch.hip, the bf16 conv-GEMM tiles), so these tests are
what pins THOSE kernels at step level, at the benchmarked shapes:

  * BetaVAE-H, B=32 (BASELINE configs[2] per GPU; models/beta_vae.py:129-152)
  * IWAE K=5, B=64 (configs[3]; the decoder at B*S = 320 rows; models/iwae.py:95-160)
  * Autoencoder big_ae, B=64 (configs/big_ae.yaml; models/autoencoder.py:16-86)
  * VQ-VAE, B=128 (configs[4]; models/vq_vae.py) — EVERY gradient tensor, the residual stacks'
    3x3 / 1x1 weights (c3w / c1w outputs) included; the oracle is teacher-forced with the GPU's
    code indices (both the fp32 and the autocast one), so the comparison is of the rest of the step.

Bar: every gradient's relative-norm error against the fp32 oracle within
2x the autocast oracle's own error on that tensor + 2e-3; the loss terms within 2x the autocast
oracle's error + 1e-4 relative."""
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _record_coverage(tag, test, names):
    """The kernels a passing step-level test ran (vae_launch_log), for tools/kernel_coverage.py."""
    from stepcheck import kernel_names
    out = os.path.join(REPO, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"kernel_coverage_{tag}.json"), "w") as f:
        json.dump({"test": f"tests/test_gpu_bf16_shapes.py::{test}", "step_kernels": kernel_names(names),
                   "coverage": {k: [test] for k in kernel_names(names)}}, f, indent=1)


def _loss_bar(got, o32, oac, keys):
    for i, k in enumerate(keys):
        ref = float(o32["loss"][k])
        e_ac = abs(float(oac["loss"][k]) - ref) / abs(ref)
        e_hip = abs(got[i] - ref) / abs(ref)
        assert e_hip <= 2 * e_ac + 1e-4, (k, got[i], ref, e_hip, e_ac)


def _grad_bar(g16, o32, oac, tag, skip=lambda n: False):
    rows = []
    for name, gr in o32["grads"].items():
        if skip(name):
            continue
        d = gr.double()
        if float(d.norm()) == 0.0:
            continue
        e_ac = float((oac["grads"][name].double() - d).norm() / d.norm())
        e_hip = float((g16[name].double() - d).norm() / d.norm())
        rows.append((name, e_hip, e_ac))
    print(f"{tag}: " + "; ".join(f"{n}: hip {a:.3e} autocast {b:.3e}" for n, a, b in rows))
    bad = [(n, a, b) for n, a, b in rows if not a <= 2 * b + 2e-3]
    assert not bad, bad
    return len(rows)


def _pre_bn_bias(name):
    # a conv bias followed by train-mode BatchNorm: analytically zero gradient
    return name.endswith(".0.bias") and not name.startswith("final_layer.3")


def _oracles(arch, sd, x, eps, **kw):
    from oracle import vae_oracle as O
    o32 = O.train_step(arch, sd, x, eps, do_adam=False, **kw)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        oac = O.train_step(arch, sd, x, eps, do_adam=False, **kw)
    return o32, oac


def _vanilla_family_step(loss, batch, samples, M_N):
    from oracle import vae_oracle as O
    from vae_amd import _lib as L
    from vae_amd.engine import FusedAdam
    from vae_amd.net import StepPlan, VAENet
    sd = O.make_params(O.vanilla_param_spec(), 1265)
    x, eps = O.make_inputs(batch, 128, 17, samples=samples if samples > 1 else None)
    net = VAENet(latent_dim=128, dtype=torch.bfloat16, device="cuda")
    net.load_reference_state_dict(sd)
    plan = StepPlan(net, batch, loss=loss, kld_weight=M_N, samples=samples)
    opt = FusedAdam(net, lr=0.005)
    plan.x.copy_(x)
    plan.eps.copy_(eps.reshape(plan.eps.shape))
    st = L.stream_ptr()
    L.call("vae_step_begin", plan.zero.data_ptr(), plan.zero.numel() * 4, opt.step.data_ptr(), st)
    if plan.loss_kind == L.LOSS_BETA_B:
        plan.num_iter.add_(1.0)
    plan.forward(st)
    plan.backward(st)
    torch.cuda.synchronize()
    g16 = {k: v.cpu() for k, v in net.layout.export_reference(plan.grads).items()}
    return sd, x, eps, plan, g16


def test_betaH_b32_bf16_tracks_autocast_oracle():
    sd, x, eps, plan, g16 = _vanilla_family_step("betaH", 32, 1, 2.5e-4)
    o32, oac = _oracles("BetaVAE", sd, x, eps, M_N=2.5e-4, beta=4.0, loss_type="H")
    _loss_bar(plan.out.cpu().tolist(), o32, oac, ("loss", "Reconstruction_Loss", "KLD"))
    assert _grad_bar(g16, o32, oac, "betaH B=32", _pre_bn_bias) >= 30


def test_iwae_64x5_bf16_tracks_autocast_oracle():
    sd, x, eps, plan, g16 = _vanilla_family_step("iwae", 64, 5, 2.5e-4)
    o32, oac = _oracles("IWAE", sd, x, eps, M_N=2.5e-4)
    _loss_bar(plan.out.cpu().tolist(), o32, oac, ("loss", "Reconstruction_Loss", "KLD"))
    assert _grad_bar(g16, o32, oac, "IWAE 64x5", _pre_bn_bias) >= 30


def test_big_ae_b64_bf16_tracks_autocast_oracle():
    """configs/big_ae.yaml at the bench's B=64 through the graph-replayed fused step (the
    Autoencoder model's fused_train_step, as bench.py --arch ae_big times it)."""
    from oracle import vae_oracle as O
    from vae_amd.models import vae_models
    hd = [128, 256, 512, 1024, 2048]
    sd = O.make_params(O.ae_param_spec(latent_dim=128, hidden_dims=hd), 5)
    x, _ = O.make_inputs(64, 128, 5)
    model = vae_models["Autoencoder"](in_channels=3, latent_dim=128, hidden_dims=hd, dtype=torch.bfloat16,
                                      device="cuda")
    model.load_reference_state_dict(sd)
    step = model.fused_train_step(64, 0.0, lr=0.0005, graph=True)
    from gpu_util import launched
    xs = x.cuda()
    names = launched(lambda: step(xs))
    torch.cuda.synchronize()
    got = step.loss_terms()
    o32, oac = _oracles("Autoencoder", sd, x, None, M_N=0.0, hidden_dims=hd)
    _loss_bar(got, o32, oac, ("loss", "Reconstruction_Loss"))
    g_all = {k: v.cpu() for k, v in model.net.layout.export_reference(step.plan.grads).items()}
    g16 = {n: g_all["fc_mu." + n[3:] if n.startswith("fc.") else n] for n in o32["grads"]}
    assert _grad_bar(g16, o32, oac, "big_ae B=64", _pre_bn_bias) >= 30
    _record_coverage("ae_big_64", "test_big_ae_b64_bf16_tracks_autocast_oracle", names)


def test_vq_b128_bf16_tracks_autocast_oracle_every_gradient():
    from oracle import vae_oracle as O
    from vae_amd import _lib as L
    from vae_amd.engine import FusedAdam
    from vae_amd.vq import VQNet, VQStepPlan
    B = 128
    sd = O.make_params(O.vq_param_spec(), 1265)
    x = torch.rand(B, 3, 64, 64, generator=torch.Generator().manual_seed(1265 + B))
    net = VQNet(dtype=torch.bfloat16, device="cuda")
    net.load_reference_state_dict(sd)
    plan = VQStepPlan(net, B, beta=0.25)
    opt = FusedAdam(net, lr=0.005)
    from gpu_util import launched
    from vae_amd.engine import TrainStep
    # bench.py --arch vq's step: the graph-replayed TrainStep (step head, forward, loss, backward,
    # Adam); the capture restores the state its warm-up step changed, so the replay is one step
    # from these parameters (the gradients stay in plan.grads)
    step = TrainStep(net, plan, opt, graph=True)
    xs = x.cuda()
    names = launched(lambda: step(xs))
    torch.cuda.synchronize()
    idx = plan.indices.cpu()
    o32, oac = _oracles("VQVAE", sd, x, None, M_N=0.0, vq_beta=0.25, vq_indices=idx)
    _loss_bar([plan.loss_dict()[k] for k in ("loss", "Reconstruction_Loss", "VQ_Loss")], o32, oac,
              ("loss", "Reconstruction_Loss", "VQ_Loss"))
    g16 = {k: v.cpu() for k, v in net.layout.export_reference(plan.grads).items()}
    n = _grad_bar(g16, o32, oac, "VQ B=128")
    assert n == len(o32["grads"]), (n, len(o32["grads"]))       # every tensor has a gradient and is checked
    assert any("res" in k or "encoder.3" in k for k in o32["grads"])
    _record_coverage("vq_128", "test_vq_b128_bf16_tracks_autocast_oracle_every_gradient", names)
