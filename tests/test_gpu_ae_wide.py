"""The fork's wide Autoencoder configs (models/autoencoder.py:16-86 with the hidden_dims of
configs/big_ae.yaml, patient_vbig_ae.yaml and patient_vvbig_ae.yaml: BatchNorm widths of
1024-4096 channels, a 128-512-channel final layer) on the MI355X kernels.

  * big_ae at B=4: the reference's own golden vectors (ae_big_b4, made by the reference's modules)
    — covered by tests/test_gpu_models.py::test_autoencoder_against_reference;
  * patient_vbig_ae / patient_vvbig_ae in fp32 (the parity mode) against the CPU oracle at B=2:
    loss within 1e-4 relative (north_star), reconstructions, z, every gradient's norm within 1e-3
    (BatchNorm affine 3e-3) — the bars of the golden tests;
  * big_ae in bf16 (the throughput mode, graph-replayed TrainStep) against the same step in fp32 on
    the GPU from the same parameters: the bf16 bar is stated per quantity below.

The oracle's fixtures for the two widest configs are not pinned by reference-generated vectors
(only big_ae is, through ae_big_b4): the oracle's Autoencoder path is the same code at every width,
and ae_big_b4 pins it (tests/test_oracle_golden.py)."""
import numpy as np
import pytest
import torch

from golden_util import summary

pytestmark = pytest.mark.gpu

WIDTHS = {"patient_vbig_ae": [256, 512, 1024, 2048, 4096], "patient_vvbig_ae": [512, 1024, 2048, 4096, 4096],
          "big_ae": [128, 256, 512, 1024, 2048]}


def _oracle_inputs(hd, batch, seed=11):
    from oracle import vae_oracle as O
    sd = O.make_params(O.ae_param_spec(latent_dim=128, hidden_dims=hd), seed)
    x, _ = O.make_inputs(batch, 128, seed)
    return sd, x


@pytest.mark.parametrize("cfg", ["patient_vbig_ae", "patient_vvbig_ae"])
def test_wide_autoencoder_fp32_matches_oracle(cfg):
    from oracle import vae_oracle as O
    from vae_amd.models import vae_models
    hd = WIDTHS[cfg]
    B = 2
    sd, x = _oracle_inputs(hd, B)
    ref = O.train_step("Autoencoder", sd, x, M_N=0.0, hidden_dims=hd, do_adam=False)
    model = vae_models["Autoencoder"](in_channels=3, latent_dim=128, hidden_dims=list(hd), dtype=torch.float32,
                                      device="cuda")
    model.load_reference_state_dict(sd)
    model.train()
    results = model(x.cuda())
    losses = model.loss_function(*results, M_N=0.0, optimizer_idx=0, batch_idx=0)
    for k in ("loss", "Reconstruction_Loss"):
        want = float(ref["loss"][k])
        assert abs(float(losses[k]) - want) <= 1e-4 * abs(want), (k, float(losses[k]), want)
    np.testing.assert_allclose(results[0].detach().cpu().numpy(), ref["recon"].numpy(), rtol=0, atol=1e-4)
    z = model.encode(x.cuda())[0]
    np.testing.assert_allclose(z.detach().cpu().numpy(), ref["z"].numpy(), rtol=0,
                               atol=1e-4 * float(ref["z"].abs().max()))
    model.train()
    results = model(x.cuda())                # (encode() ran a forward of its own: redo the step's)
    losses = model.loss_function(*results, M_N=0.0, optimizer_idx=0, batch_idx=0)
    model.zero_grad(set_to_none=True)
    losses["loss"].backward()
    g_all = model.net.layout.export_reference(model.flat.grad.detach())
    checked = 0
    for name, rg in ref["grads"].items():
        if name.endswith(".0.bias") and not name.startswith("final_layer.3"):
            continue                        # conv bias before a BatchNorm: analytically zero
        src = "fc_mu." + name[3:] if name.startswith("fc.") else name
        got, want = summary(g_all[src]), summary(rg)
        bound = 3e-3 if name.endswith(".1.weight") or name.endswith(".1.bias") else 1e-3
        assert abs(got[1] - want[1]) / max(want[1], 1e-12) < bound, (name, got, want)
        checked += 1
    assert checked >= 20
    for n in ("fc_var.weight", "fc_var.bias"):
        assert float(g_all[n].abs().max()) == 0.0


def _ae_step(hd, batch, dtype, sd, x):
    """One fused Autoencoder training step (forward, MSE, backward, Adam) through TrainStep."""
    from vae_amd.models import vae_models
    model = vae_models["Autoencoder"](in_channels=3, latent_dim=128, hidden_dims=list(hd), dtype=dtype, device="cuda")
    model.load_reference_state_dict(sd)
    step = model.fused_train_step(batch, 0.0, lr=0.0005, graph=dtype == torch.bfloat16)
    step(x.cuda())
    torch.cuda.synchronize()
    return model, step


def test_big_autoencoder_bf16_step_tracks_fp32():
    """configs/big_ae.yaml in the bf16 throughput mode (the graph-replayed step the bench times)
    against the fp32 parity mode from the same parameters and batch.  bf16 stores every
    pre-BatchNorm activation and gradient (eleven layers deep), so the bars are a regression guard
    on that rounding, not parity (parity is the fp32 mode's, above).  Measured (B=16): loss 2e-6
    relative, reconstructions 4.4e-3 mean / 4.5e-2 max absolute, gradient error growing smoothly
    from 2e-4 at the head through 1.3e-2 (final ConvT) to 0.20 at decoder.0 (the backward
    amplifies rounding layer by layer, as the VanillaVAE's does: tests/test_gpu_step.py
    test_bf16_gradients_close_to_fp32), encoder / bottleneck gradients cosine 0.96-0.99.  Bars:
    loss 1e-3 relative; reconstructions 1e-2 mean / 0.1 max; head and final layer within 2e-2,
    every decoder gradient within 0.4 relative norm; encoder gradients cosine > 0.93."""
    hd = WIDTHS["big_ae"]
    B = 16
    sd, x = _oracle_inputs(hd, B, seed=3)
    m16, s16 = _ae_step(hd, B, torch.bfloat16, sd, x)
    m32, s32 = _ae_step(hd, B, torch.float32, sd, x)
    l16, l32 = s16.loss_terms()[0], s32.loss_terms()[0]
    r16, r32 = s16.plan.recon.float().cpu(), s32.plan.recon.float().cpu()
    d = (r16 - r32).abs()
    g16 = m16.net.layout.export_reference(s16.plan.grads)
    g32 = m32.net.layout.export_reference(s32.plan.grads)
    dec, enc = {}, {}
    for name, b in g32.items():
        if name.startswith("fc_var") or (name.endswith(".0.bias") and not name.startswith("final_layer.3")):
            continue
        a = g16[name].double().flatten().cpu()
        b = b.double().flatten().cpu()
        if float(b.norm()) == 0.0:
            continue
        if name.startswith(("decoder.", "final_layer.")):
            dec[name] = float((a - b).norm() / b.norm())
        else:
            enc[name] = float(a.dot(b) / (a.norm() * b.norm()))
    print(f"loss bf16 {l16:.6f} fp32 {l32:.6f}; recon |d| mean {float(d.mean()):.2e} max {float(d.max()):.2e}")
    print("decoder rel:", {k: round(v, 4) for k, v in dec.items()})
    print("encoder cos:", {k: round(v, 4) for k, v in enc.items()})
    assert np.isfinite(l16) and abs(l16 - l32) <= 1e-3 * abs(l32), (l16, l32)
    assert float(d.mean()) < 1e-2 and float(d.max()) < 0.1
    assert max(v for k, v in dec.items() if k.startswith("final_layer")) < 2e-2
    assert max(dec.values()) < 0.4
    assert min(enc.values()) > 0.93
