"""Every non-default plan route (the routing knobs are constructor arguments now, no
environment variables), each a bf16 training step against the fp32 CPU oracle under the bf16
autocast bar of tests/test_gpu_bf16_shapes.py (every gradient's relative-norm error within 2x the
autocast oracle's own error + 2e-3; loss terms within 2x + 1e-4):

  StepPlan(latent_kernels=False)  fc_mu|fc_var, reparameterize, decoder_input as per-op calls
                                  (models/vanilla_vae.py:36-43, 107-117) instead of vae_latent_*
  StepPlan(pad_rgb=False)         the first conv reads the NCHW fp32 image directly
  StepPlan(batch_wgrads=False)    one weight-gradient call per layer (no vae_conv_bwd_filter_batch)
  StepPlan(wg_overlap=True)       the decoder's weight gradients on a side stream in the graph, and
                                  Adam over their prefix of the buffer right behind them there
  TrainStep(begin_ex=False)       vae_step_begin + padding calls instead of vae_step_begin_ex
  StepPlan(head_kernels=False)    a 64-channel final layer on the conv-GEMM + vae_recon_fwd route
  StepPlan(materialise=..., mat_min_flops=...)  materialised vs fused BatchNorm operands
                                  (Autoencoder big_ae widths, VQ-VAE strided layers)"""
import pytest
import torch

from test_gpu_bf16_shapes import _grad_bar, _loss_bar, _oracles, _pre_bn_bias

pytestmark = pytest.mark.gpu


def _launched_names(fn):
    from gpu_util import launched
    return launched(fn)


VANILLA_ROUTES = [
    ("latent_kernels_off", dict(latent_kernels=False), {}, None, "latent_fc_fwd"),
    ("pad_rgb_off", dict(pad_rgb=False), {}, None, None),
    ("per_layer_wgrads", dict(batch_wgrads=False), {}, None, "wg3_kernel"),
    ("wg_overlap", dict(wg_overlap=True), {}, "wg3_kernel", None),
    ("begin_plain", {}, dict(begin_ex=False), "step_begin_kernel", "step_begin_ex"),
]


@pytest.mark.parametrize("name,plan_kw,step_kw,must,must_not", VANILLA_ROUTES, ids=[r[0] for r in VANILLA_ROUTES])
def test_vanilla_family_route(name, plan_kw, step_kw, must, must_not):
    from oracle import vae_oracle as O
    from vae_amd.engine import FusedAdam, TrainStep
    from vae_amd.net import StepPlan, VAENet
    B = 16
    sd = O.make_params(O.vanilla_param_spec(), 1265)
    x, eps = O.make_inputs(B, 128, 23)
    net = VAENet(latent_dim=128, dtype=torch.bfloat16, device="cuda")
    net.load_reference_state_dict(sd)
    plan = StepPlan(net, B, loss="betaH", kld_weight=2.5e-4, **plan_kw)
    opt = FusedAdam(net, lr=0.005)
    step = TrainStep(net, plan, opt, graph=True, **step_kw)
    xs, es = x.cuda(), eps.cuda()
    names = _launched_names(lambda: step(xs, es))     # (the capture's warm-up step launches every kernel)
    torch.cuda.synchronize()
    if must:
        assert must in names, (name, names)
    if must_not:
        assert must_not not in names, (name, names)
    # the graph replay ran the step once more from the restored state: the same inputs, one step
    g16 = {k: v.cpu() for k, v in net.layout.export_reference(plan.grads).items()}
    o32, oac = _oracles("BetaVAE", sd, x, eps, M_N=2.5e-4, beta=4.0, loss_type="H")
    _loss_bar(step.loss_terms(), o32, oac, ("loss", "Reconstruction_Loss", "KLD"))
    assert _grad_bar(g16, o32, oac, f"route {name}", _pre_bn_bias) >= 30
    if name == "wg_overlap":
        # the optimizer split in two launches at the decoder's gradients (TrainStep._adam_split: the
        # prefix on the side stream): the parameters are torch Adam's first step on these gradients
        assert step._adam_split > 0
        p_got = {k: v.cpu() for k, v in net.layout.export_reference(net.params).items()}
        for k, g in g16.items():
            p0 = sd[k].clone().float().requires_grad_(True)
            ref = torch.optim.Adam([p0], lr=0.005)
            p0.grad = g.float().reshape(p0.shape)
            ref.step()
            err = (p_got[k].reshape(p0.shape) - p0.detach()).abs().max().item()
            assert err <= 1e-5, (k, err)


AE_ROUTES = [
    ("head_kernels_on", [64, 128, 256, 512, 512], {}, "head_fwd_mfma<64"),
    ("head_kernels_off", [64, 128, 256, 512, 512], dict(head_kernels=False), "recon_kernel"),
    ("materialised", [128, 256, 512, 1024, 2048], dict(mat_min_flops=0.0), "bn_apply"),
    ("not_materialised", [128, 256, 512, 1024, 2048], dict(materialise=False), None),
]


@pytest.mark.parametrize("name,hd,opts,must", AE_ROUTES, ids=[r[0] for r in AE_ROUTES])
def test_autoencoder_route(name, hd, opts, must):
    from oracle import vae_oracle as O
    from vae_amd.models import vae_models
    B = 8
    sd = O.make_params(O.ae_param_spec(latent_dim=128, hidden_dims=hd), 5)
    x, _ = O.make_inputs(B, 128, 5)
    model = vae_models["Autoencoder"](in_channels=3, latent_dim=128, hidden_dims=hd, dtype=torch.bfloat16,
                                      device="cuda")
    model.load_reference_state_dict(sd)
    step = model.fused_train_step(B, 0.0, lr=0.0005, graph=True, plan_options=opts)
    xs = x.cuda()
    names = _launched_names(lambda: step(xs))
    torch.cuda.synchronize()
    if must:
        assert must in names, (name, names)
    if name == "not_materialised":
        assert "bn_apply" not in names, names
    got = step.loss_terms()
    o32, oac = _oracles("Autoencoder", sd, x, None, M_N=0.0, hidden_dims=hd)
    _loss_bar(got, o32, oac, ("loss", "Reconstruction_Loss"))
    g_all = {k: v.cpu() for k, v in model.net.layout.export_reference(step.plan.grads).items()}
    g16 = {n: g_all["fc_mu." + n[3:] if n.startswith("fc.") else n] for n in o32["grads"]}
    assert _grad_bar(g16, o32, oac, f"AE route {name}", _pre_bn_bias) >= 30


@pytest.mark.parametrize("opts", [dict(mat_min_flops=0.0), dict(materialise=False)], ids=["materialised", "fused"])
def test_vq_route(opts):
    from oracle import vae_oracle as O
    from vae_amd import _lib as L
    from vae_amd.engine import FusedAdam
    from vae_amd.vq import VQNet, VQStepPlan
    B = 16
    sd = O.make_params(O.vq_param_spec(), 1265)
    x = torch.rand(B, 3, 64, 64, generator=torch.Generator().manual_seed(77))
    net = VQNet(dtype=torch.bfloat16, device="cuda")
    net.load_reference_state_dict(sd)
    plan = VQStepPlan(net, B, beta=0.25, **opts)
    opt = FusedAdam(net, lr=0.005)
    plan.x.copy_(x)
    st = L.stream_ptr()

    def run():
        L.call("vae_step_begin", plan.zero.data_ptr(), plan.zero.numel() * 4, opt.step.data_ptr(), st)
        plan.forward(st)
        plan.backward(st)
    names = _launched_names(run)
    torch.cuda.synchronize()
    assert ("bn_apply" in names) == ("mat_min_flops" in opts), names
    idx = plan.indices.cpu()
    o32, oac = _oracles("VQVAE", sd, x, None, M_N=0.0, vq_beta=0.25, vq_indices=idx)
    _loss_bar([plan.loss_dict()[k] for k in ("loss", "Reconstruction_Loss", "VQ_Loss")], o32, oac,
              ("loss", "Reconstruction_Loss", "VQ_Loss"))
    g16 = {k: v.cpu() for k, v in net.layout.export_reference(plan.grads).items()}
    assert _grad_bar(g16, o32, oac, f"VQ route {opts}") == len(o32["grads"])
