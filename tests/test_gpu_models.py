"""The BaseVAE drop-in (vae_amd.models) against the reference's golden vectors: forward
outputs, the loss dict of the reference formulas, gradients reached through
loss.backward() (the fused HIP backward behind autograd), and one torch.optim.Adam step on
the flat parameter — fp32 parity mode, same bars as tests/test_gpu_step.py."""
import numpy as np
import pytest
import torch

from golden_util import case_inputs, load_case, summary

pytestmark = pytest.mark.gpu

CASES = ["vanilla_b16", "betaH_b16", "betaB_b8", "iwae_b4"]


def _build(meta, dtype=torch.float32):
    from vae_amd.models import vae_models
    kw = dict(meta["ctor"])
    kw.pop("name", None)
    model = vae_models[meta["arch"]](**kw, dtype=dtype, device="cuda")
    return model


@pytest.mark.parametrize("via", ["gpu_elbo", "torch_loss"])
@pytest.mark.parametrize("case", CASES)
def test_models_forward_loss_backward_adam(case, via):
    """via gpu_elbo: loss_function on forward's own list — vae_elbo_fwd and the fused seeds
    (what VAEXperiment.training_step runs); via torch_loss: on views of those tensors — the
    reference formula in torch, autograd's dL/drecon and dL/d[mu|log_var] seeding the backward."""
    meta, ref = load_case(case)
    sd, x, eps = case_inputs(meta)
    model = _build(meta)
    model.load_reference_state_dict(sd)
    model.train()
    S = meta["samples"] or 1
    xd, ed = x.cuda(), eps.cuda().reshape(meta["batch"] * S, -1)
    results = model(xd, eps=ed)
    if via == "torch_loss":
        results = [t.view_as(t) for t in results]
    losses = model.loss_function(*results, M_N=meta["M_N"], optimizer_idx=0, batch_idx=0)
    assert ("_HipELBO" in type(losses["loss"].grad_fn).__name__) == (via == "gpu_elbo"), type(losses["loss"].grad_fn)
    assert set(losses) == set(meta["loss"])
    for k, v in meta["loss"].items():
        got = float(losses[k])
        assert abs(got - v) <= 1e-4 * abs(v), (k, got, v)
    # forward tensors
    D = meta["ctor"]["latent_dim"]
    mu = results[2].detach().reshape(meta["batch"], -1, D)[:, 0].cpu().numpy()
    np.testing.assert_allclose(mu, ref["mu"], rtol=0, atol=1e-4 * np.abs(ref["mu"]).max())
    recon = results[0].detach().cpu().numpy()
    n_head = ref["recon_head"].shape[0]
    np.testing.assert_allclose(recon[:n_head], ref["recon_head"], rtol=0, atol=1e-4)
    # backward through autograd
    model.zero_grad(set_to_none=True)
    losses["loss"].backward()
    grads = model.net.layout.export_reference(model.flat.grad.detach())
    for name in meta["param_names"]:
        if name.endswith(".0.bias") and not name.startswith("final_layer.3"):
            continue        # analytically zero (conv bias before train-mode BN): see test_gpu_step
        rs = ref[f"grad_stats/{name}"]
        st = summary(grads[name])
        err = abs(st[1] - rs[1]) / max(rs[1], 1e-12)
        bound = 3e-3 if name.endswith(".1.weight") or name.endswith(".1.bias") else 1e-3
        assert err < bound, (name, st, rs)
    # running statistics (train-mode BatchNorm)
    run = model.reference_state_dict()
    for k in ref:
        if k.startswith("running/"):
            np.testing.assert_allclose(run[k[8:]].cpu().numpy(), ref[k], rtol=1e-4, atol=1e-6, err_msg=k)
    # a plain torch optimizer on the flat parameter (experiment.py:308-311)
    opt = torch.optim.Adam(model.parameters(), lr=meta["lr"], weight_decay=0.0)
    opt.step()
    newp = model.reference_state_dict()
    for name in meta["param_names"]:
        if name.endswith(".0.bias") and not name.startswith("final_layer.3"):
            continue
        gref = ref[f"grad_head/{name}"]
        ok = np.abs(gref) > 1e-5
        np.testing.assert_allclose(newp[name].flatten()[:64].cpu().numpy()[ok], ref[f"new_head/{name}"][ok], rtol=0,
                                   atol=1e-3 * meta["lr"] + 1e-7, err_msg=name)


def test_models_bf16_step_runs_and_trains():
    """bf16 throughput mode through the drop-in: a few Adam steps reduce the loss."""
    from vae_amd.models import VanillaVAE
    torch.manual_seed(0)
    model = VanillaVAE(3, 128, dtype=torch.bfloat16, device="cuda", seed=1265)
    opt = torch.optim.Adam(model.parameters(), lr=5e-3)
    x = torch.rand(32, 3, 64, 64, device="cuda")
    first = None
    for _ in range(8):
        res = model(x)
        loss = model.loss_function(*res, M_N=2.5e-4)["loss"]
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        first = float(loss) if first is None else first
    assert float(loss) < first


def test_vqvae_dropin_forward_loss_backward():
    """VQVAE through the drop-in (reference forward/loss_function signatures): loss dict against
    the teacher-forced oracle, flat-parameter gradients through loss.backward()."""
    from oracle import vae_oracle as O
    from vae_amd.models import vae_models
    meta, ref = load_case("vq_b4")
    sd, x, _ = case_inputs(meta)
    model = vae_models["VQVAE"](**meta["ctor"], dtype=torch.float32, device="cuda")
    model.load_reference_state_dict(sd)
    results = model(x.cuda())
    assert len(results) == 3
    losses = model.loss_function(*results, M_N=meta["M_N"], optimizer_idx=0, batch_idx=0)
    assert set(losses) == {"loss", "Reconstruction_Loss", "VQ_Loss"}
    plan = model._plan(x.shape[0])
    o = O.train_step("VQVAE", sd, x, M_N=0.0, lr=meta["lr"], vq_beta=meta["ctor"]["beta"],
                     vq_indices=plan.indices.cpu(), do_adam=False)
    for k in ("loss", "Reconstruction_Loss", "VQ_Loss"):
        assert abs(float(losses[k]) - o["loss"][k]) <= 1e-4 * abs(o["loss"][k]), (k, float(losses[k]), o["loss"][k])
    model.zero_grad(set_to_none=True)
    losses["loss"].backward()
    grads = model.net.layout.export_reference(model.flat.grad.detach())
    for name, gr in o["grads"].items():
        err = float((grads[name].cpu() - gr).norm() / gr.norm().clamp_min(1e-30))
        assert err < 1e-3, (name, err)


def test_experiment_training_step_on_gpu_model():
    """vae_amd.experiment.VAEXperiment.training_step drives the drop-in model (experiment.py:45-86)."""
    from vae_amd.experiment import VAEXperiment
    from vae_amd.models import VanillaVAE
    model = VanillaVAE(3, 128, dtype=torch.float32, device="cuda", seed=1265)
    exp = VAEXperiment(model, {'LR': 0.005, 'weight_decay': 0.0, 'scheduler_gamma': 0.95, 'kld_weight': 2.5e-4})
    optims, scheds = exp.configure_optimizers()
    x = torch.rand(16, 3, 64, 64, device="cuda")
    batch = (x, torch.zeros(16, dtype=torch.float64), [f"{i}.png" for i in range(16)])
    losses = []
    for i in range(4):
        optims[0].zero_grad(set_to_none=True)
        loss = exp.training_step(batch, i)
        loss.backward()
        optims[0].step()
        losses.append(float(exp.logged["loss"]))
    assert losses[-1] < losses[0]
    assert exp.extreme_images["highest"]["loss"] >= exp.extreme_images["lowest"]["loss"]


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 3e-2)])
def test_eval_mode_forward_uses_running_statistics(dtype, tol):
    """model.eval() (validation_step / generate, experiment.py:122-132, vanilla_vae.py:163-173):
    BatchNorm from the running statistics — against the oracle's eval forward; running
    statistics are not modified."""
    from oracle import vae_oracle as O
    from vae_amd.models import VanillaVAE
    meta, _ = load_case("vanilla_b16")
    sd, x, eps = case_inputs(meta)
    g = torch.Generator().manual_seed(5)
    for k in list(sd):                      # non-trivial running statistics
        if k.endswith("running_mean"):
            sd[k] = torch.randn(sd[k].shape, generator=g) * 0.1
        elif k.endswith("running_var"):
            sd[k] = 0.5 + torch.rand(sd[k].shape, generator=g)
    model = VanillaVAE(3, 128, dtype=dtype, device="cuda")
    model.load_reference_state_dict(sd)
    model.eval()
    with torch.no_grad():
        recon, _, mu, log_var = model(x.cuda(), eps=eps.cuda())
    P = {k: v.clone() for k, v in sd.items()}
    stats = {}
    mu_r, lv_r = O.vanilla_encode(P, x, O.DEFAULT_HIDDEN, False, stats)
    rec_r = O.vanilla_decode(P, O.reparameterize(mu_r, lv_r, eps), O.DEFAULT_HIDDEN, False, stats)
    for got, want in ((mu, mu_r), (log_var, lv_r), (recon, rec_r)):
        err = float((got.float().cpu() - want).abs().max() / want.abs().max())
        assert err < tol, err
    after = model.reference_state_dict()
    for k in sd:
        if "running" in k:
            assert torch.equal(after[k].cpu(), sd[k]), k
    # generate() and sample() run in eval mode too
    with torch.no_grad():
        assert model.generate(x.cuda()).shape == x.shape
        assert model.sample(4, "cuda").shape == (4, 3, 64, 64)


def test_state_dict_is_reference_keyed_and_roundtrips():
    """Checkpoint interop: model.state_dict() has the reference's keys/layouts (78 tensors for
    VanillaVAE), a Lightning checkpoint of it reloads into a fresh model, and the reference's own
    golden state dict loads through load_state_dict."""
    from vae_amd.models import VanillaVAE, VQVAE
    from vae_amd import run as R
    meta, _ = load_case("vanilla_b16")
    sd, _, _ = case_inputs(meta)
    m = VanillaVAE(3, 128, device="cuda")
    m.load_state_dict(sd)                                  # the reference's state dict, unchanged
    out = m.state_dict()
    assert list(out) == list(sd)
    for k in sd:
        assert torch.equal(out[k].cpu().to(sd[k].dtype), sd[k]), k
    import tempfile, os
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "last.ckpt")
        R.save_checkpoint(path, m, 0, 1)
        m2 = VanillaVAE(3, 128, device="cuda", seed=3)
        R.load_checkpoint(path, m2)
        for k, v in m2.state_dict().items():
            assert torch.equal(v.cpu(), out[k].cpu()), k
    q = VQVAE(3, 64, 512, device="cuda", seed=1)
    assert len(q.state_dict()) == 39


def test_run_cli_synthetic_end_to_end(tmp_path):
    """vae_amd.run (run.py counterpart): one epoch on synthetic images, Lightning checkpoints,
    test pass from last.ckpt."""
    import yaml
    from vae_amd import run as R
    cfg = {"model_params": {"name": "VanillaVAE", "in_channels": 3, "latent_dim": 128},
           "data_params": {"data_path": "Data/", "train_batch_size": 16, "val_batch_size": 16, "patch_size": 64},
           "exp_params": {"LR": 0.005, "weight_decay": 0.0, "scheduler_gamma": 0.95, "kld_weight": 2.5e-4,
                          "manual_seed": 1265},
           "trainer_params": {"gpus": [0], "max_epochs": 2},
           "logging_params": {"save_dir": str(tmp_path / "logs"), "name": "VanillaVAE"}}
    p = tmp_path / "vae.yaml"
    p.write_text(yaml.safe_dump(cfg))
    res = R.main(["-c", str(p), "--synthetic", "72", "--dtype", "bf16"])
    assert "loss" in res and "val_loss" in res and "test_loss" in res
    ck = tmp_path / "logs" / "VanillaVAE-128-kl_0.00025-train_synthetic" / "version_0" / "checkpoints"
    assert (ck / "last.ckpt").exists() and (ck / "best.ckpt").exists()
    sd = torch.load(ck / "last.ckpt", weights_only=True)["state_dict"]
    assert "model.encoder.0.0.weight" in sd and "model.final_layer.3.bias" in sd


@pytest.mark.parametrize("arch", ["VanillaVAE", "BetaVAE", "IWAE"])
def test_experiment_graph_engine_matches_eager(arch):
    """fit(engine="graph") — one HIP-graph TrainStep per batch with FusedAdam — against the eager
    drop-in (training_step -> GPU ELBO -> loss.backward -> torch.optim.Adam) from the same
    parameters: the logged loss terms of the first step agree to fp32 rounding, and the first Adam
    update except on a few elements whose gradient is within rounding of zero (their first step
    lr*g/|g| may flip sign)."""
    from vae_amd.experiment import GraphedSteps, VAEXperiment
    from vae_amd.models import vae_models
    kw = dict(in_channels=3, latent_dim=128, dtype=torch.float32, device="cuda", seed=1265)
    if arch == "BetaVAE":
        kw.update(loss_type="H", beta=4)
    params = {'LR': 0.005, 'weight_decay': 0.0, 'kld_weight': 2.5e-4}
    B = 16
    x = torch.rand(B, 3, 64, 64, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    batch = (x, torch.zeros(B), [f"{i}.png" for i in range(B)])
    runs = {}
    for engine in ("eager", "graph"):
        model = vae_models[arch](**kw)
        model.train()
        p0 = model.flat.detach().clone()
        exp = VAEXperiment(model, params)
        opt = exp.configure_optimizers()[0]
        torch.manual_seed(11)                          # the same eps draws on both paths
        torch.cuda.manual_seed(11)
        if engine == "eager":
            opt.zero_grad(set_to_none=True)
            loss = exp.training_step(batch, 0)
            assert "_HipELBO" in type(loss.grad_fn).__name__
            loss.backward()
            opt.step()
        else:
            GraphedSteps(exp, opt)(batch, 0)
        torch.cuda.synchronize()
        runs[engine] = ({k: float(v) for k, v in exp.logged.items()}, model.flat.detach() - p0)
    (le, de), (lg, dg) = runs["eager"], runs["graph"]
    assert set(le) == set(lg)
    for k in le:
        assert abs(le[k] - lg[k]) <= 1e-5 * abs(le[k]) + 1e-7, (k, le[k], lg[k])
    # the first Adam step is lr * g / (|g| + eps) ~ lr * sign(g): the two paths' gradients differ
    # only in atomic summation order, so only elements whose gradient is within rounding of zero
    # may move differently — a small fraction, each by at most 2 lr
    lr = params['LR']
    moved = (dg - de).abs() > 0.1 * lr
    assert float(moved.float().mean()) < 2e-3, float(moved.float().mean())
    assert float((dg - de).abs().max()) <= 2 * lr * 1.001


@pytest.mark.parametrize("case", ["ae_b16", "ae_center_b8", "ae_mssim_b8", "ae_big_b4"])
def test_autoencoder_against_reference(case):
    """Autoencoder (models/autoencoder.py) through the drop-in: reference-keyed state dict (`fc`),
    forward, loss dict (KLD and feature_loss zero), gradients through loss.backward() — the GPU
    MSE kernel for ae_b16, the centre-weighted MSE in torch seeding the HIP backward for
    ae_center_b8 — BN running stats and one torch Adam step, against the reference's golden
    vectors; fp32 parity bars as above."""
    from vae_amd.models import vae_models
    meta, ref = load_case(case)
    sd, x, _ = case_inputs(meta)
    model = vae_models["Autoencoder"](**meta["ctor"], dtype=torch.float32, device="cuda")
    model.load_reference_state_dict(sd)
    assert set(model.state_dict()) == set(sd)
    model.train()
    results = model(x.cuda())
    assert len(results) == 4 and float(results[2].abs().sum()) == 0.0
    losses = model.loss_function(*results, M_N=meta["M_N"], optimizer_idx=0, batch_idx=0)
    assert set(losses) == set(meta["loss"])
    for k, v in meta["loss"].items():
        assert abs(float(losses[k]) - v) <= 1e-4 * abs(v) + 1e-12, (k, float(losses[k]), v)
    n_head = ref["recon_head"].shape[0]
    np.testing.assert_allclose(results[0].detach()[:n_head].cpu().numpy(), ref["recon_head"], rtol=0, atol=1e-4)
    ref_keys = {k: v.clone() for k, v in model.reference_state_dict().items()}   # BN stats after one step
    z = model.encode(x.cuda())[0]
    model.train()
    np.testing.assert_allclose(z.cpu().numpy(), ref["z"], rtol=0, atol=1e-4 * np.abs(ref["z"]).max())
    results = model(x.cuda())                           # encode() above ran its own forward; redo the step's
    losses = model.loss_function(*results, M_N=meta["M_N"], optimizer_idx=0, batch_idx=0)
    model.zero_grad(set_to_none=True)
    losses["loss"].backward()
    flat_grad = model.flat.grad.detach()
    g_all = model.net.layout.export_reference(flat_grad)
    for name in meta["param_names"]:
        if name.endswith(".0.bias") and not name.startswith("final_layer.3"):
            continue
        src = "fc_mu." + name[3:] if name.startswith("fc.") else name
        rs = ref[f"grad_stats/{name}"]
        st = summary(g_all[src])
        bound = 3e-3 if name.endswith(".1.weight") or name.endswith(".1.bias") else 1e-3
        assert abs(st[1] - rs[1]) / max(rs[1], 1e-12) < bound, (name, st, rs)
    for n in ("fc_var.weight", "fc_var.bias"):            # the pinned half gets no gradient
        assert float(g_all[n].abs().max()) == 0.0
    opt = torch.optim.Adam(model.parameters(), lr=meta["lr"])
    opt.step()
    newp = model.reference_state_dict()
    assert float(model.net.reference_state_dict()["fc_var.weight"].abs().max()) == 0.0
    for k in ref:
        if k.startswith("running/"):
            np.testing.assert_allclose(ref_keys[k[8:]].cpu().numpy(), ref[k], rtol=1e-4, atol=1e-6, err_msg=k)
    for name in meta["param_names"]:
        if name.endswith(".0.bias") and not name.startswith("final_layer.3"):
            continue
        gref = ref[f"grad_head/{name}"]
        ok = np.abs(gref) > 1e-5
        np.testing.assert_allclose(newp[name].flatten()[:64].cpu().numpy()[ok], ref[f"new_head/{name}"][ok], rtol=0,
                                   atol=1e-3 * meta["lr"] + 1e-7, err_msg=name)


@pytest.mark.gpu
def test_graph_engine_mixed_batch_sizes_share_one_adam_state():
    """every batch size's TrainStep shares ONE FusedAdam whose moments are the torch
    optimizer's own exp_avg / exp_avg_sq (the partial last batch of an epoch must not start from
    a fresh Adam state).  Four graph steps at B = 16, 8, 16, 8; after each, that step's gradient
    (its plan's grads buffer) drives a torch.optim.Adam on a copy of the parameters (teacher
    forced): parameters and both moments must follow torch's single-state Adam to fp32 rounding.
    (A fresh state on the B = 8 steps would restart bias correction: a ~lr*sign(g) step.)"""
    from vae_amd.experiment import GraphedSteps, VAEXperiment
    from vae_amd.models import vae_models
    kw = dict(in_channels=3, latent_dim=128, dtype=torch.float32, device="cuda", seed=1265)
    params = {'LR': 0.005, 'weight_decay': 0.0, 'kld_weight': 2.5e-4}
    gen = torch.Generator(device="cuda").manual_seed(5)
    xs = [torch.rand(b, 3, 64, 64, device="cuda", generator=gen) for b in (16, 8, 16, 8)]
    batches = [(x, torch.zeros(x.shape[0]), [f"{i}.png" for i in range(x.shape[0])]) for x in xs]
    model = vae_models["VanillaVAE"](**kw)
    model.train()
    exp = VAEXperiment(model, params)
    opt = exp.configure_optimizers()[0]
    ref = model.flat.detach().clone().requires_grad_(True)
    ref_opt = torch.optim.Adam([ref], lr=params['LR'])
    gs = GraphedSteps(exp, opt)
    for i, b in enumerate(batches):
        gs(b, i)
        step = gs.steps[b[0].shape[0]]
        ref.grad = step.plan.grads.detach().clone()
        ref_opt.step()
    torch.cuda.synchronize()
    st = opt.state[model.flat]
    assert int(float(st['step'])) == 4
    assert len(gs.steps) == 2                                       # one TrainStep per batch size ...
    assert all(s.opt is gs.fused for s in gs.steps.values())        # ... sharing one Adam
    assert st['exp_avg'].data_ptr() == gs.fused.m.data_ptr()
    assert st['exp_avg_sq'].data_ptr() == gs.fused.v.data_ptr()
    rs = ref_opt.state[ref]
    torch.testing.assert_close(st['exp_avg'], rs['exp_avg'], rtol=1e-5, atol=1e-9)
    torch.testing.assert_close(st['exp_avg_sq'], rs['exp_avg_sq'], rtol=1e-5, atol=1e-12)
    torch.testing.assert_close(model.flat.detach(), ref.detach(), rtol=1e-5, atol=1e-6)
    gs.flush()


@pytest.mark.parametrize("normalize,size", [(True, 64), (False, 64), (True, 40)])
def test_mssim_dropin_matches_torch_restatement(normalize, size):
    """Autoencoder(use_mssim_loss=True).loss_function on CUDA tensors: 64x64 planes on the HIP MS-SSIM
    kernel (vae_recon_loss) with the module's own `normalize` (the drop-in always used
    normalize=True), other plane sizes (40x40: the pyramid does not halve exactly, the reference's
    avg_pool2d floors it) on the torch restatement instead of an error — loss within 1e-4 and
    dL/drecon within 1e-3 relative of the torch MSSIM (mssim_vae.py:182-282) on the CPU."""
    from vae_amd.models import MSSIM, vae_models
    model = vae_models["Autoencoder"](in_channels=3, latent_dim=128, use_mssim_loss=True, dtype=torch.float32,
                                      device="cuda")
    model.mssim.normalize = normalize
    g = torch.Generator().manual_seed(7)
    x = torch.rand(2, 3, size, size, generator=g)
    r = (x + 0.05 * torch.randn(x.shape, generator=g)).clamp(0, 1)
    rc = r.cuda().requires_grad_(True)
    loss = model.loss_function(rc, x.cuda())["loss"]
    loss.backward()
    ref_mod = MSSIM(3, normalize=normalize)
    rr = r.clone().requires_grad_(True)
    want = ref_mod(rr, x)
    want.backward()
    assert torch.isfinite(want)
    assert abs(float(loss) - float(want)) <= 1e-4 * abs(float(want)) + 1e-7, (float(loss), float(want))
    gd = rc.grad.cpu().double()
    gw = rr.grad.double()
    assert float((gd - gw).norm() / gw.norm()) < 1e-3
