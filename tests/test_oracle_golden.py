"""Pin the CPU oracle (oracle/vae_oracle.py) against the reference's golden vectors.

Both sides are fp32 ATen on CPU, so agreement is near bit-level; the bounds below leave
room only for thread-count-dependent reduction order."""
import numpy as np
import pytest
import torch

from golden_util import CASES, case_inputs, load_case, oracle_kwargs, rel_err, summary
from oracle import vae_oracle as O


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference(case):
    meta, ref = load_case(case)
    sd, x, eps = case_inputs(meta)
    out = O.train_step(meta["arch"], sd, x, eps, **oracle_kwargs(meta))
    for k, v in meta["loss"].items():
        assert abs(out["loss"][k] - v) <= 1e-5 * max(abs(v), 1e-3), (k, out["loss"][k], v)
    recon = out["recon"]
    n_head = ref["recon_head"].shape[0]
    assert rel_err(recon[:n_head].numpy(), ref["recon_head"]) < 1e-5
    flat = recon.reshape(-1, recon[0].numel() if meta["arch"] != "IWAE" else recon[0, 0].numel()).double()
    np.testing.assert_allclose(flat.sum(1).numpy(), ref["recon_sum"], rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(out["per_img_mse"].numpy(), ref["per_img_mse"], rtol=1e-5)
    if "mu" in ref:
        assert rel_err(out["mu"].numpy(), ref["mu"]) < 1e-5
        assert rel_err(out["log_var"].numpy(), ref["log_var"]) < 1e-5
    if meta["arch"] == "IWAE":
        np.testing.assert_allclose(out["log_weight"].numpy(), ref["log_weight"], rtol=1e-5)
        np.testing.assert_allclose(out["weight"].numpy(), ref["weight"], rtol=1e-4, atol=1e-7)
    if meta["arch"] == "Autoencoder":
        assert rel_err(out["z"].numpy(), ref["z"]) < 1e-5
    if meta["arch"] == "VQVAE":
        sure = ref["gap"] > 1e-6
        assert np.array_equal(out["indices"].numpy()[sure], ref["indices"][sure])
    for name in meta["param_names"]:
        g = out["grads"][name]
        st = summary(g)
        ref_st = ref[f"grad_stats/{name}"]
        scale = max(ref_st[1], 1e-12)
        assert abs(st[1] - ref_st[1]) <= 1e-4 * scale + 1e-12, (name, st, ref_st)
        np.testing.assert_allclose(g.flatten()[:64].numpy(), ref[f"grad_head/{name}"],
                                   rtol=1e-3, atol=1e-4 * ref_st[2] + 1e-12)
        p = out["new_params"][name]
        np.testing.assert_allclose(p.flatten()[:64].numpy(), ref[f"new_head/{name}"], rtol=1e-5, atol=1e-6)
    for k, v in out["running"].items():
        np.testing.assert_allclose(v.numpy(), ref[f"running/{k}"], rtol=1e-5, atol=1e-6)


def test_recipe_is_deterministic():
    a = O.make_params(O.vanilla_param_spec(), 7)
    b = O.make_params(O.vanilla_param_spec(), 7)
    assert all(torch.equal(a[k], b[k]) for k in a)
    assert sum(t.numel() for k, t in a.items() if not k.endswith("num_batches_tracked")) == 3937635 + 2 * 1504
