"""Native <-> reference state-dict layout (CPU only)."""
import torch

from oracle import vae_oracle as O
from vae_amd.layout import reference_key_order, vanilla_layout


def test_roundtrip_reference_state_dict():
    sd = O.make_params(O.vanilla_param_spec(), 3)
    lay = vanilla_layout(3, 128, [32, 64, 128, 256, 512])
    flat = torch.zeros(lay.total)
    run = torch.zeros(lay.bn_total)
    lay.load_reference(flat, run, sd)
    back = lay.export_reference(flat, run, 0, reference_key_order(3, 128, [32, 64, 128, 256, 512]))
    assert list(back) == list(sd)
    for k in sd:
        assert torch.equal(back[k], sd[k]), k


def test_native_fc_layout_is_nhwc_flatten():
    lay = vanilla_layout(3, 128, [32, 64, 128, 256, 512])
    sd = O.make_params(O.vanilla_param_spec(), 4)
    flat = torch.zeros(lay.total)
    lay.load_reference(flat, torch.zeros(lay.bn_total), sd)
    y = torch.randn(2, 512, 2, 2)
    ref = torch.nn.functional.linear(y.flatten(1), sd["fc_mu.weight"])
    w = lay.view(flat, "fc_mu.weight")
    nat = torch.nn.functional.linear(y.permute(0, 2, 3, 1).reshape(2, -1), w)
    assert torch.allclose(ref, nat, atol=1e-5)
    z = torch.randn(2, 128)
    h_ref = torch.nn.functional.linear(z, sd["decoder_input.weight"], sd["decoder_input.bias"]).view(2, 512, 2, 2)
    h_nat = torch.nn.functional.linear(z, lay.view(flat, "decoder_input.weight"), lay.view(flat, "decoder_input.bias"))
    assert torch.allclose(h_ref.permute(0, 2, 3, 1).reshape(2, -1), h_nat, atol=1e-5)


def test_fused_fc_is_contiguous():
    lay = vanilla_layout(3, 128, [32, 64, 128, 256, 512])
    mu, var = lay.by_name["fc_mu.weight"], lay.by_name["fc_var.weight"]
    assert var.offset == mu.offset + mu.numel
    assert lay.total >= 3937635


def test_vq_layout_matches_reference_spec_and_roundtrips():
    from vae_amd.layout import vq_layout, vq_param_spec
    ospec = O.vq_param_spec()
    assert [(n, tuple(s), k) for n, s, k in ospec] == [(n, tuple(s), k) for n, s, k in vq_param_spec(3, 64, 512, [128, 256])]
    sd = O.make_params(ospec, 5)
    lay = vq_layout(3, 64, 512, [128, 256])
    assert lay.bns == [] and set(p.name for p in lay.params) == set(sd)
    flat = torch.zeros(lay.total)
    lay.load_reference(flat, torch.zeros(0), sd)
    back = lay.export_reference(flat, None, 0, [n for n, _, _ in ospec])
    assert list(back) == list(sd)
    for k in sd:
        assert torch.equal(back[k], sd[k]), k
    # every bias directly follows its weight (default_init draws the bias bound from it)
    names = [p.name for p in lay.params]
    for i, n in enumerate(names):
        if n.endswith(".bias"):
            assert names[i - 1] == n[:-4] + "weight"
