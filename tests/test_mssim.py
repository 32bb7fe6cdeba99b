"""The Autoencoder's MSSIM reconstruction loss (models/mssim_vae.py:182-282, used by
models/autoencoder.py:266-267 when use_mssim_loss) — CPU: the product's torch restatement
(vae_amd.models.MSSIM) against the oracle's (oracle.vae_oracle.mssim_loss), which
tests/test_oracle_golden.py pins to the reference's own MSSIM through the ae_mssim_b8 fixture
(loss value and every gradient of one training step)."""
import torch

from oracle import vae_oracle as O
from vae_amd.models import MSSIM


def test_mssim_value_and_gradient_match_the_oracle():
    g = torch.Generator().manual_seed(7)
    a = (torch.rand(4, 3, 64, 64, generator=g) * 2 - 1).requires_grad_(True)
    b = torch.rand(4, 3, 64, 64, generator=g) * 2 - 1
    a2 = a.detach().clone().requires_grad_(True)
    v = MSSIM(3)(a, b)
    w = O.mssim_loss(a2, b)
    assert abs(float(v) - float(w)) <= 1e-6 * abs(float(w))
    v.backward()
    w.backward()
    torch.testing.assert_close(a.grad, a2.grad, rtol=1e-5, atol=1e-9)


def test_mssim_of_identical_images_is_zero_and_window_is_the_reference_one():
    x = torch.rand(2, 3, 64, 64)
    assert abs(float(MSSIM(3)(x, x))) < 1e-6
    win = MSSIM(3)._window[0, 0]
    # mssim_vae.py:205-209: exp(+(i - 5)^2 / 4.5), normalised — largest at the window's edges
    assert float(win[0, 0]) > float(win[5, 5]) and abs(float(win.sum()) - 1.0) < 1e-6
