"""The drop-in's Python surface mirrors the reference's models package (no GPU needed)."""
import inspect

import pytest


def test_registry_names_and_aliases_mirror_reference():
    from vae_amd import models as M
    # models/__init__.py:35-56 (22 names) and :29-33 aliases
    names = {'HVAE', 'LVAE', 'IWAE', 'SWAE', 'MIWAE', 'VQVAE', 'DFCVAE', 'DIPVAE', 'BetaVAE', 'InfoVAE', 'WAE_MMD',
             'VampVAE', 'GammaVAE', 'MSSIMVAE', 'JointVAE', 'BetaTCVAE', 'FactorVAE', 'Autoencoder', 'LogCoshVAE',
             'VanillaVAE', 'ConditionalVAE', 'CategoricalVAE'}
    assert set(M.vae_models) == names
    assert M.VAE is M.VanillaVAE and M.GaussianVAE is M.VanillaVAE
    for name in ('VanillaVAE', 'BetaVAE', 'IWAE', 'VQVAE'):
        assert issubclass(M.vae_models[name], M.BaseVAE)


def test_families_off_the_path_fail_loudly():
    from vae_amd import models as M
    with pytest.raises(NotImplementedError):
        M.vae_models['WAE_MMD'](in_channels=3, latent_dim=128)


def test_constructor_kwargs_match_reference():
    from vae_amd import models as M
    # the YAML model_params of configs/vae/{vae,bhvae,iwae}.yaml pass straight through
    p = inspect.signature(M.BetaVAE.__init__).parameters
    for k in ('in_channels', 'latent_dim', 'hidden_dims', 'beta', 'gamma', 'max_capacity', 'Capacity_max_iter',
              'loss_type'):
        assert k in p
    assert 'num_samples' in inspect.signature(M.IWAE.__init__).parameters
    assert list(inspect.signature(M.VanillaVAE.forward).parameters)[:2] == ['self', 'input']
    q = inspect.signature(M.VQVAE.__init__).parameters
    for k in ('in_channels', 'embedding_dim', 'num_embeddings', 'hidden_dims', 'beta', 'img_size'):
        assert k in q                                   # configs/vae/vq_vae.yaml model_params
