"""vae_amd — MI355X-native VAE training step (drop-in for bplaut/PyTorch-VAE's hot path).

Importing the package does not touch the GPU; the HIP library is loaded on first use and
there is no fallback when it is missing.
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
