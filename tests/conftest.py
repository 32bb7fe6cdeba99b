"""pytest config: the `gpu` marker and import paths.

`-m "not gpu"` runs here (no GPU): oracle vs golden vectors, host logic, C-ABI symbol
checks, gloo multi-rank tests.  `-m gpu` runs on an MI355X and calls the HIP kernels
through the C ABI.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "pytorch-vae_amd")
for p in (REPO, PKG_ROOT, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
