"""Shared pytest setup.

Markers: `gpu` — needs a ROCm device (run on the MI355X box with `-m gpu`).
Paths: the repo root (oracle/, bench helpers) and the drop-in root
retinex-image-enhancement_amd/ (models/, enhancers/, upr/) go on sys.path,
the same way the reference is used from its own root directory.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "retinex-image-enhancement_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires a ROCm (MI355X) device")


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name))
    return load
