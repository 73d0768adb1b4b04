"""Shared pytest setup.

Markers: ``gpu`` -- needs a real MI355X (run with ``-m gpu``); everything else
runs on CPU.  Both the oracle (``oracle/``, test infrastructure) and the host
package (``node-fhe-accelerate_amd/fhe_gpu``) are put on sys.path here.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "node-fhe-accelerate_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs a real MI355X GPU")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def gpu_available():
    import torch

    return torch.cuda.is_available()
