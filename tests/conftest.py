"""Shared test setup: marker registration and import paths.

``-m "not gpu"`` tests run anywhere (oracle vs golden vectors, C-ABI export
surface, host logic, gloo multi-process); ``-m gpu`` tests call the HIP
engine through the C-ABI on a real MI355X and compare with the oracle.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "fm-index-constrained-decoding_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden_index_cases():
    import json

    with open(os.path.join(GOLDEN, "index_cases.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def golden_dir():
    import pathlib

    return pathlib.Path(GOLDEN)
