"""Shared pytest setup: the `gpu` marker, repo on sys.path, package import.

`-m "not gpu"` tests need no GPU (oracle vs golden fixtures, host logic, C-ABI
exports); `-m gpu` tests are the HIP parity tests and call through the C-ABI.
"""
import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the libsfmhip kernels")


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(autouse=True)
def _knobs_follow_env():
    """Library knobs are read once per process (sfmhip_knobs_reload re-reads them).
    Autouse and independent of monkeypatch, so this teardown runs after
    monkeypatch has restored the environment: the next test sees the defaults."""
    yield
    abi = sys.modules.get("3d_reconstruction_amd._abi")
    if abi is not None:
        abi.knobs_reload()


@pytest.fixture
def knob(monkeypatch):
    """knob(name, value): set SFMHIP_<name> for this test and reload the library's knobs."""
    def set_knob(name, value):
        monkeypatch.setenv("SFMHIP_" + name, str(value))
        sys.modules["3d_reconstruction_amd._abi"].knobs_reload()
    return set_knob


@pytest.fixture(scope="session")
def sfm():
    """The product package (directory name is not an identifier)."""
    return importlib.import_module("3d_reconstruction_amd")


@pytest.fixture(scope="session")
def gpu(sfm):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test run without a HIP device")
    return torch.device("cuda", 0)
