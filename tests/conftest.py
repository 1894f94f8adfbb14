"""Shared pytest setup.

Markers: `gpu` = needs an MI355X (run with -m gpu); everything else runs on CPU.
The oracle (oracle/) is imported here only as the checker.
"""
import importlib.util
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")


def load_pkg():
    """Import crlot-dsp_amd/ (hyphenated directory) as module `crlot_dsp_amd`."""
    if "crlot_dsp_amd" in sys.modules:
        return sys.modules["crlot_dsp_amd"]
    path = os.path.join(ROOT, "crlot-dsp_amd", "__init__.py")
    spec = importlib.util.spec_from_file_location("crlot_dsp_amd", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["crlot_dsp_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def pkg():
    return load_pkg()


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


def _npz(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


@pytest.fixture(scope="session")
def ref_tables():
    return _npz("ref_tables.npz")


@pytest.fixture(scope="session")
def kiss_gst():
    return _npz("kiss_gst.npz")


@pytest.fixture(scope="session")
def e2e_gold():
    return _npz("e2e_oracle.npz")


@pytest.fixture(scope="session")
def fq_gold():
    return _npz("fq_oracle.npz")


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch
