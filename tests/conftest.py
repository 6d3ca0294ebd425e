import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ace-step-1.5_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long CPU test")


def load_golden(name):
    from safetensors.torch import load_file
    return load_file(os.path.join(GOLDEN, name + ".safetensors"))


def golden_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def rel_l2(a, b):
    a = a.double().flatten()
    b = b.double().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def cosine(a, b):
    a = a.double().flatten()
    b = b.double().flatten()
    return float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-30))


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def set_knob(monkeypatch, name, value):
    """Set one ACEHIP_* A/B switch for this test: the library reads its knobs once, so the
    environment change is followed by acehip_reload_knobs (undone by the next test's reload)."""
    from acehip import _ffi
    monkeypatch.setenv(name, str(value))
    _ffi.reload_knobs()


@pytest.fixture(autouse=True)
def _fresh_knobs():
    """Every test starts from the knobs of the (restored) environment."""
    from acehip import _ffi
    if _ffi._LIB is not None:
        _ffi.reload_knobs()
    yield
