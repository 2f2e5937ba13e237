import json
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a MI355X (HIP) device; parity tests of the gfx950 kernels")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden_kernels():
    from safetensors.torch import load_file
    return load_file(os.path.join(GOLDEN, "kernels.safetensors"))


@pytest.fixture(scope="session")
def golden_layouts():
    with open(os.path.join(GOLDEN, "bucket_layouts.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_loss():
    with open(os.path.join(GOLDEN, "loss_curve_tiny.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_init_fp():
    with open(os.path.join(GOLDEN, "tiny_init_fingerprint.json")) as f:
        return json.load(f)


def rel_l2(a, b):
    a = a.double()
    b = b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def max_abs(a, b):
    return float((a.double() - b.double()).abs().max())
