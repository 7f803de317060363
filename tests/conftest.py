import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import helpers as H  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: larger sizes")


@pytest.fixture(scope="session")
def oracle():
    return H.Oracle()


@pytest.fixture(scope="session")
def fixtures():
    return H.load_npz(os.path.join(H.GOLDEN, "fixtures.npz"))


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(H.GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def ctx():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test without a visible HIP device")
    import combblas_amd as cb

    c = cb.Context(0)
    yield c
    torch.cuda.synchronize()
    c.close()


@pytest.fixture(scope="session")
def apps():
    return H.load_npz(os.path.join(H.GOLDEN, "apps.npz"))


@pytest.fixture(scope="session")
def apps_meta():
    with open(os.path.join(H.GOLDEN, "apps.json")) as f:
        return json.load(f)
