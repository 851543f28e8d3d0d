import importlib
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "adversarial-collaborative-filtering_amd"
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def acf():
    return importlib.import_module(PKG)


@pytest.fixture(scope="session")
def ops():
    return importlib.import_module(PKG + ".ops")


@pytest.fixture(scope="session")
def oracle():
    import apr_oracle
    return apr_oracle.COracle()


@pytest.fixture(scope="session")
def dev():
    import torch
    return torch.device("cuda:0")
