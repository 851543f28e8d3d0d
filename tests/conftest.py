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


@pytest.fixture(scope="session")
def fp32_parity():
    """Multi-step fp32 parity bar: every element within 1e-5
    absolute of the oracle (scaled by max(1, max|want|)), and at most a 1e-5
    fraction (>= 2 elements) outside rtol 1e-5 / atol 1e-6.  Single steps are
    held to rtol 1e-5 / atol 1e-6 outright; this bar is for results after many
    steps, where the adversarial map amplifies summation-order rounding in rows
    whose clean gradient nearly cancels."""
    import numpy as np

    def check(got, want, name):
        got = got.detach().cpu().numpy() if hasattr(got, "detach") else np.asarray(got)
        err = np.abs(got.astype(np.float64) - want)
        scale = max(1.0, float(np.abs(want).max()))
        assert float(err.max()) <= 1e-5 * scale, f"{name}: max abs diff {err.max():.3e}"
        bad = int((err > 1e-6 + 1e-5 * np.abs(want)).sum())
        assert bad <= max(2, int(1e-5 * want.size)), f"{name}: {bad} of {want.size} elements outside 1e-5"
    return check
