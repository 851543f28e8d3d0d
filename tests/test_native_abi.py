"""The C-ABI boundary without a GPU: the library builds for gfx950, loads, and
exports exactly what include/acf_apr.h declares; the product path has no CPU
fallback and never imports the oracle."""
import importlib
import os
import re

import pytest
import torch

from conftest import PKG, REPO

HEADER = os.path.join(REPO, "include", "acf_apr.h")


def header_functions():
    text = open(HEADER).read()
    return set(re.findall(r"^\s*(?:int|const char\*)\s+(acf_\w+)\s*\(", text, re.M))


@pytest.fixture(scope="module")
def native():
    mod = importlib.import_module(PKG + "._native")
    if not os.path.exists(mod.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return mod


def test_header_declares_the_documented_entry_points():
    fns = header_functions()
    assert {"acf_apr_create", "acf_apr_plan", "acf_apr_delta_update", "acf_apr_optimizer_step",
            "acf_apr_train_planned", "acf_bpr_forward", "acf_eval_positions_all",
            "acf_eval_positions_list", "acf_sample_epoch", "acf_dns_select"} <= fns


def test_binding_covers_header(native):
    assert set(native.SIGNATURES) == header_functions()


def test_library_exports_every_header_symbol(native):
    assert native.exported_symbols() == header_functions()
    lib = native.load()
    assert lib.acf_apr_abi_version() == native.ABI_VERSION


def test_library_is_gfx950_code_object(native):
    blob = open(native.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_errors_surface_as_exceptions(native):
    import ctypes
    p = ctypes.c_void_p()
    with pytest.raises(native.NativeError, match="dim"):
        native.call("acf_apr_create", ctypes.byref(p), 10, 10, 6, 4, 1)  # dim 6 unsupported


def test_no_cpu_path(acf):
    ops = importlib.import_module(PKG + ".ops")
    P = torch.zeros(4, 8)
    u = torch.zeros(4, dtype=torch.int32)
    with pytest.raises(ValueError, match="HIP device"):
        ops.bpr_forward(P, P, u, u, u, 4)
    with pytest.raises(TypeError):
        ops.bpr_forward(P.double(), P, u, u, u, 4)


def test_product_never_imports_the_oracle():
    pkg = os.path.join(REPO, PKG)
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(root, f)).read()
                assert "apr_oracle" not in src and "import oracle" not in src, f
