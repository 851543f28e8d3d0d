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


NEUMF_HEADER = os.path.join(REPO, "include", "acf_neumf.h")


def neumf_header_functions():
    text = open(NEUMF_HEADER).read()
    return set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(acf_\w+)\s*\(", text, re.M))


def test_neumf_library_exports_every_header_symbol(native):
    assert set(native.NEUMF_SIGNATURES) == neumf_header_functions()
    assert native.neumf_exported_symbols() == neumf_header_functions()
    assert b"gfx950" in open(native.NEUMF_LIB_PATH, "rb").read()


def test_neumf_layout_matches_keras_shapes(native):
    """The flat buffer holds the ten Keras tensors in order, 16-B aligned (host-only calls)."""
    import ctypes
    import numpy as np
    import neumf_oracle as N
    U1, I1, d = 31, 17, 12
    lib = native.load_neumf()
    off = (ctypes.c_int64 * 10)()
    native.call_neumf("acf_neumf_param_offsets", U1, I1, d, off)
    sizes = [int(np.prod(s)) for s in N.shapes(U1, I1, d).values()]
    assert list(off) == list(np.concatenate([[0], np.cumsum(sizes)[:-1]]))
    assert all(o % 4 == 0 for o in off)
    assert lib.acf_neumf_param_count(U1, I1, d) == off[9] + 4
    assert lib.acf_neumf_param_count(U1, I1, 6) == -1  # dim must be a multiple of 4


def test_product_never_imports_the_neumf_oracle():
    pkg = os.path.join(REPO, PKG)
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(root, f)).read()
                assert not re.search(r"^\s*(from|import)\s+\S*neumf_oracle", src, re.M), f


def test_torch_custom_ops_register():
    """lib/libacf_torch.so registers every acf:: op of SURVEY §8(b) (loads without a GPU)."""
    import importlib
    tops = importlib.import_module("adversarial-collaborative-filtering_amd.torch_ops")
    acf = tops.load()
    for name in tops.OPS:
        assert hasattr(acf, name), name
    schema = str(acf.bpr_apr_step.default._schema)
    assert "Tensor(a!) P" in schema and "-> (Tensor loss_clean, Tensor loss_adv, Tensor n_correct)" in schema


def test_torch_custom_ops_refuse_cpu_tensors():
    import importlib
    import torch
    acf = importlib.import_module("adversarial-collaborative-filtering_amd.torch_ops").load()
    with pytest.raises(Exception):
        acf.l2norm_perturb(torch.zeros(2, 8), 0.5)


def test_alias_table_reproduces_the_weights():
    """acf_alias_build (Vose, host): the column probabilities of the table sum
    back to w / sum(w) for every item, and each column is a valid (prob, alias)."""
    import importlib
    import numpy as np
    ops = importlib.import_module(PKG + ".ops")
    rng = np.random.default_rng(1)
    for w in (rng.gamma(0.5, size=1000), np.ones(17), np.r_[np.zeros(5), rng.random(20)], (np.arange(1, 300) ** -1.0)):
        w = w.astype(np.float32)
        prob, alias = ops.alias_table(w)
        n = len(w)
        assert ((prob >= 0) & (prob <= 1)).all() and ((alias >= 0) & (alias < n)).all()
        p = prob.astype(np.float64) / n
        np.add.at(p, alias, (1.0 - prob.astype(np.float64)) / n)
        np.testing.assert_allclose(p, w / w.astype(np.float64).sum(), atol=1e-6)
    with pytest.raises(Exception):
        ops.alias_table(np.zeros(4, np.float32))
