"""ctypes binding of ``libacf_apr.so`` (C-ABI declared in ``include/acf_apr.h``).

This is the only route from Python to the HIP kernels.  There is no CPU fallback:
if the library is missing or the machine has no HIP device, every op raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

from . import build_native

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libacf_apr.so")

ACF_OK, ACF_E_INVALID, ACF_E_RANGE, ACF_E_HIP, ACF_E_NOMEM, ACF_E_STATE = range(6)
ABI_VERSION = 2

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_F = ctypes.c_float


class Tables(ctypes.Structure):
    """acf_apr_tables: embedding_P, embedding_Q and their Adagrad slots."""
    _fields_ = [("P", _P), ("Q", _P), ("accP", _P), ("accQ", _P)]


class HParams(ctypes.Structure):
    """acf_apr_hparams (APR.py:86-97 + graph constants)."""
    _fields_ = [
        ("lr", _F), ("eps", _F), ("reg", _F), ("reg_adv", _F), ("clip_lo", _F), ("clip_hi", _F),
        ("adver", _I32), ("adv_mode", _I32), ("seed", _U64), ("zero_delta", _I32),
        ("reserved", _I32),
    ]


# (name, restype, argtypes) for every function declared in include/acf_apr.h
SIGNATURES = {
    "acf_apr_abi_version": (ctypes.c_int, []),
    "acf_apr_last_error": (ctypes.c_char_p, []),
    "acf_apr_build_hash": (ctypes.c_char_p, []),
    "acf_apr_create": (ctypes.c_int, [ctypes.POINTER(_P), _I64, _I64, _I32, _I32, _I32]),
    "acf_apr_destroy": (ctypes.c_int, [_P]),
    "acf_apr_plan": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, _P]),
    "acf_apr_delta_update": (ctypes.c_int, [_P, ctypes.POINTER(Tables), ctypes.POINTER(HParams), _I32, _P]),
    "acf_apr_optimizer_step": (ctypes.c_int, [_P, ctypes.POINTER(Tables), ctypes.POINTER(HParams), _I32, _P]),
    "acf_apr_train_planned": (ctypes.c_int, [_P, ctypes.POINTER(Tables), ctypes.POINTER(HParams), _I32, _I32,
                                             _I32, _P]),
    "acf_apr_train": (ctypes.c_int, [_P, ctypes.POINTER(Tables), ctypes.POINTER(HParams), _P, _P, _P, _I32,
                                     _I32, _I32, _I32, _P]),
    "acf_apr_time_kernels": (ctypes.c_int, [_P, ctypes.POINTER(Tables), ctypes.POINTER(HParams), _I32, _I32,
                                            ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I32), _P]),
    "acf_apr_set_slot_mapping": (ctypes.c_int, [_P, _I32]),
    "acf_apr_set_fusion": (ctypes.c_int, [_P, _I32]),
    "acf_apr_set_plan_mode": (ctypes.c_int, [_P, _I32]),
    "acf_apr_plan_kind": (ctypes.c_int, [_P]),
    "acf_apr_set_stream": (ctypes.c_int, [_P, _I32]),
    "acf_apr_step_errors": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int32), _P]),
    "acf_apr_set_failsafe": (ctypes.c_int, [_P, _I32]),
    "acf_apr_set_spin_limit": (ctypes.c_int, [_P, _I32]),
    "acf_apr_stream_recoveries": (ctypes.c_int, [_P, ctypes.POINTER(_I64)]),
    "acf_apr_resolve": (ctypes.c_int, [_P]),
    "acf_apr_resolve_all": (ctypes.c_int, []),
    "acf_apr_share_failsafe": (ctypes.c_int, [_P, _P]),
    "acf_apr_copy_losses": (ctypes.c_int, [_P, _P, _P, _P]),
    "acf_apr_delta_scatter": (ctypes.c_int, [_P, _P, _P, _P]),
    "acf_bpr_forward": (ctypes.c_int, [_P, _P, _I64, _I64, _I32, _P, _P, _P, _I32, _I32, _F, _F, _P, _P,
                                       _P, _P, _P]),
    "acf_eval_positions_all": (ctypes.c_int, [_P, _P, _I64, _I64, _I32, _P, _P, _I32, _I32, _P, _P, _P,
                                              _P]),
    "acf_eval_positions_all_kernel": (ctypes.c_int, [_P, _P, _I64, _I64, _I32, _P, _P, _I32, _I32, _P, _P, _P,
                                                     _I32, _P]),
    "acf_eval_positions_list": (ctypes.c_int, [_P, _P, _I64, _I64, _I32, _P, _P, _I32, _P, _P, _P, _P]),
    "acf_sample_epoch": (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _I32, _P, _P, _U64, _I32, _I32, _P, _P,
                                        _P, _P]),
    "acf_gather_bpr_fwd_bwd": (ctypes.c_int, [_P, _P, _I64, _I64, _I32, _P, _P, _P, _I64, _F, _F, _P, _P, _P,
                                              _P, _P, _P, _P]),
    "acf_row_segment_sum_workspace": (ctypes.c_int, [_I64, ctypes.POINTER(ctypes.c_size_t)]),
    "acf_row_segment_sum": (ctypes.c_int, [_P, _P, _I64, _I32, _I64, _P, ctypes.c_size_t, _P, _P, _P, _P, _P]),
    "acf_l2norm_perturb": (ctypes.c_int, [_P, _I64, _I32, _F, _P, _P]),
    "acf_sparse_adagrad_apply": (ctypes.c_int, [_P, _P, _I64, _I32, _P, _P, _I64, _F, _P]),
    "acf_sample_epoch_alias": (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _I32, _P, _P, _P, _P, _U64, _I32, _I32,
                                              _P, _P, _P, _P]),
    "acf_alias_build": (ctypes.c_int, [_P, _I64, _P, _P]),
    "acf_dns_select": (ctypes.c_int, [_P, _P, _I64, _I64, _I32, _P, _P, _I64, _I32, _P, _P]),
    "acf_apr_set_shard_mode": (ctypes.c_int, [_P, _I32, _I32]),
    "acf_apr_set_shard_batch": (ctypes.c_int, [_P, _I32]),
    "acf_apr_shard_pass": (ctypes.c_int, [_P, ctypes.POINTER(Tables), ctypes.POINTER(HParams), _I32, _P]),
    "acf_apr_shard_items": (ctypes.c_int, [_P, _I32, _P, _I64, _P]),
    "acf_apr_shard_items_mapped": (ctypes.c_int, [_P, _I32, _P, _P, _I64, _P]),
    "acf_apr_shard_pass_export": (ctypes.c_int, [_P, ctypes.POINTER(Tables), ctypes.POINTER(HParams), _I32, _P, _P,
                                                 _I64, _P]),
    "acf_shard_reduce_delta": (ctypes.c_int, [_P, _P, _P, _I32, _I32, ctypes.POINTER(HParams), _P, _P, _P]),
    "acf_shard_reduce_apply": (ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _I32, ctypes.POINTER(HParams), _P, _P,
                                              _P, _I32, _P]),
}


class NativeError(RuntimeError):
    """A C-ABI call returned an error code."""

    def __init__(self, code: int, func: str, msg: str):
        self.code = code
        super().__init__(f"{func} failed (code {code}): {msg}")


class NativeIndexError(NativeError, IndexError):
    """ACF_E_RANGE: an index outside its table (TF Gather's InvalidArgument)."""


_lib = None
_lock = threading.Lock()


def _open(path: str, name: str, sigs: dict, hash_fn: str, root: str) -> ctypes.CDLL:
    """dlopen a library after checking that it was built from the sources under
    ``root`` as they are now (build_native.verify: ImportError otherwise), and
    check the hash it reports once loaded."""
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: the HIP extension is not built. Run "
            "`python adversarial-collaborative-filtering_amd/build_native.py` "
            "(or __graft_entry__.build()). There is no CPU fallback.")
    build_native.verify(name, path, root)
    lib = ctypes.CDLL(path)
    for fname, (res, args) in sigs.items():
        fn = getattr(lib, fname)
        fn.restype = res
        fn.argtypes = args
    got = getattr(lib, hash_fn)().decode().split("=", 1)[-1]
    if got != build_native.source_hash(name, root):
        raise ImportError(f"{path} reports build hash {got}, not its sources' ({path} was replaced "
                          "after the check?): rebuild it")
    return lib


def load(path: str = LIB_PATH, root: str = build_native.REPO) -> ctypes.CDLL:
    """Load the HIP library (once).  Raises ImportError if it was never built or
    was built from other sources than those under ``root``."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        lib = _open(path, "apr", SIGNATURES, "acf_apr_build_hash", root)
        ver = lib.acf_apr_abi_version()
        if ver != ABI_VERSION:
            raise ImportError(f"libacf_apr ABI {ver} != expected {ABI_VERSION}; rebuild it")
        _lib = lib
        return lib


def call(name: str, *args) -> None:
    """Invoke a C-ABI function and raise NativeError on a non-zero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != ACF_OK:
        call_failed(rc, name)


def call_failed(rc: int, name: str) -> None:
    """Raise the NativeError of a failed C-ABI call (status rc)."""
    msg = load().acf_apr_last_error().decode("utf-8", "replace")
    cls = NativeIndexError if rc == ACF_E_RANGE else NativeError
    raise cls(rc, name, msg)


def exported_symbols(path: str = LIB_PATH) -> set[str]:
    """Names from SIGNATURES that the shared object exports (no GPU needed)."""
    lib = ctypes.CDLL(path)
    return {n for n in SIGNATURES if hasattr(lib, n)}


# --- libacf_neumf.so (include/acf_neumf.h) ------------------------------------
NEUMF_LIB_PATH = os.path.join(PKG_DIR, "lib", "libacf_neumf.so")


class NeuMFHParams(ctypes.Structure):
    """acf_neumf_hparams."""
    _fields_ = [("lr", _F), ("beta1", _F), ("beta2", _F), ("adam_eps", _F), ("eps", _F),
                ("reg_adv", _F), ("adver", _I32), ("reserved", _I32)]


NEUMF_SIGNATURES = {
    "acf_neumf_last_error": (ctypes.c_char_p, []),
    "acf_neumf_build_hash": (ctypes.c_char_p, []),
    "acf_neumf_param_count": (_I64, [_I64, _I64, _I32]),
    "acf_neumf_param_offsets": (ctypes.c_int, [_I64, _I64, _I32, ctypes.POINTER(_I64)]),
    "acf_neumf_create": (ctypes.c_int, [ctypes.POINTER(_P), _I64, _I64, _I32, _I32]),
    "acf_neumf_destroy": (ctypes.c_int, [_P]),
    "acf_neumf_set_rows_in_line": (ctypes.c_int, [_P, _I32]),
    "acf_neumf_set_spin_limit": (ctypes.c_int, [_P, _I32]),
    "acf_neumf_set_failsafe": (ctypes.c_int, [_P, _I32]),
    "acf_neumf_recoveries": (ctypes.c_int, [_P, ctypes.POINTER(_I64)]),
    "acf_neumf_grad": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I32, ctypes.POINTER(NeuMFHParams), _P,
                                      _I32, _P]),
    "acf_neumf_adam": (ctypes.c_int, [_P, _P, _P, _P, _P, _I64, ctypes.POINTER(NeuMFHParams), _P]),
    "acf_neumf_predict": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _P]),
    "acf_neumf_train": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I32, _I64,
                                       ctypes.POINTER(NeuMFHParams), _P, _P]),
    "acf_kbpr_create": (ctypes.c_int, [ctypes.POINTER(_P), _I64, _I64, _I32, _I32]),
    "acf_kbpr_destroy": (ctypes.c_int, [_P]),
    "acf_kbpr_train": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I32, _I64,
                                      ctypes.POINTER(NeuMFHParams), _P, _P]),
    "acf_kbpr_predict": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _P]),
    "acf_amf_param_count": (_I64, [_I64, _I64, _I32]),
    "acf_amf_create": (ctypes.c_int, [ctypes.POINTER(_P), _I64, _I64, _I32, _I32]),
    "acf_amf_destroy": (ctypes.c_int, [_P]),
    "acf_amf_grad": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I32, _P, _P]),
    "acf_amf_train": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I32, _I64,
                                     ctypes.POINTER(NeuMFHParams), _P, _P]),
    "acf_amf_predict": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _P]),
}

_neumf = None


def load_neumf(path: str = NEUMF_LIB_PATH, root: str = build_native.REPO) -> ctypes.CDLL:
    """Load libacf_neumf.so (once).  Raises ImportError if it was never built or
    was built from other sources than those under ``root``."""
    global _neumf
    with _lock:
        if _neumf is not None:
            return _neumf
        _neumf = _open(path, "neumf", NEUMF_SIGNATURES, "acf_neumf_build_hash", root)
        return _neumf


def call_neumf(name: str, *args) -> None:
    lib = load_neumf()
    rc = getattr(lib, name)(*args)
    if rc != ACF_OK:
        msg = lib.acf_neumf_last_error().decode("utf-8", "replace")
        cls = NativeIndexError if rc == ACF_E_RANGE else NativeError
        raise cls(rc, name, msg)


def neumf_exported_symbols(path: str = NEUMF_LIB_PATH) -> set[str]:
    lib = ctypes.CDLL(path)
    return {n for n in NEUMF_SIGNATURES if hasattr(lib, n)}
