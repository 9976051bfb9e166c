"""ctypes binding of ``libmpo.so`` (the C ABI declared in ``include/mpo.h``).

The product path has no CPU fallback: if the library is missing or a HIP call
fails, :func:`lib` / :func:`check` raise.  Device buffers are torch tensors;
only their ``data_ptr()`` and the raw HIP stream handle cross the ABI.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmpo.so")

MPO_OK = 0
MPO_ACQ_EI = 1
MPO_ACQ_PI = 2
MPO_ACQ_LCB = 4
MPO_TOPK_MAX = 8
ACQ_FLAGS = {"EI": MPO_ACQ_EI, "PI": MPO_ACQ_PI, "LCB": MPO_ACQ_LCB}
# MpoCnnSpec.options: option3's --loss / --optimizer (include/mpo.h MPO_LOSS_* | MPO_OPT_*)
LOSS_CODES = {"binary_crossentropy": 0x0, "categorical_crossentropy": 0x1}
OPT_CODES = {"adam": 0x000, "sgd": 0x100}
ACQ_ROW = {"EI": 0, "PI": 1, "LCB": 2}


class MpoError(RuntimeError):
    pass


class MpoGpModel(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int32), ("d", ctypes.c_int32), ("dp", ctypes.c_int32), ("np16", ctypes.c_int32),
        ("amp", ctypes.c_double), ("y_mean", ctypes.c_double), ("y_std", ctypes.c_double),
        ("xs", ctypes.c_void_p), ("ls", ctypes.c_void_p), ("alpha", ctypes.c_void_p),
        ("wfrag", ctypes.c_void_p), ("L", ctypes.c_void_p), ("W", ctypes.c_void_p),
        ("info", ctypes.c_void_p), ("wmeta", ctypes.c_void_p), ("xb", ctypes.c_void_p),
    ]


class MpoLbfgsbOptions(ctypes.Structure):
    _fields_ = [("ftol", ctypes.c_double), ("gtol", ctypes.c_double), ("maxiter", ctypes.c_int32),
                ("maxfun", ctypes.c_int32), ("maxcor", ctypes.c_int32), ("maxls", ctypes.c_int32)]


#: objective callback of mpo_lbfgsb_batched (tests drive the host L-BFGS-B with it)
FG_BATCH_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                               ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double),
                               ctypes.POINTER(ctypes.c_double), ctypes.c_void_p)


class MpoCnnSpec(ctypes.Structure):
    _fields_ = [("nb_filters", ctypes.c_int32), ("kernel_size", ctypes.c_int32), ("pool_size", ctypes.c_int32),
                ("dense", ctypes.c_int32), ("lr", ctypes.c_float), ("dropout", ctypes.c_float),
                ("seed", ctypes.c_uint32), ("options", ctypes.c_int32)]


class MpoPopSizes(ctypes.Structure):
    _fields_ = [("n_params", ctypes.c_int64), ("act_floats", ctypes.c_int64), ("table_bytes", ctypes.c_int64),
                ("n_members", ctypes.c_int32), ("batch", ctypes.c_int32)]


class MpoDnArch(ctypes.Structure):
    _fields_ = [("H", ctypes.c_int32), ("W", ctypes.c_int32), ("C", ctypes.c_int32), ("classes", ctypes.c_int32),
                ("depth", ctypes.c_int32), ("nb_dense_block", ctypes.c_int32), ("growth", ctypes.c_int32),
                ("nb_filter", ctypes.c_int32)]


class MpoDnSizes(ctypes.Structure):
    _fields_ = [("n_params", ctypes.c_int64), ("n_state", ctypes.c_int64), ("act_floats", ctypes.c_int64),
                ("n_members", ctypes.c_int32), ("batch", ctypes.c_int32), ("n_layers", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_D = ctypes.c_double
_SZ = ctypes.c_size_t
_U = ctypes.c_uint

# name -> (restype, argtypes); keep in the order of include/mpo.h
SIGNATURES = {
    "mpo_last_error": (ctypes.c_char_p, []),
    "mpo_version": (ctypes.c_char_p, []),
    "mpo_gp_kernel_matrix": (_I, [_P, _I, _I, _P, _D, _D, _P, _I, _P]),
    "mpo_chol_f64": (_I, [_P, _I, _I, _P, _P]),
    "mpo_trsm_f64": (_I, [_P, _I, _I, _P, _I, _I, _I, _P]),
    "mpo_gp_prepare_ws_bytes": (_SZ, [_I, _I]),
    "mpo_gp_prepare": (_I, [_P, _P, _I, _I, _P, _D, _D, _D, _D, ctypes.POINTER(MpoGpModel), _P, _SZ, _P]),
    "mpo_gp_lml_ws_bytes": (_SZ, [_I, _I, _I]),
    "mpo_gp_lml_grad": (_I, [_P, _P, _I, _I, _P, _I, _P, _P, _P, _P, _SZ, _P]),
    "mpo_gp_lml_io_bytes": (_SZ, [_I, _I]),
    "mpo_gp_lml_grad_host": (_I, [_P, _P, _I, _I, _P, _I, _P, _P, _SZ, _P, _SZ, _P]),
    "mpo_gp_score_ws_bytes": (_SZ, [ctypes.POINTER(MpoGpModel), _I64, _I]),
    "mpo_gp_acq_score": (_I, [ctypes.POINTER(MpoGpModel), _P, _I64, _D, _D, _D, _U, _P, _P, _P, _I, _P, _P,
                              _P, _SZ, _P]),
    "mpo_gp_ei_score": (_I, [ctypes.POINTER(MpoGpModel), _P, _I64, _D, _D, _P, _P, _P, _P, _P, _SZ, _P]),
    "mpo_gp_acq_grad": (_I, [ctypes.POINTER(MpoGpModel), _P, _I, _P, _D, _D, _D, _P, _P, _P]),
    "mpo_gp_acq_grad_host": (_I, [ctypes.POINTER(MpoGpModel), _P, _I, _P, _D, _D, _D, _P, _P, _P]),
    "mpo_lbfgsb_batched": (_I, [_I, _I, _P, _P, ctypes.POINTER(MpoLbfgsbOptions), FG_BATCH_FN, _P, _P, _P, _P,
                                _P]),
    "mpo_gp_lml_batcher_create": (_I, [_I, ctypes.POINTER(ctypes.c_void_p)]),
    "mpo_gp_lml_batcher_destroy": (_I, [_P]),
    "mpo_gp_lml_batcher_stats": (_I, [_P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "mpo_gp_fit_lml_host": (_I, [_P, _P, _I, _I, _P, _I, _P, ctypes.POINTER(MpoLbfgsbOptions), _P, _P, _P, _SZ, _P,
                                 _SZ, _P, _P, _P, _P, _P, _P]),
    "mpo_gp_polish_host": (_I, [ctypes.POINTER(MpoGpModel), _P, _P, _I, _P, ctypes.POINTER(MpoLbfgsbOptions), _D,
                                _D, _D, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "mpo_pop_create": (_I, [ctypes.POINTER(MpoCnnSpec), _I, _I, ctypes.POINTER(ctypes.c_void_p)]),
    "mpo_pop_destroy": (_I, [_P]),
    "mpo_pop_sizes": (_I, [_P, ctypes.POINTER(MpoPopSizes)]),
    "mpo_pop_param_layout": (_I, [_P, _I, ctypes.POINTER(ctypes.c_int64)]),
    "mpo_pop_act_layout": (_I, [_P, _I, ctypes.POINTER(ctypes.c_int64)]),
    "mpo_pop_bind": (_I, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "mpo_pop_train_step": (_I, [_P, _P, _P, _P, _I64, _I64, ctypes.c_int32, _P, _P]),
    "mpo_pop_eval_step": (_I, [_P, _P, _P, _P, _I64, _I64, _P, _P, _P]),
    "mpo_pop_profile": (_I, [_P, _P, _SZ, _I]),
    "mpo_dn_create": (_I, [ctypes.POINTER(MpoDnArch), _I, _I, ctypes.POINTER(ctypes.c_void_p)]),
    "mpo_dn_destroy": (_I, [_P]),
    "mpo_dn_sizes": (_I, [_P, ctypes.POINTER(MpoDnSizes)]),
    "mpo_dn_layer": (_I, [_P, _I, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)]),
    "mpo_dn_bind": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "mpo_dn_train_step": (_I, [_P, _P, _P, _P, _I64, _I64, ctypes.c_int32, _P, _P]),
    "mpo_dn_eval_step": (_I, [_P, _P, _P, _P, _I64, _I64, _P, _P, _P]),
    "mpo_dn_penalty": (_I, [_P, _P, _P]),
    "mpo_kfold_gather": (_I, [_P, _P, _I64, _I, _P, _P]),
}

_LIB = None


def lib():
    """Load libmpo.so (once).  Raises if it has not been built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise MpoError(f"{LIB_PATH} is missing: build it with `make -C mpi_opt_amd/csrc` "
                           "or `python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback)")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = handle
    return _LIB


def check(rc: int, what: str = "mpo call"):
    if rc != MPO_OK:
        msg = lib().mpo_last_error()
        raise MpoError(f"{what} failed (status {rc}): {msg.decode() if msg else ''}")


def ptr(t) -> int:
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


_BATCHERS = {}
_BATCHERS_LOCK = __import__("threading").Lock()


def lml_batcher(device_index: int):
    """The process-wide LML round batcher of one GPU (mpo_gp_lml_batcher_create),
    shared by every refit on that device; lives as long as the process."""
    with _BATCHERS_LOCK:
        h = _BATCHERS.get(device_index)
        if h is None:
            out = ctypes.c_void_p()
            check(lib().mpo_gp_lml_batcher_create(int(device_index), ctypes.byref(out)), "mpo_gp_lml_batcher_create")
            h = _BATCHERS[device_index] = out.value
        return h


def stream_handle(device=None) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream
