"""The C-ABI library loads and exports every symbol include/mpo.h declares
(CPU-only: no compute calls, only host-side size queries)."""
import ctypes
import os
import re

import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mpo.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mpo_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_functions():
    names = declared_functions()
    assert "mpo_gp_acq_score" in names and "mpo_last_error" in names
    assert len(names) >= 10


def test_library_exports_every_declared_symbol():
    from mpi_opt_amd import _lib

    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), f"libmpo.so lacks {name}"
    # the Python binding declares exactly the header's functions
    assert set(_lib.SIGNATURES) == set(declared_functions())


def test_version_and_host_queries():
    from mpi_opt_amd import _lib

    L = _lib.lib()
    assert L.mpo_version().decode().startswith("mpo ")
    assert L.mpo_gp_prepare_ws_bytes(200, 10) > 200 * 200 * 8 * 2
    assert L.mpo_gp_prepare_ws_bytes(200, 33) == 0      # d > 32 unsupported
    assert L.mpo_gp_prepare_ws_bytes(0, 10) == 0
    m = _lib.MpoGpModel(n=200, d=10, dp=12, np16=208)
    assert L.mpo_gp_score_ws_bytes(ctypes.byref(m), 1_000_000, 5) > 0
    assert L.mpo_gp_score_ws_bytes(ctypes.byref(m), 1_000, 9) == 0  # k > MPO_TOPK_MAX


def test_invalid_arguments_report_errors_without_gpu():
    from mpi_opt_amd import _lib

    L = _lib.lib()
    rc = L.mpo_chol_f64(None, 10, 10, None, None)
    assert rc == 1
    assert b"null" in L.mpo_last_error()
    with pytest.raises(_lib.MpoError):
        _lib.check(rc, "mpo_chol_f64")
