"""The C-ABI library loads and exports every entry point declared in include/mpas_dycore.h
(no compute calls: there is no GPU in the build container)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mpas_dycore.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(mpas_dyc_[a-z_]+)\s*\(", src)))


def test_header_declares_boundary():
    fns = declared_functions()
    for required in ("mpas_dyc_create", "mpas_dyc_timestep", "mpas_dyc_init_diagnostics",
                     "mpas_dyc_shift_time_levels", "mpas_dyc_set_field", "mpas_dyc_get_field"):
        assert required in fns


def test_library_exports_every_declared_symbol():
    from mpas_dycore import _lib
    if not os.path.isfile(_lib.LIBPATH):
        pytest.skip("libmpas_dycore.so not built (__graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIBPATH)
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert set(_lib.EXPORTS) <= set(declared_functions())


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from mpas_dycore import _lib
    monkeypatch.setattr(_lib, "LIBPATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(RuntimeError):
        _lib.load()
