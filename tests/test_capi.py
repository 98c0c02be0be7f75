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
    return sorted(set(re.findall(r"\b(mpas_dyc_[a-z0-9_]+)\s*\(", src)))


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


def test_four_builds_are_dispatched_by_level_count():
    """The library links four builds of dycore.hip (one wavefront per column up to
    MPAS_DYC_MAX_LEVELS_WAVE levels, one 128-lane workgroup per column up to
    MPAS_DYC_MAX_LEVELS_WIDE, one 256-lane workgroup up to MPAS_DYC_MAX_LEVELS_256, one 512-lane
    workgroup up to MPAS_DYC_MAX_LEVELS): the public entry
    points (api_dispatch.cpp) and the builds' renames (api_rename.h) are generated from the header and
    up to date, every public function forwards to the builds, and every build is in the library."""
    import subprocess
    import sys
    gen = os.path.join(ROOT, "mpas-model_amd", "csrc", "gen_api.py")
    r = subprocess.run([sys.executable, gen, "--check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    src = open(HEADER).read()
    assert int(re.search(r"#define MPAS_DYC_MAX_LEVELS_WAVE (\d+)", src).group(1)) == 63
    assert int(re.search(r"#define MPAS_DYC_MAX_LEVELS_WIDE (\d+)", src).group(1)) == 127
    assert int(re.search(r"#define MPAS_DYC_MAX_LEVELS_256 (\d+)", src).group(1)) == 255
    assert int(re.search(r"#define MPAS_DYC_MAX_LEVELS (\d+)", src).group(1)) == 511
    disp = open(os.path.join(ROOT, "mpas-model_amd", "csrc", "api_dispatch.cpp")).read()
    for f in declared_functions():
        assert re.search(rf"\b{f}\(", disp), f
    from mpas_dycore import _lib
    if not os.path.isfile(_lib.LIBPATH):
        pytest.skip("libmpas_dycore.so not built (__graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIBPATH)
    for tag in ("n", "w", "x", "y"):
        missing = [f for f in declared_functions() if not hasattr(lib, f.replace("mpas_dyc_", f"mpas_dyc{tag}_"))]
        assert not missing, (tag, missing)
