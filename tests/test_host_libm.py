"""The case builder's C-library loops (csrc/host_libm.c, mpas_dycore/init_atm.py): each array function
equals the C library's scalar function element by element, and _sincos is the library's sincos() --
which the compiled reference uses where it takes sin and cos of one argument, and which differs from
separate sin / cos in the last bit for a small fraction of arguments (the reason the restatement
calls it: tests/test_init_pinned.py)."""
import ctypes
import ctypes.util
import math

import numpy as np
import pytest

from mpas_dycore import init_atm


@pytest.fixture(scope="module")
def x():
    return np.random.default_rng(7).uniform(-7.0, 7.0, 200000)


def test_helper_built():
    assert init_atm._HOST is not None, "csrc/libmpas_host.so not built (__graft_entry__.build)"


def test_array_functions_equal_scalar_library_calls(x):
    u = np.abs(x) / 7.0  # asin / acos domain, pow base
    checks = [(init_atm._exp(x / 4), [math.exp(v) for v in x / 4]),
              (init_atm._tan(x), [math.tan(v) for v in x]),
              (init_atm._asin(u), [math.asin(v) for v in u]),
              (init_atm._acos(u), [math.acos(v) for v in u]),
              (init_atm._pow(u + 0.01, 0.2857142857142857), [math.pow(v + 0.01, 0.2857142857142857) for v in u])]
    for got, want in checks:
        assert np.array_equal(got, np.array(want))


def test_sincos_is_the_library_sincos(x):
    libm = ctypes.CDLL(ctypes.util.find_library("m"))
    libm.sincos.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    s, c = init_atm._sincos(x)
    sv, cv = ctypes.c_double(), ctypes.c_double()
    for i in range(0, x.size, 97):
        libm.sincos(float(x[i]), ctypes.byref(sv), ctypes.byref(cv))
        assert s[i] == sv.value and c[i] == cv.value
    # and it is not the separate functions everywhere: the fused call rounds some arguments
    # differently (measured here: a few per ten thousand)
    sep = np.array([math.sin(v) for v in x]), np.array([math.cos(v) for v in x])
    ndiff = int((s != sep[0]).sum() + (c != sep[1]).sum())
    assert 0 < ndiff < x.size // 100
