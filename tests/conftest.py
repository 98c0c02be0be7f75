import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mpas-model_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def rel_linf(a, b):
    import numpy as np
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.max(np.abs(b))
    if den == 0.0:
        return float(np.max(np.abs(a - b)))
    return float(np.max(np.abs(a - b)) / den)


@pytest.fixture(scope="session")
def small_case():
    from mpas_dycore.mesh import build_mesh
    from mpas_dycore.init_atm import build_case
    m = build_mesh(3, lloyd_iters=20)
    return build_case(m, K=26, ns=1)


@pytest.fixture(scope="session")
def moist_case():
    from mpas_dycore.cases import jw_case
    return jw_case(642, K=26, ns=3, moist=True, cache=False)


@pytest.fixture(scope="session")
def varres_case_small():
    """Variable-resolution SCVT (4x refinement, pentagons/hexagons/heptagons, maxEdges=7)."""
    from mpas_dycore.cases import varres_case
    return varres_case(2562, ratio=4.0, K=26, ns=3, moist=True, lloyd_iters=30, cache=False)
