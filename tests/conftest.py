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


def physics_forcing(case, scale: float = 1.0) -> dict:
    """Smooth prescribed physics tendencies for the physics-coupling tests (what physics_get_tend
    hands the dycore, mpas_atm_time_integration.F:424-449): coupled momentum / theta / density
    tendencies and scalar tendencies of typical magnitude, element-major.  The water-vapour
    tendency is negative aloft so that the clip of negative mixing ratios (1642-1644) is exercised."""
    import numpy as np
    K, ns = case["nVertLevels"], case["num_scalars"]
    kk = (np.arange(K) + 0.5) / K
    latc, lonc = case["latCell"][:, None], case["lonCell"][:, None]
    late, lone = case["latEdge"][:, None], case["lonEdge"][:, None]
    f = dict(
        tend_ru_physics=scale * 2e-4 * np.cos(late) * np.sin(2 * lone) * (1 - kk),
        tend_rtheta_physics=scale * 3e-4 * np.cos(latc) ** 2 * np.exp(-3 * kk) * (1 + 0.5 * np.sin(lonc)),
        tend_rho_physics=scale * 1e-7 * np.sin(latc) * np.cos(lonc) * (1 - kk),
    )
    st = np.zeros((case["nCells"], K, ns))
    for i in range(ns):
        st[:, :, i] = scale * 1e-7 * np.cos((i + 1) * latc) * np.sin(lonc + i) * (1 - kk) ** (i + 1)
    st[:, :, 0] -= scale * 5e-7 * kk ** 2  # drying aloft: drives some qv negative -> clipped
    f["scalars_tend"] = st
    return f
