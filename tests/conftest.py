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


_CAPMAN = None


@pytest.fixture(autouse=True, scope="session")
def _capture_manager(request):
    global _CAPMAN
    _CAPMAN = request.config.pluginmanager.getplugin("capturemanager")
    yield


def progress(msg: str):
    """A progress line that bypasses pytest's output capture (and, on a GPU box, is appended to
    gpurun_out/progress.log): long full-size tests stay visibly alive."""
    import time
    line = f"[{time.strftime('%H:%M:%S')}] {msg}"
    if _CAPMAN is not None:
        with _CAPMAN.global_and_fixture_disabled():
            print(line, file=sys.stderr, flush=True)
    else:
        print(line, file=sys.stderr, flush=True)
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", "progress.log"), "a") as f:
            f.write(line + "\n")


class heartbeat:
    """``with heartbeat("what"):`` -- a progress line every ``every`` seconds until the block ends."""

    def __init__(self, what: str, every: float = 30.0):
        self.what, self.every = what, every

    def __enter__(self):
        import threading
        import time
        self.t0 = time.time()
        self.stop = threading.Event()

        def run():
            while not self.stop.wait(self.every):
                progress(f"{self.what}: {time.time() - self.t0:.0f} s")
        self.th = threading.Thread(target=run, daemon=True)
        self.th.start()
        progress(f"{self.what} ...")
        return self

    def __exit__(self, *exc):
        import time
        self.stop.set()
        self.th.join()
        progress(f"{self.what}: done in {time.time() - self.t0:.0f} s")
        return False


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
