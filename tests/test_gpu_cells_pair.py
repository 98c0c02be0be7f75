"""The pair-layout acoustic cell phase (k_acoustic_cells_p: two cells per wavefront, 16-byte column
loads, two-level lane-shift tridiagonal sweeps; MPAS_DYCORE_CELLS_PAIR=1) evaluates
atm_advance_acoustic_step's cell loop (mpas_atm_time_integration.F:2600-2723) in the same operation
order as the one-column kernel, so it must reproduce its bits -- on the reference acoustic fixture,
over whole moist monotone steps (maxEdges 6 and 7) and through decomposed blocks."""
import os

import numpy as np
import pytest

from test_gpu_kernels import POST, _fixture_dycore

pytestmark = pytest.mark.gpu


class _env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.saved = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_pair_cells_bitwise_vs_reference_fixture():
    """Three fused sub-steps (none a stage's last, so the pair kernel runs) equal the one-column
    kernel bit for bit, and one sub-step equals the reference fixture bit for bit."""
    outs = []
    for flag in ("0", "1"):
        with _env(MPAS_DYCORE_CELLS_PAIR=flag):
            z, dy = _fixture_dycore()
        dy.time_acoustic_step(float(z["dts"]), small_step=int(z["small_step"]), reps=3)
        dy.synchronize()
        outs.append({n: dy.get("diag", n) for n in POST})
        dy.close()
    for n in POST:
        assert np.array_equal(outs[0][n], outs[1][n]), n
    with _env(MPAS_DYCORE_CELLS_PAIR="1"):
        z, dy = _fixture_dycore()
    dy.time_acoustic_step(float(z["dts"]), small_step=int(z["small_step"]), reps=1)
    dy.synchronize()
    for n in POST:
        got = dy.get("diag", n).reshape(z["post_diag." + n].shape)
        nd = int(np.count_nonzero(got != z["post_diag." + n]))
        assert nd == 0, f"{n}: {nd} values differ"
    dy.close()


def _steps(case, flag, nsteps=3, dt=2880.0):
    from mpas_dycore import Dycore
    with _env(MPAS_DYCORE_CELLS_PAIR=flag, MPAS_DYCORE_KERNELS="pair"):
        dy = Dycore(case, device=0, moist_end=case["num_scalars"])
    dy.init_diagnostics(dt)
    for i in range(nsteps):
        dy.atm_timestep(dt, i + 1)
        dy.shift_time_levels()
    dy.synchronize()
    out = {n: dy.get("state", n, 1) for n in ("u", "w", "theta_m", "rho_zz", "scalars")}
    out.update({n: dy.get("diag", n) for n in ("rho_pp", "rtheta_pp", "rw_p", "ruAvg", "wwAvg", "exner")})
    dy.close()
    return out


@pytest.mark.parametrize("which", ["moist_case", "varres_case_small"])
def test_pair_cells_whole_steps_bitwise(which, request):
    case = request.getfixturevalue(which)
    dt = float(case["dt"]) if which == "varres_case_small" else 2880.0
    ref = _steps(case, "0", dt=dt)
    got = _steps(case, "1", dt=dt)
    for n in ref:
        assert np.array_equal(got[n], ref[n]), n
