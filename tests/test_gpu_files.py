"""GPU: a dycore started from an MPAS init file (mpas_dycore.mpas_files, netCDF CDF-5) steps to the
same bits as one started from the in-memory case the file was written from (SURVEY.md §8(f)
row 3), on the moist variable-resolution mesh (maxEdges = 7) and the icosahedral one."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(case, nsteps=2):
    from mpas_dycore import Dycore
    dt = 2880.0 if case["nCells"] <= 700 else float(case["dt"])
    dy = Dycore(case, device=0, moist_end=case["num_scalars"])
    dy.init_diagnostics(dt)
    for i in range(nsteps):
        dy.atm_timestep(dt, i + 1)
        dy.shift_time_levels()
    dy.synchronize()
    out = {n: dy.get("state", n, 1) for n in ("u", "w", "theta_m", "rho_zz", "scalars")}
    dy.close()
    return out


@pytest.mark.parametrize("which", ["moist_case", "varres_case_small"])
def test_init_file_run_is_bitwise_equal(which, request, tmp_path):
    from mpas_dycore import mpas_files
    case = request.getfixturevalue(which)
    p = str(tmp_path / "init.nc")
    mpas_files.write_init(p, case, version=5)
    from_file = mpas_files.read_init(p, config=case["config"])
    from_file["dt"] = case.get("dt", 2880.0)
    a, b = _run(case), _run(from_file)
    for n in a:
        assert np.array_equal(a[n], b[n]), n
