"""The oracle is pinned to the reference: the C restatement (oracle/c) reproduces the
reference acoustic sub-step bit for bit on the committed fixture, and the compiled
reference itself reproduces the committed trajectories (when it is built here)."""
import os

import numpy as np
import pytest

from conftest import rel_linf

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _acoustic_fixture():
    z = np.load(os.path.join(GOLD, "acoustic_x1.162_K16.npz"))
    mesh = {k[5:]: z[k] for k in z.files if k.startswith("mesh_")}
    mesh.update(nCells=int(z["nCells"]), nEdges=int(z["nEdges"]), K=int(z["K"]), maxEdges=int(z["maxEdges"]))
    pre = {k[4:]: z[k] for k in z.files if k.startswith("pre_")}
    post = {k[5:]: z[k] for k in z.files if k.startswith("post_")}
    return z, mesh, pre, post


def port_inputs(pre):
    m = {"state.theta_m.tl1": "theta_m", "state.rho_zz.tl2": "rho_zz", "state.w.tl2": "w", "tend.u": "tend_ru",
         "tend.rho_zz": "tend_rho", "tend.theta_m": "tend_rt", "tend.w": "tend_rw"}
    return {m.get(k, k.split(".", 1)[1]): v for k, v in pre.items()}


def test_port_acoustic_bitwise_vs_reference():
    from oracle import port
    if not port.available():
        pytest.skip("oracle/_ref/libatm_port.so not built (make -C oracle port)")
    z, mesh, pre, post = _acoustic_fixture()
    f = port_inputs(pre)
    out = port.acoustic_substep(mesh, f, float(z["dts"]), int(z["small_step"]), float(z["epssm"]),
                                float(z["smdiv"]), float(z["len_disp"]), nthreads=2)
    for n in ("ru_p", "ruAvg", "rho_pp", "rtheta_pp", "rtheta_pp_old", "rw_p", "wwAvg"):
        ref = post["diag." + n]
        assert np.array_equal(out[n], ref), f"{n}: max diff {np.abs(out[n] - ref).max():.3e}"


def test_fixture_changes_state():
    """Guard against a degenerate fixture: the sub-step must move every updated field."""
    _, _, pre, post = _acoustic_fixture()
    for n in ("ru_p", "rho_pp", "rtheta_pp", "rw_p", "wwAvg"):
        assert np.abs(post["diag." + n] - pre["diag." + n]).max() > 0


def test_reference_reproduces_trajectory_fixture():
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    from mpas_dycore.cases import jw_case
    z = np.load(os.path.join(GOLD, "srk3_x1.642_K26_ns3.npz"))
    case = jw_case(642, K=26, ns=3, moist=True, cache=False)
    res, _ = ref_runner.run_reference(case, nsteps=10, dt=float(z["dt"]), dump_steps=[1, 10], nthreads=2)
    for s in (1, 10):
        for key in ("state.u.tl1", "state.theta_m.tl1", "state.rho_zz.tl1", "state.w.tl1", "state.scalars.tl1"):
            ref = z[f"step{s}_{key}"]
            got = res[s][key].reshape(ref.shape)
            assert rel_linf(got, ref) <= 1e-12, (s, key)


def test_physics_oracle_build():
    """The DO_PHYSICS reference build (prescribed tendencies through the physics_get_tend test
    double) with zero tendencies reproduces the plain build bit for bit; nonzero tendencies move
    u, theta_m, rho_zz and the scalars, and rqvdynten is (qv(n+1) - qv(n)) / dt before the clip."""
    from conftest import physics_forcing
    from oracle import ref_runner
    from mpas_dycore.cases import jw_case
    if not (ref_runner.available() and ref_runner.available(ref_runner.PHYS_HARNESS)):
        pytest.skip("oracle/_ref not built")
    case = jw_case(642, K=26, ns=3, moist=True, cache=False)
    dt = float(case["dt"])
    zero = {k: np.zeros_like(v) for k, v in physics_forcing(case).items()}
    a, _ = ref_runner.run_reference(case, 2, dt, [2], nthreads=2)
    b, _ = ref_runner.run_reference(case, 2, dt, [2], nthreads=2, physics=zero)
    keys = ("state.u.tl1", "state.theta_m.tl1", "state.rho_zz.tl1", "state.w.tl1", "state.scalars.tl1")
    for k in keys:
        assert np.array_equal(a[2][k], b[2][k]), k
    phys = dict(physics_forcing(case), convection_scheme="cu_tiedtke")
    c, _ = ref_runner.run_reference(case, 2, dt, [1, 2], nthreads=2, physics=phys)
    for k in keys[:3] + keys[4:]:
        assert not np.array_equal(a[2][k], c[2][k]), k
    assert c[2]["state.scalars.tl1"].min() >= 0.0
    # the monotone transport adds dt * scalars_tend / rho_zz to time level 1 in place (3748), so
    # rqvdynten differences against that updated level -- time level 2 of the dump after the shift
    q1, q2 = c[2]["state.scalars.tl2"][..., 0], c[2]["state.scalars.tl1"][..., 0]
    rqv = c[2]["tend_physics.rqvdynten"]
    pos = q2 > 0  # where the clip did not act, rqvdynten is the exact difference quotient
    assert (~pos).any() and pos.any()
    assert np.array_equal(rqv[pos], ((q2 - q1) / dt)[pos])
