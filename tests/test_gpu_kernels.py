"""Per-kernel GPU parity: the HIP acoustic sub-step (k_acoustic_edges + k_acoustic_cells + k_divdamp,
through the C ABI) on the committed reference fixture.  Every input the kernels read is uploaded
from the fixture, so the comparison is independent of the host that built it."""
import os

import numpy as np
import pytest

from conftest import rel_linf

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _pad(a):
    a = np.asarray(a, dtype=np.float64)
    return np.ascontiguousarray(np.concatenate([a, np.zeros((1,) + a.shape[1:])], 0))


def _fixture_dycore():
    from mpas_dycore import Dycore
    from mpas_dycore.cases import jw_case
    z = np.load(os.path.join(GOLD, "acoustic_x1.162_K16.npz"))
    case = jw_case(162, K=16, ns=1, cache=False)
    for k in z.files:
        if k.startswith("mesh_"):
            case[k[5:]] = z[k]
    dy = Dycore(case, device=0)
    for k in z.files:
        if not k.startswith("pre_"):
            continue
        key = k[4:]
        parts = key.split(".")
        pool, name = parts[0], parts[1]
        tl = int(parts[2][2:]) if len(parts) > 2 else 1
        a = z[k]
        img = np.ascontiguousarray(a, dtype=np.float64) if name == "cofrz" else _pad(a)
        dy.set_raw(pool, name, img, tl)
    return z, dy


POST = ("ru_p", "ruAvg", "rho_pp", "rtheta_pp", "rtheta_pp_old", "rw_p", "wwAvg")


def test_acoustic_substep_matches_reference_fixture():
    z, dy = _fixture_dycore()
    dy.time_acoustic_step(float(z["dts"]), small_step=int(z["small_step"]), reps=1)
    dy.synchronize()
    for n in POST:
        got = dy.get("diag", n)
        ref = z["post_diag." + n]
        err = rel_linf(got.reshape(ref.shape), ref)
        assert err <= 1e-14, f"{n}: rel Linf {err:.3e}"
    dy.close()


def test_fused_substep_loop_equals_substeps_with_damping():
    """A 3-sub-step loop (each damping fused into the next sub-step's edge phase) gives the same
    bits as three single sub-steps each followed by its own damping kernel (the reference order)."""
    z, a = _fixture_dycore()
    for _ in range(3):
        a.time_acoustic_step(float(z["dts"]), small_step=int(z["small_step"]), reps=1)
    a.synchronize()
    want = {n: a.get("diag", n) for n in POST}
    a.close()
    z, b = _fixture_dycore()
    b.time_acoustic_step(float(z["dts"]), small_step=int(z["small_step"]), reps=3)
    b.synchronize()
    for n in POST:
        assert np.array_equal(b.get("diag", n), want[n]), n
    b.close()


def test_acoustic_substep_bitwise_vs_reference_fixture():
    """The acoustic sub-step is +,-,*,/ only (no pow / transcendental), evaluated in the reference's
    operation order with FMA contraction off, so it reproduces the reference's doubles exactly --
    including the tridiagonal sweeps, which run as DPP wavefront-shift iterations."""
    z, dy = _fixture_dycore()
    dy.time_acoustic_step(float(z["dts"]), small_step=int(z["small_step"]), reps=1)
    dy.synchronize()
    for n in POST:
        got = dy.get("diag", n).reshape(z["post_diag." + n].shape)
        ref = z["post_diag." + n]
        nd = int(np.count_nonzero(got != ref))
        assert nd == 0, f"{n}: {nd} values differ, max abs {np.max(np.abs(got - ref)):.3e}"
    dy.close()


def _steps_with_kernels(case, family, nsteps=3, dt=None):
    from mpas_dycore import Dycore
    saved = {k: os.environ.get(k) for k in ("MPAS_DYCORE_KERNELS",)}
    os.environ["MPAS_DYCORE_KERNELS"] = family
    try:
        dy = Dycore(case, device=0, moist_end=case["num_scalars"])
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    dt = dt or 2880.0
    dy.init_diagnostics(dt)
    for i in range(nsteps):
        dy.atm_timestep(dt, i + 1)
        dy.shift_time_levels()
    dy.synchronize()
    out = {n: dy.get("state", n, 1) for n in ("u", "w", "theta_m", "rho_zz", "scalars")}
    out.update({n: dy.get("diag", n) for n in ("pv_edge", "rho_edge", "exner", "ru", "rw", "uReconstructX",
                                                "uReconstructY", "uReconstructZ", "uReconstructZonal",
                                                "uReconstructMeridional")})
    dy.close()
    return out


@pytest.mark.parametrize("which", ["moist_case", "varres_case_small"])
def test_kernel_families_give_identical_bits(which, request):
    """The general (one column per wave), batched (per-cell records, loads up front) and pair
    (two edges per wave, 16-byte loads) kernel families evaluate the same expressions in the same
    order, so three moist monotone steps agree to the bit -- on the icosahedral mesh and on the
    variable-resolution mesh with heptagons (maxEdges = 7)."""
    case = request.getfixturevalue(which)
    dt = float(case["dt"]) if which == "varres_case_small" else 2880.0
    ref = _steps_with_kernels(case, "general", dt=dt)
    for fam in ("batched", "pair"):
        got = _steps_with_kernels(case, fam, dt=dt)
        for n in ref:
            assert np.array_equal(got[n], ref[n]), f"{fam}: {n}"


def test_odd_level_count_pair_layout_matches_general():
    """K = 25 (odd): the pair layout's last pair holds level K-1 and a level past the column that is
    loaded and never stored; the pair family matches the general one (one column per wave)."""
    from mpas_dycore.cases import jw_case
    case = jw_case(642, K=25, ns=2, moist=True, cache=False)
    ref = _steps_with_kernels(case, "general", nsteps=2)
    got = _steps_with_kernels(case, "pair", nsteps=2)
    for n in ref:
        assert np.array_equal(got[n], ref[n]), n


def _steps_env(case, env, nsteps=3, dt=None, blocks=0):
    """nsteps moist monotone steps with the environment variables env set while the context is
    created (the library reads its switches then); blocks > 0: that many MPAS blocks on the device,
    exchanging through RCCL."""
    from mpas_dycore import Dycore, decomp
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        if blocks:
            bl = decomp.decompose(case, decomp.partition_sfc(case["nCells"], blocks))
            dy = Dycore.from_blocks(bl, device=0, comm_id=Dycore.comm_unique_id(), nranks=1, rank=0,
                                    rccl_local=True, moist_end=case["num_scalars"])
        else:
            dy = Dycore(case, device=0, moist_end=case["num_scalars"])
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    dt = dt or 2880.0
    dy.init_diagnostics(dt)
    dy.use_graph(True)
    for i in range(nsteps):
        dy.atm_timestep(dt, i + 1)
        dy.shift_time_levels()
    dy.synchronize()
    if blocks:
        n_glob = {"cell": case["nCells"], "edge": case["nEdges"]}
        out = {n: decomp.gather_owned(bl, [dy.get("state", n, 1, block=i) for i in range(len(bl))],
                                      "edge" if n == "u" else "cell", n_glob["edge" if n == "u" else "cell"])
               for n in ("u", "w", "theta_m", "rho_zz", "scalars")}
    else:
        out = {n: dy.get("state", n, 1) for n in ("u", "w", "theta_m", "rho_zz", "scalars")}
    dy.close()
    return out


@pytest.mark.parametrize("ns,blocks", [(3, 0), (6, 0), (5, 4)])
def test_mono_scalar_pairs_bitwise(ns, blocks):
    """The monotone transport's per-scalar pipeline (3798-4210) runs two scalars side by side with
    two sets of scratch and one scale_arr exchange per pair (dycore.hip, advance_scalars_mono):
    equal bit for bit to one scalar at a time (MPAS_DYCORE_MONO_PAIRS=0), odd and even scalar
    counts, and on 4 RCCL blocks."""
    from mpas_dycore.cases import jw_case
    case = jw_case(642, K=26, ns=ns, moist=True, cache=False)
    ref = _steps_env(case, {"MPAS_DYCORE_MONO_PAIRS": "0"}, blocks=blocks)
    got = _steps_env(case, {"MPAS_DYCORE_MONO_PAIRS": "1"}, blocks=blocks)
    for n in ref:
        assert np.array_equal(got[n], ref[n]), n
