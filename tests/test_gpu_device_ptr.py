"""GPU: the zero-copy device pointers (mpas_dyc_field_device_ptr, include/mpas_dycore.h) across steps.

The step rotates buffers instead of copying them (the _save copies of atm_rk_integration_setup and
atm_rk_dynamics_substep_finish, mpas_atm_time_integration.F:1847-1850, 6051-6054; theta_m_1 =
theta_m_2 at 6058; the time levels at mpas_pool_shift_time_levels), so the header documents a pointer
as valid until the next step.  Checked here: a pointer queried after each step holds exactly the
field's image (what mpas_dyc_get_field returns), for the rotated fields and fixed ones, and the
fixed ones never move.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROTATED = [("diag", "ru", 1), ("diag", "ru_save", 1), ("diag", "rw", 1), ("diag", "rw_save", 1),
           ("diag", "rtheta_p", 1), ("diag", "rtheta_p_save", 1), ("diag", "rho_p", 1), ("diag", "rho_p_save", 1),
           ("state", "theta_m", 1), ("state", "theta_m", 2), ("state", "u", 1), ("state", "rho_zz", 1)]
FIXED = [("diag", "pressure_p", 1), ("diag", "exner", 1), ("diag", "pv_edge", 1)]


def _hip():
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipMemcpy.restype = C.c_int
    return hip


def _read(hip, ptr, nbytes):
    buf = np.empty(nbytes // 8, dtype=np.float64)
    assert hip.hipMemcpy(buf.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), nbytes, 2) == 0  # DeviceToHost
    return buf


def test_pointers_requeried_after_each_step_hold_the_field(moist_case):
    from mpas_dycore import Dycore
    hip = _hip()
    dy = Dycore(moist_case, device=0, moist_end=3)
    dt = 2880.0
    dy.init_diagnostics(dt)
    dy.use_graph(True)
    seen = {}
    for it in range(3):
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
        dy.synchronize()
        for pool, name, tl in ROTATED + FIXED:
            ptr = dy.lib.mpas_dyc_field_device_ptr(dy.h, pool.encode(), name.encode(), tl)
            assert ptr, f"{pool}.{name}"
            nb = dy.lib.mpas_dyc_field_bytes(dy.h, pool.encode(), name.encode())
            want = dy.get_raw(pool, name, tl)
            assert np.array_equal(_read(hip, ptr, nb), want), f"step {it + 1}: {pool}.{name} tl{tl}"
            seen.setdefault((pool, name, tl), set()).add(ptr)
    for key in FIXED:
        assert len(seen[key]) == 1, f"{key} moved"
    moved = [k for k in ROTATED if len(seen[k]) > 1]
    print("pointers that moved over 3 steps:", moved)
    dy.close()


def test_writes_through_packed_mesh_pointers_reach_the_kernels(moist_case):
    """The maxEdges-strided mesh fields and zb_cell / zb3_cell are read by the kernels from packed copies
    (pack_mesh, zb_p / zb_m).  A write through their device pointers must reach the next step as a
    mpas_dyc_set_field of the same image does: the library packs again after handing out such a pointer."""
    from mpas_dycore import Dycore
    hip = _hip()
    dt = 2880.0
    scale = {"zb3_cell": 0.5, "defc_a": 1.001}
    runs = {}
    for mode in ("none", "set", "ptr"):
        dy = Dycore(moist_case, device=0, moist_end=3)
        dy.init_diagnostics(dt)
        dy.use_graph(True)
        dy.atm_timestep(dt, 1)
        dy.shift_time_levels()
        dy.synchronize()
        for n, f in scale.items():
            img = dy.get_raw("mesh", n) * f
            if mode == "ptr":
                ptr = dy.lib.mpas_dyc_field_device_ptr(dy.h, b"mesh", n.encode(), 1)
                assert hip.hipMemcpy(C.c_void_p(ptr), img.ctypes.data_as(C.c_void_p), img.nbytes, 1) == 0
            elif mode == "set":
                dy.set_raw("mesh", n, img)
        for it in range(2):
            dy.atm_timestep(dt, it + 2)
            dy.shift_time_levels()
        dy.synchronize()
        runs[mode] = {n: dy.get("state", n, 1) for n in ("u", "w", "theta_m")}
        dy.close()
    assert not np.array_equal(runs["none"]["w"], runs["set"]["w"]), "the changed fields did not change the run"
    for n in runs["set"]:
        assert np.array_equal(runs["set"][n], runs["ptr"][n]), f"{n}: the write through the pointer did not reach the kernels"
