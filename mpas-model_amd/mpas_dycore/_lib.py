"""ctypes binding of the C ABI in include/mpas_dycore.h (libmpas_dycore.so).

The product path has exactly one implementation: the HIP kernels in
mpas-model_amd/csrc.  If the shared library is missing this module raises --
there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

# int fn(const void* send, void* recv, int64_t nbytes, void* user) -- mpas_dyc_comm_init_host
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p)

HERE = os.path.dirname(os.path.abspath(__file__))
LIBPATH = os.environ.get("MPAS_DYCORE_LIB") or os.path.join(os.path.dirname(HERE), "csrc", "libmpas_dycore.so")

EXPORTS = (
    "mpas_dyc_create", "mpas_dyc_destroy", "mpas_dyc_last_error", "mpas_dyc_set_field", "mpas_dyc_get_field",
    "mpas_dyc_field_bytes", "mpas_dyc_field_device_ptr", "mpas_dyc_init_diagnostics", "mpas_dyc_timestep",
    "mpas_dyc_shift_time_levels", "mpas_dyc_synchronize", "mpas_dyc_time_acoustic_step", "mpas_dyc_use_graph",
    "mpas_dyc_acoustic_bytes", "mpas_dyc_create_blocks", "mpas_dyc_num_blocks", "mpas_dyc_set_block_field",
    "mpas_dyc_get_block_field", "mpas_dyc_block_field_bytes", "mpas_dyc_block_field_device_ptr",
    "mpas_dyc_set_exchange_list", "mpas_dyc_comm_unique_id_bytes", "mpas_dyc_comm_unique_id", "mpas_dyc_comm_init",
    "mpas_dyc_set_transport", "mpas_dyc_set_p2p", "mpas_dyc_get_p2p", "mpas_dyc_comm_init_host", "mpas_dyc_halo_exchange", "mpas_dyc_set_overlap", "mpas_dyc_output_diagnostics",
    "mpas_dyc_set_physics", "mpas_dyc_set_summary", "mpas_dyc_get_summary", "mpas_dyc_plan_exchanges",
    "mpas_dyc_graph_active", "mpas_dyc_solve_diagnostics", "mpas_dyc_set_lbc", "mpas_dyc_finish_step",
    "mpas_dyc_get_block_summary", "mpas_dyc_block_layout", "mpas_dyc_set_profile", "mpas_dyc_get_profile",
    "mpas_dyc_last_exchange", "mpas_dyc_rccl_version", "mpas_dyc_model_init", "mpas_dyc_set_exchange_positions",
    "mpas_dyc_init_deriv_two", "mpas_dyc_init_zb", "mpas_dyc_init_reconstruct",
)
HOST_ONLY = -2  # MPAS_DYC_HOST_ONLY: planner-only context
PRINT_GLOBAL_MINMAX_VEL, PRINT_DETAILED_MINMAX_VEL, PRINT_GLOBAL_MINMAX_SCA = 1, 2, 4
CELL, EDGE, VERTEX = 0, 1, 2
SEND, RECV = 0, 1


class Dims(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "nCells", "nEdges", "nVertices", "nVertLevels", "maxEdges", "maxEdges2", "num_scalars",
        "nCellsSolve", "nEdgesSolve", "nVerticesSolve", "moist_start", "moist_end", "index_qv")]


_CFG_INT = ("config_time_integration_order", "config_number_of_sub_steps", "config_dynamics_split_steps",
            "config_number_rayleigh_damp_u_levels", "config_split_dynamics_transport", "config_scalar_advection",
            "config_positive_definite", "config_monotonic", "config_mix_full", "config_rayleigh_damp_u",
            "config_horiz_mixing")
_CFG_DBL = ("config_h_mom_eddy_visc2", "config_h_mom_eddy_visc4", "config_v_mom_eddy_visc2",
            "config_h_theta_eddy_visc2", "config_h_theta_eddy_visc4", "config_v_theta_eddy_visc2",
            "config_len_disp", "config_visc4_2dsmag", "config_del4u_div_factor", "config_coef_3rd_order",
            "config_smagorinsky_coef", "config_epssm", "config_smdiv", "config_apvm_upwinding",
            "config_mpas_cam_coef", "config_rayleigh_damp_u_timescale_days")


class Config(C.Structure):
    _fields_ = [(n, C.c_int32) for n in _CFG_INT] + [(n, C.c_double) for n in _CFG_DBL]


class Extreme(C.Structure):
    _fields_ = [("value", C.c_double), ("lat", C.c_double), ("lon", C.c_double), ("k", C.c_int32),
                ("index", C.c_int32)]


class Summary(C.Structure):
    _fields_ = ([("flags", C.c_int32)] + [(n, C.c_double) for n in ("w_min", "w_max", "u_min", "u_max")]
                + [(n, Extreme) for n in ("w_min_at", "w_max_at", "u_min_at", "u_max_at", "wsp_max_at")]
                + [("nan_w", C.c_int64), ("nan_u", C.c_int64)])


class PlanMsg(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("point", "direction", "block", "peer_rank", "peer_block")] + [
        ("count", C.c_int64)]


def make_config(cfg: dict) -> Config:
    c = Config()
    for n in _CFG_INT:
        v = cfg[n]
        if n == "config_horiz_mixing":
            v = 1 if v == "2d_smagorinsky" else 0
        setattr(c, n, int(v))
    for n in _CFG_DBL:
        setattr(c, n, float(cfg[n]))
    return c


_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.isfile(LIBPATH):
        raise RuntimeError(f"MI355X dycore library not built: {LIBPATH} (run __graft_entry__.build())")
    lib = C.CDLL(LIBPATH)
    if os.environ.get("MPAS_DYCORE_LIB"):
        # an A/B build (tools/ab_*.sh) may predate the newest entry points: bind what it has
        class _Lenient:
            def __init__(self, real):
                object.__setattr__(self, "_real", real)

            def __getattr__(self, name):
                try:
                    return getattr(self._real, name)
                except AttributeError:
                    return type("Missing", (), {"argtypes": None, "restype": None})()
        _real, lib = lib, _Lenient(lib)
    vp, i32, i64, dbl = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    lib.mpas_dyc_create.argtypes = [C.POINTER(Dims), C.POINTER(Config), C.c_int, C.POINTER(vp)]
    lib.mpas_dyc_destroy.argtypes = [vp]
    lib.mpas_dyc_destroy.restype = None
    lib.mpas_dyc_last_error.argtypes = [vp]
    lib.mpas_dyc_last_error.restype = C.c_char_p
    lib.mpas_dyc_set_field.argtypes = [vp, C.c_char_p, C.c_char_p, i32, vp, i64]
    lib.mpas_dyc_get_field.argtypes = [vp, C.c_char_p, C.c_char_p, i32, vp, i64]
    lib.mpas_dyc_field_bytes.argtypes = [vp, C.c_char_p, C.c_char_p]
    lib.mpas_dyc_field_bytes.restype = i64
    lib.mpas_dyc_field_device_ptr.argtypes = [vp, C.c_char_p, C.c_char_p, i32]
    lib.mpas_dyc_field_device_ptr.restype = vp
    lib.mpas_dyc_init_diagnostics.argtypes = [vp, dbl]
    lib.mpas_dyc_solve_diagnostics.argtypes = [vp, dbl]
    lib.mpas_dyc_set_lbc.argtypes = [vp, i32, dbl]
    lib.mpas_dyc_timestep.argtypes = [vp, dbl, i32]
    lib.mpas_dyc_shift_time_levels.argtypes = [vp]
    lib.mpas_dyc_synchronize.argtypes = [vp]
    lib.mpas_dyc_output_diagnostics.argtypes = [vp, i32]
    lib.mpas_dyc_set_physics.argtypes = [vp, i32]
    lib.mpas_dyc_time_acoustic_step.argtypes = [vp, dbl, i32, i32, C.POINTER(dbl), C.POINTER(dbl)]
    lib.mpas_dyc_use_graph.argtypes = [vp, i32]
    lib.mpas_dyc_acoustic_bytes.argtypes = [vp]
    lib.mpas_dyc_acoustic_bytes.restype = dbl
    lib.mpas_dyc_create_blocks.argtypes = [i32, C.POINTER(Dims), C.POINTER(Config), C.c_int, C.POINTER(vp)]
    lib.mpas_dyc_num_blocks.argtypes = [vp]
    lib.mpas_dyc_num_blocks.restype = i32
    lib.mpas_dyc_set_block_field.argtypes = [vp, i32, C.c_char_p, C.c_char_p, i32, vp, i64]
    lib.mpas_dyc_get_block_field.argtypes = [vp, i32, C.c_char_p, C.c_char_p, i32, vp, i64]
    lib.mpas_dyc_block_field_bytes.argtypes = [vp, i32, C.c_char_p, C.c_char_p]
    lib.mpas_dyc_block_field_bytes.restype = i64
    lib.mpas_dyc_block_field_device_ptr.argtypes = [vp, i32, C.c_char_p, C.c_char_p, i32]
    lib.mpas_dyc_block_field_device_ptr.restype = vp
    lib.mpas_dyc_set_exchange_list.argtypes = [vp, i32, i32, i32, i32, i32, i32, vp, i32]
    lib.mpas_dyc_comm_unique_id_bytes.argtypes = []
    lib.mpas_dyc_comm_unique_id_bytes.restype = i64
    lib.mpas_dyc_comm_unique_id.argtypes = [vp, i64]
    lib.mpas_dyc_comm_init.argtypes = [vp, vp, i64, i32, i32]
    lib.mpas_dyc_set_transport.argtypes = [vp, i32]
    lib.mpas_dyc_set_p2p.argtypes = [vp, i32]
    lib.mpas_dyc_get_p2p.argtypes = [vp]
    lib.mpas_dyc_comm_init_host.argtypes = [vp, i32, i32, ALLGATHER_FN, vp]
    lib.mpas_dyc_halo_exchange.argtypes = [vp, C.c_char_p, C.c_char_p, i32, i32]
    lib.mpas_dyc_set_overlap.argtypes = [vp, i32]
    lib.mpas_dyc_set_summary.argtypes = [vp, i32]
    lib.mpas_dyc_get_summary.argtypes = [vp, C.POINTER(Summary), C.POINTER(dbl), i32]
    lib.mpas_dyc_get_block_summary.argtypes = [vp, i32, C.POINTER(Summary), C.POINTER(dbl), i32]
    lib.mpas_dyc_finish_step.argtypes = [vp, dbl]
    lib.mpas_dyc_plan_exchanges.argtypes = [vp, i32, i32, dbl, C.POINTER(PlanMsg), i64, C.POINTER(i64), C.c_char_p,
                                            i64, C.POINTER(i64)]
    lib.mpas_dyc_graph_active.argtypes = [vp]
    lib.mpas_dyc_block_layout.argtypes = [vp, i32, C.POINTER(i32)]
    lib.mpas_dyc_set_profile.argtypes = [vp, i32]
    lib.mpas_dyc_get_profile.argtypes = [vp, C.POINTER(dbl), i32]
    lib.mpas_dyc_last_exchange.argtypes = [vp]
    lib.mpas_dyc_last_exchange.restype = C.c_char_p
    lib.mpas_dyc_rccl_version.argtypes = []
    lib.mpas_dyc_rccl_version.restype = i32
    lib.mpas_dyc_model_init.argtypes = [vp, i32, dbl, dbl]
    lib.mpas_dyc_init_deriv_two.argtypes = [vp, i32, vp, vp, vp, vp]
    lib.mpas_dyc_init_zb.argtypes = [vp, i32, i32]
    lib.mpas_dyc_init_reconstruct.argtypes = [vp]
    lib.mpas_dyc_set_exchange_positions.argtypes = [vp, i32, i32, i32, i32, i32, vp, vp, i32]
    if os.environ.get("MPAS_DYCORE_LIB"):
        lib = _real
    _lib = lib
    return lib
